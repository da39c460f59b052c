// Host cost per C-ABI call (planner + launch) versus a bare kernel launch; not part of the
// product.  Build: hipcc --offload-arch=gfx950 -O2 tools/capi_overhead.cpp -Iinclude
//                  -Lsuperbblas_amd -lsuperbblas_amd -o tools/capi_overhead
#include "../include/superbblas_amd/sbx.h"
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void empty_kernel(double *p) {
    if (threadIdx.x == 1000000) p[0] = 1;
}

int main() {
    double *a, *b;
    const int L = 4, n4 = 8;
    const long vol0 = (long)L * L * L * L * 4 * 3, vol1 = vol0 * n4;
    (void)hipMalloc(&a, 16 * vol0);
    (void)hipMalloc(&b, 16 * vol1);
    int p0[12] = {0, 0, 0, 0, 0, 0, L, L, L, L, 4, 3};
    int d0[6] = {L, L, L, L, 4, 3}, f0[6] = {0, 0, 0, 0, 0, 0};
    int p1[14] = {0, 0, 0, 0, 0, 0, 0, L, n4, 4, L, L, L, 3};
    int d1[7] = {L, n4, 4, L, L, L, 3}, f1[7] = {0, 1, 0, 0, 0, 0, 0};
    sbx_context ctx{SBX_GPU, 0};
    const void *v0[1] = {a};
    void *v1[1] = {b};
    double alpha[2] = {1, 0};
    const int n = 20000;
    hipStream_t s;
    (void)sbx_stream_get(0, (void **)&s);
    for (int rep = 0; rep < 2; ++rep) {
        double t = now();
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, a);
        t = now() - t;
        std::printf("bare hipLaunchKernelGGL: %.2f us/call\n", t / n * 1e6);
        (void)hipDeviceSynchronize();
        t = now();
        for (int i = 0; i < n; ++i)
            if (sbx_copy(6, 7, alpha, SBX_CDOUBLE, SBX_CDOUBLE, p0, 1, "xyztsc", f0, d0, d0, v0,
                         &ctx, p1, 1, "tnsxyzc", f1, d1, v1, &ctx, nullptr, SBX_SLOW_TO_FAST,
                         SBX_COPY, 0)) {
                std::printf("error %s\n", sbx_last_error());
                return 1;
            }
        t = now() - t;
        std::printf("sbx_copy (permute into a slice): %.2f us/call\n", t / n * 1e6);
        (void)hipDeviceSynchronize();
        t = now();
        for (int i = 0; i < n; ++i)
            sbx_xgemm_batch_strided(SBX_CDOUBLE, 'N', 'N', 4, 4, 4, alpha, a, 4, 0, b, 4, 0, alpha,
                                    b, 4, 0, 1, 0);
        t = now() - t;
        std::printf("sbx_xgemm_batch_strided: %.2f us/call\n", t / n * 1e6);
        (void)hipDeviceSynchronize();
    }
    return 0;
}
