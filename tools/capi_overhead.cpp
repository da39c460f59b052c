// Host cost per C-ABI call (planner + launch) on tiny tensors; not part of the product.
#include "../include/superbblas_amd/sbx.h"
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    double *a, *b;
    (void)hipMalloc(&a, 16 * 16);
    (void)hipMalloc(&b, 16 * 16);
    int p[4] = {0, 0, 4, 4}, from[2] = {0, 0}, dim[2] = {4, 4};
    sbx_context ctx{SBX_GPU, 0};
    const void *v0[1] = {a};
    void *v1[1] = {b};
    double alpha[2] = {1, 0};
    const int n = 20000;
    for (int rep = 0; rep < 2; ++rep) {
        double t = now();
        for (int i = 0; i < n; ++i)
            if (sbx_copy(2, 2, alpha, SBX_CDOUBLE, SBX_CDOUBLE, p, 1, "xy", from, dim, dim, v0, &ctx,
                         p, 1, "yx", from, dim, v1, &ctx, nullptr, SBX_SLOW_TO_FAST, SBX_COPY, 0)) {
                std::printf("error %s\n", sbx_last_error());
                return 1;
            }
        t = now() - t;
        std::printf("sbx_copy: %.2f us/call\n", t / n * 1e6);
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
