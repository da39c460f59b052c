// Host cost per C-ABI call (planner + launch) versus a bare kernel launch; not part of the
// product.  Build: hipcc --offload-arch=gfx950 -O2 tools/capi_overhead.cpp -Iinclude
//                  -Lsuperbblas_amd -lsuperbblas_amd -o tools/capi_overhead
#include "../include/superbblas_amd/sbx.h"
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void empty_kernel(double *p) {
    if (threadIdx.x == 1000000) p[0] = 1;
}

// The reference's dist.cpp permute loop (tests/dist.cpp:237-266) called eagerly from C++: copy
// an xyztsc field into each of the n slices of tnsxyzc, one sbx_copy per slice, timed with HIP
// events on the library stream; and the reference's "dummy copying" loop it is compared with
// (tests/dist.cpp:205-235: the same field copied contiguously into n slices, one device memcpy
// each) -- its "overhead" = permute time / memcpy time.  `cf` = the reference's own element type
// (complex<float>, dist.cpp:200), `cd` = complex<double> (configs[1]).  Prints one JSON line.
static int permute(int L, int n4, int reps, bool cf) {
    const long vol0 = (long)L * L * L * L * 4 * 3, vol1 = vol0 * n4;
    const int es = cf ? 8 : 16, t = cf ? SBX_CFLOAT : SBX_CDOUBLE;
    void *a, *b;
    if (hipMalloc(&a, es * vol0) != hipSuccess || hipMalloc(&b, es * vol1) != hipSuccess) return 1;
    (void)hipMemset(a, 0, es * vol0);
    int p0[12] = {0, 0, 0, 0, 0, 0, L, L, L, L, 4, 3};
    int d0[6] = {L, L, L, L, 4, 3}, f0[6] = {0, 0, 0, 0, 0, 0};
    int p1[14] = {0, 0, 0, 0, 0, 0, 0, L, n4, 4, L, L, L, 3};
    int d1[7] = {L, n4, 4, L, L, L, 3};
    sbx_context ctx{SBX_GPU, 0};
    const void *v0[1] = {a};
    void *v1[1] = {b};
    double alpha[2] = {1, 0};
    hipStream_t s;
    (void)sbx_stream_get(0, (void **)&s);
    auto loop = [&]() {
        for (int k = 0; k < n4; ++k) {
            int f1[7] = {0, k, 0, 0, 0, 0, 0};
            if (sbx_copy(6, 7, alpha, t, t, p0, 1, "xyztsc", f0, d0, d0, v0, &ctx, p1, 1,
                         "tnsxyzc", f1, d1, v1, &ctx, nullptr, SBX_SLOW_TO_FAST, SBX_COPY, 0))
                return false;
        }
        return true;
    };
    auto memcpy_loop = [&]() {
        for (int k = 0; k < n4; ++k)
            (void)hipMemcpyAsync((char *)b + (long)es * vol0 * k, a, es * vol0,
                                 hipMemcpyDeviceToDevice, s);
    };
    if (!loop()) {
        std::printf("{\"error\": \"%s\"}\n", sbx_last_error());
        return 1;
    }
    (void)hipStreamSynchronize(s);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double t0 = now();
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < reps; ++r) loop();
    (void)hipEventRecord(e1, s);
    const double host = (now() - t0) / reps / n4;
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double tp = ms / 1e3 / reps;
    memcpy_loop();
    (void)hipStreamSynchronize(s);
    (void)hipEventRecord(e0, s);
    for (int r = 0; r < reps; ++r) memcpy_loop();
    (void)hipEventRecord(e1, s);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double tm = ms / 1e3 / reps;
    std::printf("{\"op\": \"permute_eager\", \"type\": \"%s\", \"L\": %d, \"n\": %d, "
                "\"ms\": %.4f, \"GBps\": %.1f, \"host_us_per_copy\": %.3f, \"memcpy_ms\": %.4f, "
                "\"memcpy_GBps\": %.1f, \"overhead_vs_memcpy\": %.3f}\n",
                cf ? "cf" : "cd", L, n4, tp * 1e3, 2.0 * es * vol1 / tp / 1e9, host * 1e6, tm * 1e3,
                2.0 * es * vol1 / tm / 1e9, tp / tm);
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}

int main(int argc, char **argv) {
    if (argc >= 2 && std::string(argv[1]) == "permute")
        return permute(argc > 2 ? std::atoi(argv[2]) : 16, argc > 3 ? std::atoi(argv[3]) : 64,
                       argc > 4 ? std::atoi(argv[4]) : 5, argc > 5 && std::string(argv[5]) == "cf");
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
