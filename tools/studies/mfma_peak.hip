// Microbenchmark (not part of the product): sustained v_mfma_f64_16x16x4_f64 rate on every
// SIMD of the chip, operands in registers, random data; also the in-kernel clock
// (s_memtime / s_memrealtime at 100 MHz).  Gives the measured FP64 MFMA ceiling the GEMM is
// judged against.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void __launch_bounds__(256) mfma_loop(double *out, int iters, unsigned long long *clk) {
    const int lane = threadIdx.x & 63;
    double a = 0.5 + lane * 1e-3, b = 0.25 - lane * 1e-3;
    d4 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = d4{(double)i, 1.0, 2.0, 3.0};
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    double s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

__global__ void __launch_bounds__(256) fma_loop(double *out, int iters) {
    double a[8], x = 1.0 + threadIdx.x * 1e-6, y = 0.999999;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = i;
    for (int it = 0; it < iters; ++it)
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = __builtin_fma(a[i], y, x);
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    double *out;
    unsigned long long *clk;
    (void)hipMalloc(&out, sizeof(double) * 256 * 4096);
    (void)hipMalloc(&clk, 16);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 20000;
    for (int blocks_per_cu : {1, 2, 4}) {
        const int blocks = 256 * blocks_per_cu;
        mfma_loop<8><<<blocks, 256>>>(out, iters / 10, clk);
        (void)hipEventRecord(e0);
        mfma_loop<8><<<blocks, 256>>>(out, iters, clk);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        unsigned long long c[2];
        (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
        const double flops = 2.0 * 16 * 16 * 4 * 8.0 * iters * (blocks * 4.0);
        std::printf("mfma f64 16x16x4: %d WG(256 thr)/CU  %.3f ms  %.2f TFLOP/s  clock %.3f GHz  "
                    "cycles/mfma %.1f\n",
                    blocks_per_cu, ms, flops / ms / 1e9, c[0] / (c[1] / 100e6) / 1e9,
                    (double)c[0] / (8.0 * iters));
    }
    for (int blocks_per_cu : {2, 8}) {
        const int blocks = 256 * blocks_per_cu;
        fma_loop<<<blocks, 256>>>(out, iters / 10);
        (void)hipEventRecord(e0);
        fma_loop<<<blocks, 256>>>(out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double flops = 2.0 * 8 * iters * (blocks * 256.0);
        std::printf("v_fma_f64: %d WG/CU  %.3f ms  %.2f TFLOP/s\n", blocks_per_cu, ms,
                    flops / ms / 1e9);
    }
    return 0;
}
