// FP64 issue study (not part of the product): does a wave64 FP64 FMA (v_fma_f64) issue in 4 or 8
// cycles on gfx950, and do FP64 MFMAs (v_mfma_f64_4x4x4_4b, v_mfma_f64_16x16x4) execute beside
// FP64 VALU work of other waves on the same SIMD?  Every SIMD runs W waves of one of the modes
// (0: FMAs only, 1: 4x4x4 MFMAs only, 2: both interleaved in each wave, 3: half the waves FMAs,
// half MFMAs, 4: 16x16x4 MFMAs only, 5: 16x16x4 + FMA waves); 8 independent chains per wave,
// cycles per loop iteration from s_memtime, the clock from s_memrealtime.
// Build: hipcc -O3 --offload-arch=gfx950 fp64_coissue.hip -o fp64_coissue
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void __launch_bounds__(256) run(double *out, unsigned long long *clk, int iters) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    double v[8], s = 1.0000001 + lane * 1e-9, t = 1e-12;
    double a = 0.5 + lane * 1e-3, b = 0.25 - lane * 1e-3;
    double m[8];
    d4 m16[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = i + lane, m[i] = i * 0.5;
#pragma unroll
    for (int i = 0; i < 4; ++i) m16[i] = d4{0, 0, 0, 0};
    const bool fma_wave = MODE == 0 || MODE == 2 || ((MODE == 3 || MODE == 5) && (w & 1) == 0);
    const bool mfma_wave = MODE == 1 || MODE == 2 || (MODE == 3 && (w & 1) == 1);
    const bool m16_wave = MODE == 4 || (MODE == 5 && (w & 1) == 1);
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if (fma_wave) {
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = __builtin_fma(v[i], s, t);
        }
        if (mfma_wave) {
#pragma unroll
            for (int i = 0; i < 8; ++i) m[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, m[i], 0, 0, 0);
        }
        if (m16_wave) {
#pragma unroll
            for (int i = 0; i < 4; ++i) m16[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, m16[i], 0, 0, 0);
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    double acc = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc += v[i] + m[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) acc += m16[i][0] + m16[i][1] + m16[i][2] + m16[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = acc;
    if (lane == 0) {
        clk[(blockIdx.x * 4 + w) * 2] = c1 - c0;
        clk[(blockIdx.x * 4 + w) * 2 + 1] = r1 - r0;
    }
}

template <int MODE> void go(int blocks, int iters, double *out, unsigned long long *clk, const char *name) {
    hipLaunchKernelGGL(run<MODE>, dim3(blocks), dim3(256), 0, 0, out, clk, iters);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(run<MODE>, dim3(blocks), dim3(256), 0, 0, out, clk, iters);
    hipDeviceSynchronize();
    const int nw = blocks * 4;
    unsigned long long *h = (unsigned long long *)malloc(sizeof(unsigned long long) * 2 * nw);
    hipMemcpy(h, clk, sizeof(unsigned long long) * 2 * nw, hipMemcpyDeviceToHost);
    double cyc = 0, rt = 0;
    for (int i = 0; i < nw; ++i) cyc += h[2 * i], rt += h[2 * i + 1];
    cyc /= nw, rt /= nw;
    // waves per SIMD: blocks * 4 waves over 256 CUs x 4 SIMDs
    const double wps = (double)nw / 1024.0;
    printf("{\"mode\": \"%s\", \"waves_per_simd\": %.1f, \"cycles_per_iter_per_wave\": %.1f, "
           "\"simd_cycles_per_iter\": %.1f, \"clock_GHz\": %.3f}\n",
           name, wps, cyc / iters, cyc / iters / wps, cyc / (rt / 100e6) / 1e9);
    free(h);
}

int main(int argc, char **argv) {
    const int iters = 4096;
    double *out;
    unsigned long long *clk;
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int blocks = 256 * wps; // 4 waves per block, 1024 SIMDs
        hipMalloc(&out, sizeof(double) * blocks * 256);
        hipMalloc(&clk, sizeof(unsigned long long) * blocks * 8);
        go<0>(blocks, iters, out, clk, "fma x8");
        go<1>(blocks, iters, out, clk, "mfma4x4x4 x8");
        go<2>(blocks, iters, out, clk, "fma x8 + mfma4x4x4 x8 (same wave)");
        go<3>(blocks, iters, out, clk, "fma waves | mfma4x4x4 waves");
        go<4>(blocks, iters, out, clk, "mfma16x16x4 x4");
        go<5>(blocks, iters, out, clk, "fma waves | mfma16x16x4 waves");
        hipFree(out);
        hipFree(clk);
    }
    return 0;
}
