// The FP32 MFMA instruction stream of the chain's y^H y GEMM (gemm_wave_kernel: a 48x48
// complex<float> tile per wave = 9 16x16 tiles, the 4-multiplication complex form, 36
// v_mfma_f32_16x16x4_f32 per k-step) with its operands held in registers: no LDS, no DMA, no
// barrier.  What the matrix pipe delivers for exactly this mix, at 1-4 waves per SIMD, with and
// without the sign flips between the MFMAs.  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/mfma_f32_mix.hip -o tools/mfma_f32_mix
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float acc_t __attribute__((ext_vector_type(4)));

template <bool FLIP>
__global__ void __launch_bounds__(256) mix_kernel(float *out, int iters, unsigned mask) {
    const int lane = threadIdx.x & 63;
    float ax[3], ay[3];
    for (int i = 0; i < 3; ++i) {
        ax[i] = 1.0f + 1e-3f * (lane + i);
        ay[i] = 1.0f - 1e-3f * (lane + 2 * i);
    }
    acc_t accR[3][3], accI[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            accR[i][j] = acc_t{0, 0, 0, 0};
            accI[i][j] = acc_t{0, 0, 0, 0};
        }
    for (int it = 0; it < iters; ++it) {
        float a_y[3], b_y[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            if (FLIP) {
                a_y[i] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, ay[i]) ^ mask);
                b_y[i] = __builtin_bit_cast(float, __builtin_bit_cast(unsigned, ay[i]) ^ (mask >> 1));
            } else {
                a_y[i] = ay[i];
                b_y[i] = ay[i];
            }
        }
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                accR[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ax[i], ax[j], accR[i][j], 0, 0, 0);
                accI[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(ax[i], b_y[j], accI[i][j], 0, 0, 0);
            }
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                accR[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(-a_y[i], b_y[j], accR[i][j], 0, 0, 0);
                accI[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a_y[i], ax[j], accI[i][j], 0, 0, 0);
            }
    }
    float s = 0;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j)
            for (int r = 0; r < 4; ++r) s += accR[i][j][r] + accI[i][j][r];
    if (s == 12345.0f) out[threadIdx.x] = s; // keep the work
}

int main() {
    float *out;
    (void)hipMalloc(&out, 1024 * sizeof(float));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 2000;
    for (int flip = 0; flip < 2; ++flip)
        for (int wps = 1; wps <= 4; ++wps) { // waves per SIMD: 4 waves per workgroup, wps per CU
            const int blocks = 256 * wps;
            auto run = [&]() {
                if (flip)
                    hipLaunchKernelGGL(mix_kernel<true>, dim3(blocks), dim3(256), 0, 0, out, iters, 0x80000000u);
                else
                    hipLaunchKernelGGL(mix_kernel<false>, dim3(blocks), dim3(256), 0, 0, out, iters, 0u);
            };
            run();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0, 0);
            for (int r = 0; r < 5; ++r) run();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double flops = 5.0 * blocks * 4 * (double)iters * 36 * 2048;
            std::printf("{\"flip\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f}\n", flip,
                        wps, ms, flops / (ms / 1e3) / 1e12);
        }
    return 0;
}
