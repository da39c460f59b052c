// The FP32 MFMA instruction stream of the chain's y^H y GEMM (gemm_wave_kernel: a 48x48
// complex<float> tile per wave = 9 16x16 tiles, the 4-multiplication complex form, 36
// v_mfma_f32_16x16x4_f32 per k-step) with its operands held in registers: no LDS, no DMA, no
// barrier.  What the matrix pipe delivers for exactly this mix, at 1-4 waves per SIMD, with and
// without the sign flips between the MFMAs.  Not part of the product.
// Build: hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/studies/mfma_f32_mix.hip -o tools/studies/mfma_f32_mix
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float acc_t __attribute__((ext_vector_type(4)));

// MODE 0: fragments in registers; 1: fragments read from a wave-private LDS image each k-step
// (the kernel's M-major [k][48] float2 image, 2 k-steps per 8-deep slab, 2 slots);
// 2: as 1, plus the slab's 3 LDS-DMA instructions from a global buffer (L2-resident when small,
// `span` bytes per wave) and a vmcnt wait one slab later, as gemm_wave_kernel does
template <bool FLIP, int MODE>
__global__ void __launch_bounds__(256) mix_kernel(float *out, int iters, unsigned mask,
                                                  const char *src, unsigned span) {
    __shared__ __attribute__((aligned(16))) float2 lds[4][2][8 * 48];
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float ax[3], ay[3];
    for (int i = 0; i < 3; ++i) {
        ax[i] = 1.0f + 1e-3f * (lane + i);
        ay[i] = 1.0f - 1e-3f * (lane + 2 * i);
    }
    if (MODE > 0) {
        for (int e = lane; e < 2 * 8 * 48; e += 64)
            lds[wave][e / 384][e % 384] = float2{1.0f + 1e-4f * e, 1.0f - 1e-4f * e};
        __syncthreads();
    }
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void *)src, (short)0, (int)(span * gridDim.x * 4u), 0x00020000);
    const unsigned wbase = (blockIdx.x * 4u + wave) * span;
    acc_t accR[3][3], accI[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            accR[i][j] = acc_t{0, 0, 0, 0};
            accI[i][j] = acc_t{0, 0, 0, 0};
        }
    for (int it = 0; it < iters; ++it) {
        if (MODE >= 1) {
            const int slot = (it >> 1) & 1, kk = (it & 1) * 4;
            if (MODE == 2 && (it & 1) == 0) {
                // issue the next slab's 3 DMA instructions into the other slot, wait for this one
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const unsigned off = wbase + (unsigned)(((it >> 1) * 3072u) % span);
                const unsigned dst = (unsigned)(size_t)(const __attribute__((address_space(3))) void *)&lds[wave][slot ^ 1][0];
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const unsigned o = off + (unsigned)(q * 1024 + lane * 16);
                    asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
                                 : : "v"(o), "s"(__builtin_amdgcn_readfirstlane(dst + q * 1024u)), "s"(rs) : "memory", "m0");
                }
                asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
            }
            const float2 *img = &lds[wave][slot][0];
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const float2 v = img[(kk + (lane >> 4)) * 48 + (lane & 15) + 16 * i];
                ax[i] = v.x;
                ay[i] = v.y;
            }
        }
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
    char *src;
    const size_t big = 1024ull << 20; // 1 GiB (HBM) or a 3 KB-per-wave slab set (L2)
    (void)hipMalloc(&src, big);
    (void)hipMemset(src, 0, big);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 2000;
    struct Cfg { int mode; bool flip; unsigned span; const char *what; };
    const Cfg cfgs[] = {{0, true, 3072, "registers"}, {1, true, 3072, "LDS fragments"},
                        {2, true, 3072, "LDS + DMA, L2-resident"},
                        {2, true, 0, "LDS + DMA, HBM stream"}};
    for (const Cfg &c : cfgs)
        for (int wps = 1; wps <= 4; ++wps) { // waves per SIMD: 4 waves per workgroup, wps per CU
            const int blocks = 256 * wps;
            const unsigned span = c.span ? c.span : (unsigned)(big / (blocks * 4) / 3072 * 3072);
            auto run = [&]() {
                if (c.mode == 0)
                    hipLaunchKernelGGL((mix_kernel<true, 0>), dim3(blocks), dim3(256), 0, 0, out, iters, 0x80000000u, src, span);
                else if (c.mode == 1)
                    hipLaunchKernelGGL((mix_kernel<true, 1>), dim3(blocks), dim3(256), 0, 0, out, iters, 0x80000000u, src, span);
                else
                    hipLaunchKernelGGL((mix_kernel<true, 2>), dim3(blocks), dim3(256), 0, 0, out, iters, 0x80000000u, src, span);
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
            std::printf("{\"case\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f}\n",
                        c.what, wps, ms, flops / (ms / 1e3) / 1e12);
        }
    return 0;
}
