// Microbenchmark (not part of the product): v_mfma_f64_16x16x4_f64 issue rate for the operand
// patterns of the config-2 GEMM's inner loop -- 16 MFMAs per k-step into 8 accumulators (2 x 2
// output blocks, real and imaginary), A / B from 4 + 4 different registers -- against the peak
// loop's single operand pair; 4 waves per SIMD, operands random or constant.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
#define MMA(a, b, c) c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0)

template <int MODE>
__global__ void __launch_bounds__(1024) loop(const double *in, double *out, int iters,
                                             unsigned long long *clk) {
    const int t = threadIdx.x;
    double ax0 = in[t], ay0 = in[t + 1024], ax1 = in[t + 2048], ay1 = in[t + 3072];
    double bx0 = in[t + 4096], by0 = in[t + 5120], bx1 = in[t + 6144], by1 = in[t + 7168];
    d4 r00 = {0, 0, 0, 0}, r01 = r00, r10 = r00, r11 = r00, i00 = r00, i01 = r00, i10 = r00, i11 = r00;
    // MODE 2 / 3: each k-step's four complex fragments read from LDS first (ds_read_b128 at the
    // GEMM's swizzled addresses), MODE 3 with a barrier every four k-steps (one 16-deep slab)
    __shared__ double2 lds[2 * 256 * 16];
    for (int i = t; i < 2 * 256 * 16; i += 1024) lds[i] = double2{in[i & 8191], in[(i + 7) & 8191]};
    __syncthreads();
    const int lane = t & 63, wave = t >> 6, wm = wave / 4, wn = wave % 4;
    const int frow = wm * 32 + (lane & 15), fcol = wn * 32 + (lane & 15), kq = lane >> 4;
    auto slot = [](int row, int k) { return row * 16 + ((k ^ (row & 15))); };
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
        if (MODE == 0) { // one operand pair (the peak loop's pattern), 16 MFMAs per iteration
            MMA(ax0, bx0, r00); MMA(ax0, bx0, r01); MMA(ax0, bx0, r10); MMA(ax0, bx0, r11);
            MMA(ax0, bx0, i00); MMA(ax0, bx0, i01); MMA(ax0, bx0, i10); MMA(ax0, bx0, i11);
            MMA(ax0, bx0, r00); MMA(ax0, bx0, r01); MMA(ax0, bx0, r10); MMA(ax0, bx0, r11);
            MMA(ax0, bx0, i00); MMA(ax0, bx0, i01); MMA(ax0, bx0, i10); MMA(ax0, bx0, i11);
        } else if (MODE >= 2) {
#pragma unroll
            for (int kk = 0; kk < 16; kk += 4) {
                const double2 *L = lds + ((it >> 2) & 1) * 4096; // the slab buffer alternates
                const double2 a0 = L[slot(frow, kk + kq)], a1 = L[slot(frow + 16, kk + kq)];
                const double2 b0 = L[2048 + slot(fcol, kk + kq)], b1 = L[2048 + slot(fcol + 16, kk + kq)];
                MMA(a0.x, b0.x, r00); MMA(a0.x, b1.x, r01); MMA(a1.x, b0.x, r10); MMA(a1.x, b1.x, r11);
                MMA(a0.x, b0.y, i00); MMA(a0.x, b1.y, i01); MMA(a1.x, b0.y, i10); MMA(a1.x, b1.y, i11);
                MMA(a0.y, b0.y, r00); MMA(a0.y, b1.y, r01); MMA(a1.y, b0.y, r10); MMA(a1.y, b1.y, r11);
                MMA(a0.y, b0.x, i00); MMA(a0.y, b1.x, i01); MMA(a1.y, b0.x, i10); MMA(a1.y, b1.x, i11);
            }
            if (MODE == 3) __syncthreads();
            it += 3;
        } else { // the GEMM's complex 4M pattern
            MMA(ax0, bx0, r00); MMA(ax0, bx1, r01); MMA(ax1, bx0, r10); MMA(ax1, bx1, r11);
            MMA(ax0, by0, i00); MMA(ax0, by1, i01); MMA(ax1, by0, i10); MMA(ax1, by1, i11);
            MMA(ay0, by0, r00); MMA(ay0, by1, r01); MMA(ay1, by0, r10); MMA(ay1, by1, r11);
            MMA(ay0, bx0, i00); MMA(ay0, bx1, i01); MMA(ay1, bx0, i10); MMA(ay1, bx1, i11);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
    d4 s = r00 + r01 + r10 + r11 + i00 + i01 + i10 + i11;
    out[blockIdx.x * 1024 + t] = s[0] + s[1] + s[2] + s[3];
    if (t == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = q1 - q0; }
}

__global__ void fill(double *p, int n, int rnd) {
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        unsigned x = (unsigned)i * 2654435761u;
        x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
        p[i] = rnd ? (double)(x & 0xffffff) / 8388608.0 - 1.0 : 0.5;
    }
}

template <int MODE> void run(const char *name, const double *in, double *out, unsigned long long *clk) {
    const int iters = 20000;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    loop<MODE><<<256, 1024>>>(in, out, iters / 4, clk);
    (void)hipEventRecord(e0);
    loop<MODE><<<256, 1024>>>(in, out, iters, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    const double mf = 16.0 * iters * 4; // MFMAs per SIMD (4 waves)
    std::printf("%-34s %.3f ms  %.2f TFLOP/s  clock %.3f GHz  %.1f cycles per MFMA per SIMD\n", name,
                ms, 2.0 * 1024 * mf * 1024 / ms / 1e9, c[0] / (c[1] / 100e6) / 1e9, c[0] / mf);
}

// MODE 3 plus the GEMM's operand staging: every slab's 64 KB (A and B images) moved global -> LDS
// by LDS-DMA into the other buffer while the current one feeds the MFMAs, vmcnt(0) + barrier per
// slab (the config-2 GEMM's loop without its index arithmetic)
// SPREAD: 0 = the next slab's four DMA instructions right after the barrier (the GEMM), 1 = two
// after the first and two after the second k-step's fragment reads, 2 = one per k-step
template <int SPREAD>
__global__ void __launch_bounds__(1024) loop_dma(const double2 *src, double *out, int nslab,
                                                 unsigned long long *clk) {
    __shared__ double2 lds[2 * 256 * 16];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wm = wave / 4, wn = wave % 4;
    const int frow = wm * 32 + (lane & 15), fcol = wn * 32 + (lane & 15), kq = lane >> 4;
    auto slot = [](int row, int k) { return row * 16 + ((k ^ (row & 15))); };
    d4 r00 = {0, 0, 0, 0}, r01 = r00, r10 = r00, r11 = r00, i00 = r00, i01 = r00, i10 = r00, i11 = r00;
    const double2 *base = src + (size_t)(blockIdx.x % 64) * nslab * 4096;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void *)base, (short)0, (int)(nslab * 4096 * 16), 0x00020000);
    const unsigned lbase = (unsigned)(size_t)(const __attribute__((address_space(3))) void *)lds;
    auto issue = [&](int sl, int buf, int i0 = 0, int i1 = 4) {
#pragma unroll
        for (int i = i0; i < i1; ++i) {
            const unsigned off = (unsigned)((sl * 4096 + i * 1024 + t) * 16);
            const unsigned dst = lbase + (unsigned)(buf * 4096 + i * 1024 + wave * 64) * 16;
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
                         : : "v"(off), "s"(__builtin_amdgcn_readfirstlane(dst)), "s"(rs) : "memory", "m0");
        }
    };
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), q0 = __builtin_amdgcn_s_memrealtime();
    issue(0, 0);
    for (int sl = 0; sl < nslab; ++sl) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const bool more = sl + 1 < nslab;
        if (SPREAD == 0 && more) issue(sl + 1, (sl + 1) & 1);
        const double2 *L = lds + (sl & 1) * 4096;
#pragma unroll
        for (int kk = 0; kk < 16; kk += 4) {
            const double2 a0 = L[slot(frow, kk + kq)], a1 = L[slot(frow + 16, kk + kq)];
            const double2 b0 = L[2048 + slot(fcol, kk + kq)], b1 = L[2048 + slot(fcol + 16, kk + kq)];
            if (SPREAD == 1 && more && kk < 8) issue(sl + 1, (sl + 1) & 1, kk / 2, kk / 2 + 2);
            if (SPREAD == 2 && more) issue(sl + 1, (sl + 1) & 1, kk / 4, kk / 4 + 1);
            MMA(a0.x, b0.x, r00); MMA(a0.x, b1.x, r01); MMA(a1.x, b0.x, r10); MMA(a1.x, b1.x, r11);
            MMA(a0.x, b0.y, i00); MMA(a0.x, b1.y, i01); MMA(a1.x, b0.y, i10); MMA(a1.x, b1.y, i11);
            MMA(a0.y, b0.y, r00); MMA(a0.y, b1.y, r01); MMA(a1.y, b0.y, r10); MMA(a1.y, b1.y, r11);
            MMA(a0.y, b0.x, i00); MMA(a0.y, b1.x, i01); MMA(a1.y, b0.x, i10); MMA(a1.y, b1.x, i11);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), q1 = __builtin_amdgcn_s_memrealtime();
    d4 sm = r00 + r01 + r10 + r11 + i00 + i01 + i10 + i11;
    out[blockIdx.x * 1024 + t] = sm[0] + sm[1] + sm[2] + sm[3];
    if (t == 0 && blockIdx.x == 0) { clk[0] = t1 - t0; clk[1] = q1 - q0; }
}

template <int SPREAD>
static void run_dma(const double2 *src, double *out, unsigned long long *clk) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) loop_dma<SPREAD><<<256, 1024>>>(src, out, 192, clk);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) loop_dma<SPREAD><<<256, 1024>>>(src, out, 192, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    std::printf("MODE 3 + LDS-DMA staging (spread %d), 192 slabs, 20 launches: %.4f ms per launch, "
                "wg0 loop %.1f us at %.3f GHz\n", SPREAD, ms / 20, c[1] / 100.0,
                c[0] / (c[1] / 100e6) / 1e9);
}

// MODE 3 at the config-2 GEMM's length (192 slabs of 64 MFMAs per wave), launched back to back
static void run_short(const double *in, double *out, unsigned long long *clk) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int i = 0; i < 5; ++i) loop<3><<<256, 1024>>>(in, out, 768, clk);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 20; ++i) loop<3><<<256, 1024>>>(in, out, 768, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, 16, hipMemcpyDeviceToHost);
    std::printf("MODE 3, 192 slabs per launch, 20 launches: %.4f ms per launch (ideal at 2.4 GHz "
                "1.3107), wg0 loop %.1f us at %.3f GHz\n", ms / 20, c[1] / 100.0,
                c[0] / (c[1] / 100e6) / 1e9);
}

int main() {
    double *in, *out;
    unsigned long long *clk;
    (void)hipMalloc(&in, 8192 * sizeof(double));
    (void)hipMalloc(&out, 256 * 1024 * sizeof(double));
    (void)hipMalloc(&clk, 16);
    fill<<<32, 256>>>(in, 8192, 1);
    for (int rep = 0; rep < 1; ++rep) run_short(in, out, clk);
    {
        double2 *src;
        const size_t n = (size_t)64 * 192 * 4096;
        (void)hipMalloc(&src, n * sizeof(double2));
        fill<<<4096, 256>>>((double *)src, (int)std::min<size_t>(2 * n, 0x7fffffff), 1);
        for (int rep = 0; rep < 3; ++rep) {
            run_dma<0>(src, out, clk);
            run_dma<1>(src, out, clk);
            run_dma<2>(src, out, clk);
        }
    }
    for (int rep = 0; rep < 0; ++rep) {
        fill<<<32, 256>>>(in, 8192, 0);
        run<0>("one operand pair, constant data", in, out, clk);
        run<1>("GEMM pattern, constant data", in, out, clk);
        fill<<<32, 256>>>(in, 8192, 1);
        run<0>("one operand pair, random data", in, out, clk);
        run<1>("GEMM pattern, random data", in, out, clk);
        run<2>("GEMM pattern + LDS fragment reads", in, out, clk);
        run<3>("... + a barrier per 16-deep slab", in, out, clk);
    }
    return 0;
}
