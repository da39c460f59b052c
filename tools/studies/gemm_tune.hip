// Tuning harness for the batched complex GEMM (not part of the product).  Includes the kernel
// translation unit and times tile/split variants on the lattice contraction shape with HIP
// events; every variant's output is checked against the register-staged kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form \
//        tools/studies/gemm_tune.hip superbblas_amd/csrc/runtime.cpp -o tools/studies/gemm_tune
#include "../../superbblas_amd/csrc/kernels_gemm.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <string>
#include <vector>

using namespace sbx;

__global__ void fill_kernel(double *p, long n, unsigned seed) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) {
        unsigned x = (unsigned)(i * 2654435761u) ^ seed;
        x ^= x >> 13;
        x *= 0x5bd1e995u;
        x ^= x >> 15;
        p[i] = (double)(x & 0xffffff) / 8388608.0 - 1.0;
    }
}

static double max_rel(const std::vector<double> &a, const std::vector<double> &b) {
    double num = 0, den = 0;
    for (size_t i = 0; i < a.size(); ++i) {
        num = std::max(num, std::fabs(a[i] - b[i]));
        den = std::max(den, std::fabs(b[i]));
    }
    return num / (den > 0 ? den : 1);
}

template <typename F>
void run(const char *name, F launch, const GemmKArgs &p, int reps, double flops,
         const std::vector<double> *ref, double *C, size_t nc) {
    hipStream_t s = get_stream(0);
    (void)hipMemsetAsync(C, 0, nc * sizeof(double), s);
    launch(p, s);
    (void)hipStreamSynchronize(s);
    double err = -1;
    if (ref) {
        std::vector<double> h(nc);
        (void)hipMemcpy(h.data(), C, nc * sizeof(double), hipMemcpyDeviceToHost);
        err = max_rel(h, *ref);
    }
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    static const bool sync_each = getenv("SYNC_EACH") != nullptr;
    for (int i = 0; i < reps; ++i) {
        launch(p, s);
        if (sync_each) (void)hipStreamSynchronize(s);
    }
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    std::printf("%-40s %8.3f ms  %7.2f TFLOP/s  err %.2e\n", name, ms,
                flops / (ms * 1e-3) / 1e12, err);
}

#define REG(BM, BN, BKK, WM, WN, SPL, TGT)                                                      \
    run("reg " #BM "x" #BN "x" #BKK " w" #WM "x" #WN " s" #SPL " t" #TGT,                         \
        [&](const GemmKArgs &q, hipStream_t s) {                                                 \
            launch_tiled_cfg<double, true, true, true, BM, BN, BKK, WM, WN>(q, 0, s, SPL, TGT);  \
        },                                                                                       \
        p, reps, flops, &ref, C, nc)
#define DMA(BM, BN, BKK, WM, WN, SPL, TGT)                                                      \
    run("dma " #BM "x" #BN "x" #BKK " w" #WM "x" #WN " s" #SPL " t" #TGT,                         \
        [&](const GemmKArgs &q, hipStream_t s) {                                                 \
            launch_dma_cfg<double, true, true, true, BM, BN, BKK, WM, WN>(q, 0, s, SPL, TGT);                   \
        },                                                                                       \
        p, reps, flops, &ref, C, nc)

#define DMAP(BM, BN, BKK, WM, WN, SPL, TGT)                                                     \
    run("dma-pf " #BM "x" #BN "x" #BKK " w" #WM "x" #WN " s" #SPL " t" #TGT,                      \
        [&](const GemmKArgs &q, hipStream_t s) {                                                 \
            launch_dma_cfg<double, true, true, true, BM, BN, BKK, WM, WN, false, true>(q, 0, s, SPL, TGT); \
        },                                                                                       \
        p, reps, flops, &ref, C, nc)

int main(int argc, char **argv) {
    const long L = 16, n = 64;
    const long m = 4 * n, nn = 4 * n, k = L * L * L * 3;
    const long batch = argc > 2 ? atol(argv[2]) : L;
    double *A, *B, *C;
    (void)hipMalloc(&A, sizeof(double) * 2 * m * k * batch);
    (void)hipMalloc(&B, sizeof(double) * 2 * nn * k * batch);
    const size_t nc = 2 * m * nn * batch;
    (void)hipMalloc(&C, sizeof(double) * nc);
    fill_kernel<<<4096, 256>>>(A, 2 * m * k * batch, 1);
    fill_kernel<<<4096, 256>>>(B, 2 * nn * k * batch, 2);
    (void)hipDeviceSynchronize();
    GemmDesc d;
    d.t = SBX_CDOUBLE;
    d.m = m; d.n = nn; d.k = k; d.batch = batch;
    d.a = A; d.sa_m = k; d.sa_k = 1; d.sa_b = m * k; d.conja = false;
    d.b = B; d.sb_k = 1; d.sb_n = k; d.sb_b = nn * k; d.conjb = false;
    d.c = C; d.sc_m = 1; d.sc_n = m; d.sc_b = m * nn;
    d.alpha = Scalar{1, 0};
    d.beta = Scalar{0, 0};
    GemmKArgs p = make_args(d);
    const double flops = 8.0 * m * nn * k * batch;
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    // reference output: register-staged kernel
    std::vector<double> ref(nc);
    launch_tiled_cfg<double, true, true, true, 64, 64, 16, 2, 2>(p, 0, get_stream(0), 0, 1024);
    (void)hipStreamSynchronize(get_stream(0));
    (void)hipMemcpy(ref.data(), C, nc * sizeof(double), hipMemcpyDeviceToHost);

    if (getenv("PROBE") && std::string(getenv("PROBE")) == "all") {
        // every workgroup's timeline (100 MHz ticks): start, main-loop end, end (after its
        // partial-tile stores have left the CU), relative to the earliest start
        const int lw = getenv("LOADERS") ? atoi(getenv("LOADERS")) : 0;
        g_gemm_tune.loaders = lw;
        const int nwg = 256;
        unsigned long long *probe;
        (void)hipMalloc(&probe, 8 * (2 + 3 * nwg));
        GemmKArgs q = p;
        q.probe = probe;
        q.probe_all = 1;
        for (int r = 0; r < 12; ++r) {
            if (lw == 8)
                launch_dma_cfg<double, true, true, true, 128, 128, 16, 4, 4, false, false, 1, false, 8, 1>(q, 0, get_stream(0), 0, 256);
            else
                launch_dma_cfg<double, true, true, true, 128, 128, 16, 4, 4, false>(q, 0, get_stream(0), 0, 256);
            (void)hipStreamSynchronize(get_stream(0));
            if (r < 8) continue;
            std::vector<unsigned long long> h(2 + 3 * nwg);
            (void)hipMemcpy(h.data(), probe, 8 * h.size(), hipMemcpyDeviceToHost);
            unsigned long long t0 = ~0ull, tmax = 0;
            for (int b = 0; b < nwg; ++b) {
                t0 = std::min(t0, h[2 + 3 * b]);
                tmax = std::max(tmax, h[4 + 3 * b]);
            }
            std::vector<double> st, loop, epi, end;
            for (int b = 0; b < nwg; ++b) {
                st.push_back((h[2 + 3 * b] - t0) / 100.0);
                loop.push_back((h[3 + 3 * b] - h[2 + 3 * b]) / 100.0);
                epi.push_back((h[4 + 3 * b] - h[3 + 3 * b]) / 100.0);
                end.push_back((h[4 + 3 * b] - t0) / 100.0);
            }
            auto pr = [](const char *nm, std::vector<double> v) {
                std::sort(v.begin(), v.end());
                std::printf("  %-10s min %8.1f  p10 %8.1f  med %8.1f  p90 %8.1f  max %8.1f us\n", nm,
                            v.front(), v[v.size() / 10], v[v.size() / 2], v[v.size() * 9 / 10],
                            v.back());
            };
            std::printf("rep %d (loaders %d): span %.1f us\n", r, lw, (tmax - t0) / 100.0);
            pr("start", st);
            pr("loop", loop);
            pr("epilogue", epi);
            pr("end", end);
            // per XCD (blockIdx % 8) mean loop time
            std::printf("  loop by bid%%8:");
            for (int x = 0; x < 8; ++x) {
                double a = 0;
                for (int b = x; b < nwg; b += 8) a += loop[b];
                std::printf(" %.1f", a / (nwg / 8));
            }
            std::printf("\n");
        }
        return 0;
    }
#ifdef SBX_SLAB_PROBE
    if (getenv("PROBE") && std::string(getenv("PROBE")) == "slab") {
        // workgroup 0, per wave and slab: shader clocks spent waiting (own DMA + the barrier)
        // and between barriers (fragment reads + MFMA issue), the default 8-loader form
        const long nslab = 192;
        unsigned long long *probe;
        const size_t words = 4096 + 16 * nslab * 2;
        (void)hipMalloc(&probe, 8 * words);
        GemmKArgs q = p;
        q.probe = probe;
        g_gemm_tune.loaders = 8;
        for (int r = 0; r < 12; ++r) {
            launch_dma_cfg<double, true, true, true, 128, 128, 16, 4, 4, false, false, 1, false, 8, 1>(q, 0, get_stream(0), 0, 256);
            (void)hipStreamSynchronize(get_stream(0));
            if (r < 9) continue;
            std::vector<unsigned long long> h(words);
            (void)hipMemcpy(h.data(), probe, 8 * words, hipMemcpyDeviceToHost);
            std::printf("rep %d: wg0 %.1f us at %.3f GHz\n", r, h[1] / 100.0, (double)h[0] / (h[1] / 100e6) / 1e9);
            double tw = 0, tc = 0;
            std::vector<double> waitv, compv;
            for (int w = 0; w < 16; ++w) {
                double sw = 0, sc = 0;
                for (long sl = 0; sl < nslab; ++sl) {
                    const unsigned long long *e = &h[4096 + (w * nslab + sl) * 2];
                    sw += (double)(e[1] - e[0]);
                    if (sl + 1 < nslab) sc += (double)(e[2] - e[1]);
                    waitv.push_back((double)(e[1] - e[0]));
                    if (sl + 1 < nslab) compv.push_back((double)(e[2] - e[1]));
                }
                tw += sw;
                tc += sc;
                std::printf("  wave %2d: wait+barrier %7.0f clk/slab, between barriers %7.0f clk/slab\n", w,
                            sw / nslab, sc / (nslab - 1));
            }
            auto pct = [](std::vector<double> v, double f) { std::sort(v.begin(), v.end()); return v[(size_t)(f * (v.size() - 1))]; };
            std::printf("  all waves: wait+barrier mean %.0f (p10 %.0f med %.0f p90 %.0f max %.0f), between %.0f (p10 %.0f med %.0f p90 %.0f) clk/slab;"
                        " 256 MFMAs per SIMD per slab = %d clk\n",
                        tw / (16 * nslab), pct(waitv, 0.1), pct(waitv, 0.5), pct(waitv, 0.9), pct(waitv, 1.0),
                        tc / (16 * (nslab - 1)), pct(compv, 0.1), pct(compv, 0.5), pct(compv, 0.9), 256 * 64);
        }
        return 0;
    }
#endif
    if (getenv("PROBE")) {
        // shader clock of workgroup 0 during the default 4M GEMM (s_memtime / s_memrealtime)
        unsigned long long *probe;
        (void)hipMalloc(&probe, 16);
        GemmKArgs q = p;
        q.probe = probe;
        for (int r = 0; r < 30; ++r) {
            launch_dma_cfg<double, true, true, true, 128, 128, 16, 4, 4, false>(q, 0, get_stream(0), 0, 256);
            (void)hipStreamSynchronize(get_stream(0));
            unsigned long long h[2];
            (void)hipMemcpy(h, probe, 16, hipMemcpyDeviceToHost);
            std::printf("probe rep %2d: wg0 %.1f us, clock %.3f GHz\n", r, h[1] / 100.0,
                        (double)h[0] / (h[1] / 100e6) / 1e9);
        }
        return 0;
    }
    const char *only = getenv("ONLY");
    if (only && std::string(only) == "w8") {
        // round 6: 8 waves of 64x32 (2 per SIMD, 0.19 fragment reads per MFMA instead of 0.25)
        // against the default 16 waves of 32x32, 8 loader waves
#define DMAL(NAME, WM, WN, LW)                                                                    \
    run(NAME, [&](const GemmKArgs &q, hipStream_t s) {                                            \
        launch_dma_cfg<double, true, true, true, 128, 128, 16, WM, WN, false, false, 1, false, LW, 1>(q, 0, s, 0, 256); \
    }, p, reps, flops, &ref, C, nc)
        for (int rep = 0; rep < 4; ++rep) {
            DMAL("w16 4x4 loaders 8 (default)", 4, 4, 8);
            DMAL("w8 2x4 loaders 4", 2, 4, 4);
            DMAL("w8 4x2 loaders 4", 4, 2, 4);
            DMAL("w8 2x4 loaders 8", 2, 4, 8);
            DMAL("w8 4x2 loaders 8", 4, 2, 8);
        }
        return 0;
    }
    for (int rep = 0; rep < 3; ++rep) {
        if (!only || std::string(only) == "a") DMA(128, 128, 8, 4, 2, 0, 256);
        if (!only || std::string(only) == "b") DMA(128, 128, 16, 4, 2, 0, 256);
        if (!only || std::string(only) == "c") DMA(128, 64, 8, 2, 2, 0, 512);
        if (!only || std::string(only) == "d") REG(64, 64, 16, 2, 2, 0, 1024);
        if (only && std::string(only) == "e") DMA(128, 128, 8, 4, 2, 1, 1);
        if (only && std::string(only) == "w16") {
            DMA(128, 128, 16, 4, 4, 0, 256);
            DMA(128, 128, 8, 4, 4, 0, 256);
            DMAP(128, 128, 8, 4, 4, 0, 256);
            DMA(128, 128, 16, 8, 2, 0, 256);
            DMA(128, 128, 16, 2, 8, 0, 256);
            DMA(128, 128, 16, 4, 4, 0, 512);
            DMA(128, 128, 8, 4, 4, 0, 512);
            DMA(128, 128, 8, 4, 2, 0, 256);
            continue;
        }
        if (!only || std::string(only) == "p") DMAP(128, 128, 16, 4, 2, 0, 256);
        if (!only || std::string(only) == "g") DMA(128, 128, 16, 4, 4, 0, 256);
        if (!only || std::string(only) == "gp") DMAP(128, 128, 16, 4, 4, 0, 256);
        if (!only || std::string(only) == "f") DMAP(128, 128, 16, 2, 2, 0, 256);
        if (!only || std::string(only) == "p8") DMAP(128, 128, 8, 4, 2, 0, 256);
        if (!only || std::string(only) == "s8") DMAP(128, 128, 16, 4, 2, 8, 256);
    }
    return 0;
}
