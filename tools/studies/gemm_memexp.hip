// Where the config-2 GEMM loses its last ~12 % (not part of the product): the library's default
// LDS-DMA kernel (128x128x16, 16 waves, split-K 4) timed on the config-2 shape with its operands
// (a) as in the bench, (b) the same 50 MB per operand for every batch entry (operands resident in
// the 256 MB Infinity Cache, HBM idle), (c) every row of a batch entry the same 196 KB row
// (operands L2-resident).  Outputs of (b) / (c) are not checked (different products).  Also: the
// shader clock of workgroup 0 over back-to-back launches, and the time on small-integer and on
// zero operands (MFMA switching activity).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form \
//        tools/studies/gemm_memexp.hip superbblas_amd/csrc/runtime.cpp -o tools/gemm_memexp
#include "../../superbblas_amd/csrc/kernels_gemm.hip"

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <cstring>
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

static double time_ms(const GemmKArgs &p, int reps) {
    hipStream_t s = get_stream(0);
    for (int i = 0; i < 5; ++i)
        launch_dma_cfg<double, true, true, true, 128, 128, 16, 4, 4>(p, 0, s, 0, 256);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    for (int i = 0; i < reps; ++i)
        launch_dma_cfg<double, true, true, true, 128, 128, 16, 4, 4>(p, 0, s, 0, 256);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps;
}

int main(int argc, char **argv) {
    const long L = 16, n = 64;
    const long m = 4 * n, nn = 4 * n, k = L * L * L * 3, batch = L;
    const int reps = argc > 1 ? atoi(argv[1]) : 20;
    double *A, *B, *C;
    (void)hipMalloc(&A, sizeof(double) * 2 * m * k * batch);
    (void)hipMalloc(&B, sizeof(double) * 2 * nn * k * batch);
    (void)hipMalloc(&C, sizeof(double) * 2 * m * nn * batch);
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
    const GemmKArgs p = make_args(d);
    const double flops = 8.0 * m * nn * k * batch;
    {
        // shader clock of workgroup 0 during back-to-back launches (s_memtime / s_memrealtime)
        unsigned long long *probe;
        (void)hipMalloc(&probe, 16);
        GemmKArgs q = p;
        q.probe = probe;
        for (int r = 0; r < 40; ++r) {
            launch_dma_cfg<double, true, true, true, 128, 128, 16, 4, 4, false>(q, 0, get_stream(0), 0, 256);
            if (r % 8 == 7) {
                (void)hipStreamSynchronize(get_stream(0));
                unsigned long long h[2];
                (void)hipMemcpy(h, probe, 16, hipMemcpyDeviceToHost);
                std::printf("back-to-back launch %2d: wg0 %.1f us, shader clock %.3f GHz\n", r,
                            h[1] / 100.0, (double)h[0] / (h[1] / 100e6) / 1e9);
            }
        }
    }
    for (int r = 0; r < 3; ++r) {
        GemmKArgs q = p;
        const double t0 = time_ms(q, reps);
        q.sa_b = 0;
        q.sb_b = 0;
        const double t1 = time_ms(q, reps);
        q = p;
        q.sa_m = 0;
        q.sb_n = 0;
        const double t2 = time_ms(q, reps);
        std::printf("round %d: bench operands %.4f ms (%.2f TF) | one batch entry (MALL) %.4f ms "
                    "(%.2f TF) | one row per entry (L2) %.4f ms (%.2f TF)\n",
                    r, t0, flops / t0 / 1e9, t1, flops / t1 / 1e9, t2, flops / t2 / 1e9);
    }
    // operand data: the same launches on small-integer and on zero operands (MFMA switching
    // activity; cycles per MFMA do not depend on the data, the power draw does)
    fill_kernel<<<4096, 256>>>(A, 2 * m * k * batch, 1);
    {
        const long na = 2 * m * k * batch, nb = 2 * nn * k * batch;
        std::vector<double> h(1 << 20);
        for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((long)(i * 7 % 5) - 2);
        for (long o = 0; o < na; o += (long)h.size())
            (void)hipMemcpy(A + o, h.data(), sizeof(double) * std::min<long>(h.size(), na - o), hipMemcpyHostToDevice);
        for (long o = 0; o < nb; o += (long)h.size())
            (void)hipMemcpy(B + o, h.data(), sizeof(double) * std::min<long>(h.size(), nb - o), hipMemcpyHostToDevice);
        for (int r = 0; r < 2; ++r) {
            const double t = time_ms(p, reps);
            std::printf("small-integer operands (-2..2): %.4f ms (%.2f TF)\n", t, flops / t / 1e9);
        }
        (void)hipMemset(A, 0, sizeof(double) * na);
        (void)hipMemset(B, 0, sizeof(double) * nb);
        for (int r = 0; r < 2; ++r) {
            const double t = time_ms(p, reps);
            std::printf("zero operands: %.4f ms (%.2f TF)\n", t, flops / t / 1e9);
        }
    }
    return 0;
}
