// Tuning harness for the batched complex GEMM (not part of the product).  Includes the kernel
// translation unit and times tile/split variants on the lattice contraction shape with HIP
// events.  Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_tune.hip
//                superbblas_amd/csrc/runtime.cpp -o gemm_tune
#include "../superbblas_amd/csrc/kernels_gemm.hip"

#include <cstdio>
#include <random>

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

template <int BM, int BN, int BKK, int WM, int WN>
void run(const char *name, GemmKArgs p, long splits, long target, int reps, double flops) {
    hipStream_t s = get_stream(0);
    for (int i = 0; i < 2; ++i)
        launch_tiled_cfg<double, true, true, true, BM, BN, BKK, WM, WN>(p, 0, s, splits, target);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a, s);
    for (int i = 0; i < reps; ++i)
        launch_tiled_cfg<double, true, true, true, BM, BN, BKK, WM, WN>(p, 0, s, splits, target);
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    ms /= reps;
    std::printf("%-34s splits=%-3ld target=%-5ld  %8.3f ms  %7.2f TFLOP/s\n", name, splits,
                target, ms, flops / (ms * 1e-3) / 1e12);
}

int main(int argc, char **argv) {
    const long L = 16, n = 64;
    const long m = 4 * n, nn = 4 * n, k = L * L * L * 3, batch = L;
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
    GemmKArgs p = make_args(d);
    const double flops = 8.0 * m * nn * k * batch;
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    run<64, 64, 16, 2, 2>("64x64x16 w2x2", p, 0, 1024, reps, flops);
    run<64, 64, 16, 2, 2>("64x64x16 w2x2", p, 0, 512, reps, flops);
    run<64, 64, 16, 2, 2>("64x64x16 w2x2", p, 0, 2048, reps, flops);
    run<64, 64, 32, 2, 2>("64x64x32 w2x2", p, 0, 512, reps, flops);
    run<64, 64, 32, 2, 2>("64x64x32 w2x2", p, 0, 1024, reps, flops);
    run<64, 64, 8, 2, 2>("64x64x8 w2x2", p, 0, 1024, reps, flops);
    run<128, 64, 16, 4, 2>("128x64x16 w4x2", p, 0, 512, reps, flops);
    run<128, 64, 16, 4, 2>("128x64x16 w4x2", p, 0, 1024, reps, flops);
    run<128, 128, 16, 4, 2>("128x128x16 w4x2", p, 0, 256, reps, flops);
    run<128, 128, 16, 4, 2>("128x128x16 w4x2", p, 0, 512, reps, flops);
    run<64, 64, 16, 2, 2>("64x64x16 w2x2 (again)", p, 0, 1024, reps, flops);
    return 0;
}
