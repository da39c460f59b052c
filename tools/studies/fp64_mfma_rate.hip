// FP64 matrix-core rate by instruction shape over the whole chip, timed by HIP events (not part
// of the product): v_mfma_f64_4x4x4_4b (256 MACs) against v_mfma_f64_16x16x4 (1024 MACs), NC
// independent accumulation chains per wave, W waves per SIMD; operands vary per iteration (no
// loop-invariant product).  Build: hipcc -O3 --offload-arch=gfx950 fp64_mfma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

template <int NC>
__global__ void __launch_bounds__(256) m4(double *out, int iters) {
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-6, b = 1.0 - lane * 1e-6;
    double m[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) m[i] = i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NC; ++i) m[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, m[i], 0, 0, 0);
        a += 1e-9;
        b -= 1e-9;
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NC; ++i) s += m[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int NC>
__global__ void __launch_bounds__(256) m16(double *out, int iters) {
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-6, b = 1.0 - lane * 1e-6;
    d4 m[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i) m[i] = d4{(double)i, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NC; ++i) m[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, m[i], 0, 0, 0);
        a += 1e-9;
        b -= 1e-9;
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NC; ++i) s += m[i][0] + m[i][1] + m[i][2] + m[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename K> double timeit(K k, int blocks, int iters, double *out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

int main() {
    double *out;
    const int iters = 20000;
    (void)hipMalloc(&out, sizeof(double) * 256 * 256 * 8);
    for (int wps = 1; wps <= 4; wps *= 2) {
        const int blocks = 256 * wps;
        const double waves = blocks * 4.0;
        double ms = timeit(m4<8>, blocks, iters, out);
        printf("{\"mfma\": \"4x4x4_4b\", \"chains\": 8, \"waves_per_simd\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f}\n", wps, ms,
               waves * iters * 8 * 256 * 2 / (ms * 1e-3) / 1e12);
        ms = timeit(m4<16>, blocks, iters, out);
        printf("{\"mfma\": \"4x4x4_4b\", \"chains\": 16, \"waves_per_simd\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f}\n", wps, ms,
               waves * iters * 16 * 256 * 2 / (ms * 1e-3) / 1e12);
        ms = timeit(m16<4>, blocks, iters / 4, out);
        printf("{\"mfma\": \"16x16x4\", \"chains\": 4, \"waves_per_simd\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f}\n", wps, ms,
               waves * (iters / 4) * 4 * 1024 * 2 / (ms * 1e-3) / 1e12);
        ms = timeit(m16<8>, blocks, iters / 4, out);
        printf("{\"mfma\": \"16x16x4\", \"chains\": 8, \"waves_per_simd\": %d, \"ms\": %.3f, \"TFLOPs\": %.1f}\n", wps, ms,
               waves * (iters / 4) * 8 * 1024 * 2 / (ms * 1e-3) / 1e12);
    }
    return 0;
}
