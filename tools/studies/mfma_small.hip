// Microbenchmark and layout probe (not part of the product): the small-block MFMA forms
// v_mfma_f64_4x4x4_4b_f64 (4 blocks of 4x4x4) and v_mfma_f32_4x4x1_16b_f32 (16 blocks of
// 4x4x1) against v_mfma_f64_16x16x4_f64: cycles per instruction with independent chains on every
// SIMD, and the lane maps of the A, B and C/D operands (one-hot probes).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void probe_f64(double *out) {
    // out[(la * 64 + lb) * 64 + lane] = C[lane] for A one-hot at lane la, B one-hot at lane lb
    const int lane = threadIdx.x;
    for (int la = 0; la < 64; ++la)
        for (int lb = 0; lb < 64; ++lb) {
            double c = __builtin_amdgcn_mfma_f64_4x4x4f64(lane == la ? 1.0 : 0.0, lane == lb ? 1.0 : 0.0, 0.0, 0, 0, 0);
            out[(la * 64 + lb) * 64 + lane] = c;
        }
}

__global__ void probe_f32(float *out) {
    const int lane = threadIdx.x;
    for (int la = 0; la < 64; ++la)
        for (int lb = 0; lb < 64; ++lb) {
            f4 c = __builtin_amdgcn_mfma_f32_4x4x1f32(lane == la ? 1.f : 0.f, lane == lb ? 1.f : 0.f, f4{0, 0, 0, 0}, 0, 0, 0);
            for (int r = 0; r < 4; ++r) out[((la * 64 + lb) * 64 + lane) * 4 + r] = c[r];
        }
}

template <int FORM>
__global__ void __launch_bounds__(256) rate(double *out, int iters) {
    const int lane = threadIdx.x & 63;
    double a = 0.5 + lane * 1e-3, b = 0.25 - lane * 1e-3;
    float af = (float)a, bf = (float)b;
    double c1[8];
    d4 c4[8];
    f4 cf[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        c1[i] = i;
        c4[i] = d4{(double)i, 1, 2, 3};
        cf[i] = f4{(float)i, 1, 2, 3};
    }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if constexpr (FORM == 0) c4[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c4[i], 0, 0, 0);
            else if constexpr (FORM == 1) c1[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c1[i], 0, 0, 0);
            else if constexpr (FORM == 2) cf[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(af, bf, cf[i], 0, 0, 0);
            else cf[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, bf, cf[i], 0, 0, 0);
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += c1[i] + c4[i][0] + c4[i][3] + cf[i][0] + cf[i][3];
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    double *pd;
    float *pf;
    (void)hipMalloc(&pd, 64 * 64 * 64 * sizeof(double));
    (void)hipMalloc(&pf, 64 * 64 * 64 * 4 * sizeof(float));
    probe_f64<<<1, 64>>>(pd);
    probe_f32<<<1, 64>>>(pf);
    static double hd[64 * 64 * 64];
    static float hf[64 * 64 * 64 * 4];
    (void)hipMemcpy(hd, pd, sizeof(hd), hipMemcpyDeviceToHost);
    (void)hipMemcpy(hf, pf, sizeof(hf), hipMemcpyDeviceToHost);
    // f64 4x4x4_4b: for each (la, lb) pair with a product, the output lane
    printf("f64_4x4x4_4b: la lb -> out lane (value)\n");
    for (int la = 0; la < 64; ++la)
        for (int lb = 0; lb < 64; ++lb)
            for (int l = 0; l < 64; ++l)
                if (hd[(la * 64 + lb) * 64 + l] != 0) printf("  A%d B%d -> C lane %d\n", la, lb, l);
    printf("f32_4x4x1_16b: la lb -> out lane.reg\n");
    for (int la = 0; la < 64; ++la)
        for (int lb = 0; lb < 64; ++lb)
            for (int l = 0; l < 64; ++l)
                for (int r = 0; r < 4; ++r)
                    if (hf[((la * 64 + lb) * 64 + l) * 4 + r] != 0) printf("  A%d B%d -> C lane %d reg %d\n", la, lb, l, r);
    double *o;
    (void)hipMalloc(&o, 256 * 4096 * sizeof(double));
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const char *names[] = {"f64 16x16x4", "f64 4x4x4_4b", "f32 4x4x1_16b", "f32 16x16x4"};
    const double fma_per[] = {16 * 16 * 4, 4 * 64, 16 * 16, 16 * 16 * 4};
    for (int form = 0; form < 4; ++form) {
        const int iters = 4000, blocks = 256 * 4;
        auto go = [&]() {
            if (form == 0) rate<0><<<blocks, 256>>>(o, iters);
            else if (form == 1) rate<1><<<blocks, 256>>>(o, iters);
            else if (form == 2) rate<2><<<blocks, 256>>>(o, iters);
            else rate<3><<<blocks, 256>>>(o, iters);
        };
        go();
        (void)hipEventRecord(e0);
        go();
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double inst = (double)blocks * 4 * iters * 8; // wave-instructions
        const double fmas = inst * fma_per[form];
        // cycles per instruction per SIMD at 2.4 GHz, 1024 SIMDs
        const double cyc = ms * 1e-3 * 2.4e9 * 1024 / inst;
        printf("%-14s %8.3f ms  %7.2f TFLOP/s  ~%5.1f cycles/inst (at 2.4 GHz)\n", names[form], ms,
               2 * fmas / (ms * 1e-3) / 1e12, cyc);
    }
    return 0;
}
