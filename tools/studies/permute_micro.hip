// Microbenchmark (not part of the product): the config-2p permute slice -- xyztsc {16,16,16,16,4,3}
// complex<double> into slice n of tnsxyzc {16,64,4,16,16,16,3} -- with hand-specialised transposes,
// against a plain copy of the same bytes.  After normalisation the slice is a transpose of
// q = xyz (4096 sites) and ts = (t, s) (64) in units of c = 3 elements (48 B): the source holds a
// site's 192 (t, s, c) elements contiguously (3 KB), the destination a (t, s) pair's 12 288
// (xyz, c) elements (196 KB; t stride 64 slices).  64 launches back to back (the bench's loop),
// HIP events; every output compared with the first kernel's.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

typedef double v2 __attribute__((ext_vector_type(2)));
constexpr int NQ = 4096, NTS = 64, NC = 3, SITE = NTS * NC; // 192 elements per site
constexpr long SLICE = (long)NQ * SITE;                      // 786 432 elements
constexpr long NSTR = 4L * NQ * NC;                          // n stride 49 152
constexpr long TSTR = 64L * NSTR;                            // t stride
constexpr long SSTR = (long)NQ * NC;                         // s stride 12 288

__device__ __forceinline__ long dst_off(int n, int ts, int q, int c) {
    return (long)(ts >> 2) * TSTR + (long)n * NSTR + (long)(ts & 3) * SSTR + (long)q * NC + c;
}

// plain copy of the slice's bytes into a contiguous region (the memcpy reference)
__global__ void __launch_bounds__(256) k_copy(const v2 *__restrict__ s, v2 *__restrict__ d, int n) {
    const long i = (long)blockIdx.x * 1024 + threadIdx.x;
    v2 t[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = s[i + 256 * k];
#pragma unroll
    for (int k = 0; k < 4; ++k) __builtin_nontemporal_store(t[k], d + (long)n * SLICE + i + 256 * k);
}

// QT sites per workgroup: the QT x 3 KB source run loaded coalesced (QT*192/256 elements per
// thread, all in flight), transposed through LDS (one element of padding per site), written as
// 64 runs of QT*3 elements
template <int QT, bool NT>
__global__ void __launch_bounds__(256) k_tile(const v2 *__restrict__ s, v2 *__restrict__ d, int n) {
    constexpr int E = QT * SITE, PER = E / 256, LD = SITE + 1;
    __shared__ v2 lds[QT * LD];
    const int q0 = blockIdx.x * QT, t = threadIdx.x;
    v2 r[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) r[k] = s[(long)q0 * SITE + t + 256 * k];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = t + 256 * k, ql = j / SITE, e = j - ql * SITE;
        lds[ql * LD + e] = r[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = t + 256 * k, ts = j / (QT * NC), w = j - ts * (QT * NC), ql = w / NC,
                  c = w - ql * NC;
        const v2 v = lds[ql * LD + ts * NC + c];
        v2 *p = d + dst_off(n, ts, q0 + ql, c);
        if (NT)
            __builtin_nontemporal_store(v, p);
        else
            *p = v;
    }
}

// the same kernel with ~700 B of (unused) kernel arguments, as the library's launch struct
struct Big {
    long pad[88];
};
__global__ void __launch_bounds__(256) k_tile8_bigargs(const v2 *__restrict__ s, v2 *__restrict__ d, int n, Big b) {
    constexpr int QT = 8, E = QT * SITE, PER = E / 256, LD = SITE + 1;
    __shared__ v2 lds[QT * LD];
    const int q0 = blockIdx.x * QT, t = threadIdx.x;
    v2 r[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) r[k] = s[(long)q0 * SITE + t + 256 * k + b.pad[n & 63] * 0];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = t + 256 * k, ql = j / SITE, e = j - ql * SITE;
        lds[ql * LD + e] = r[k];
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int j = t + 256 * k, ts = j / (QT * NC), w = j - ts * (QT * NC), ql = w / NC,
                  c = w - ql * NC;
        __builtin_nontemporal_store(lds[ql * LD + ts * NC + c], d + dst_off(n, ts, q0 + ql, c));
    }
}

template <typename K>
static double time_loop(K k, int blocks, const v2 *s, v2 *d, int reps = 5) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int n = 0; n < 64; ++n) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, s, d, n);
    (void)hipEventRecord(a);
    for (int r = 0; r < reps; ++r)
        for (int n = 0; n < 64; ++n) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, s, d, n);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3 / (reps * 64); // us per slice
}

int main() {
    v2 *s, *d;
    const long nd = 16L * TSTR;
    (void)hipMalloc(&s, sizeof(v2) * SLICE);
    (void)hipMalloc(&d, sizeof(v2) * nd);
    std::vector<v2> h(SLICE);
    for (long i = 0; i < SLICE; ++i) h[i] = v2{(double)i, -(double)i};
    (void)hipMemcpy(s, h.data(), sizeof(v2) * SLICE, hipMemcpyHostToDevice);
    std::vector<v2> ref(nd), out(nd);
    auto check = [&](bool first) {
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(first ? ref.data() : out.data(), d, sizeof(v2) * nd, hipMemcpyDeviceToHost);
        return first || std::memcmp(ref.data(), out.data(), sizeof(v2) * nd) == 0;
    };
    const double gb = 32.0 * SLICE / 1e3; // bytes per slice / 1e3 -> GB/s from us
    for (int rep = 0; rep < 3; ++rep) {
        double us;
        us = time_loop(k_tile<16, true>, NQ / 16, s, d);
        std::printf("tile 16 sites (48 KB LDS, 256 WGs), nt stores: %.2f us/slice %.0f GB/s %s\n", us, gb / us, check(rep == 0) ? "" : "MISMATCH");
        us = time_loop(k_tile<8, true>, NQ / 8, s, d);
        std::printf("tile  8 sites (24 KB LDS, 512 WGs), nt stores: %.2f us/slice %.0f GB/s %s\n", us, gb / us, check(false) ? "" : "MISMATCH");
        us = time_loop(k_tile<4, true>, NQ / 4, s, d);
        std::printf("tile  4 sites (12 KB LDS, 1024 WGs), nt stores: %.2f us/slice %.0f GB/s %s\n", us, gb / us, check(false) ? "" : "MISMATCH");
        us = time_loop(k_tile<8, false>, NQ / 8, s, d);
        std::printf("tile  8 sites, plain stores: %.2f us/slice %.0f GB/s %s\n", us, gb / us, check(false) ? "" : "MISMATCH");
        us = time_loop(k_tile<4, false>, NQ / 4, s, d);
        std::printf("tile  4 sites, plain stores: %.2f us/slice %.0f GB/s %s\n", us, gb / us, check(false) ? "" : "MISMATCH");
        {
            Big big{};
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a);
            for (int r = 0; r < 5; ++r)
                for (int n = 0; n < 64; ++n)
                    hipLaunchKernelGGL(k_tile8_bigargs, dim3(NQ / 8), dim3(256), 0, 0, s, d, n, big);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            us = ms * 1e3 / (5 * 64);
            std::printf("tile  8 sites, nt stores, 700 B of kernel arguments: %.2f us/slice %.0f GB/s %s\n", us, gb / us, check(false) ? "" : "MISMATCH");
        }
        us = time_loop(k_copy, (int)(SLICE / 1024), s, d);
        std::printf("plain copy of the same bytes (nt stores): %.2f us/slice %.0f GB/s\n", us, gb / us);
    }
    return 0;
}
