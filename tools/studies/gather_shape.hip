// Microbenchmark (not part of the product): rate of 16-byte-per-lane vector loads by the shape of
// one wave-instruction's footprint -- 64 lanes as 1 piece of 1 KB (lane-linear), 2 x 512 B,
// 4 x 256 B, 8 x 128 B, 10 x 96 B (6 lanes each, the 3x3 BSR kernel's x gather at 12 rhs
// columns), 64 x 16 B -- with pieces at random places of a region that stays in the L2
// (2 MB) or does not (192 MB), into VGPRs (global_load_dwordx4) or into LDS (buffer_load ... lds).
// Question answered: does the vector-memory pipeline charge per byte or per piece?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ unsigned lds_u32(const void *p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void *)p;
}

// byte offset of lane `lane`'s 16 bytes in load `k` of iteration `it`
__device__ __forceinline__ unsigned lane_off(int piece_lanes, unsigned region, unsigned wave, int it,
                                             int k, int lane) {
    const int piece = lane / piece_lanes, pl = lane - piece * piece_lanes;
    const unsigned pbytes = (unsigned)piece_lanes * 16u;
    const unsigned npieces = region / 1024u; // piece slots on a 1 KB grid (96 B pieces: unaligned)
    const unsigned slot = hash32(wave * 7919u + (unsigned)it * 131u + (unsigned)k * 17u + (unsigned)piece) % npieces;
    (void)pbytes;
    return slot * 1024u + (unsigned)pl * 16u;
}

template <int K>
__global__ void __launch_bounds__(256) gather_vgpr(const double2 *__restrict__ buf, unsigned region,
                                                   int piece_lanes, int iters, double *out) {
    const int lane = threadIdx.x & 63;
    const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    double2 acc = {0, 0};
    for (int it = 0; it < iters; ++it) {
        double2 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            v[k] = buf[lane_off(piece_lanes, region, wave, it, k, lane) / 16u];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            acc.x += v[k].x;
            acc.y += v[k].y;
        }
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y;
}

template <int K>
__global__ void __launch_bounds__(256) gather_dma(const double2 *__restrict__ buf, unsigned region,
                                                  int piece_lanes, int iters, double *out) {
    __shared__ __attribute__((aligned(16))) double2 sh[256 * K];
    const int lane = threadIdx.x & 63;
    const unsigned wave = blockIdx.x * 4u + (threadIdx.x >> 6);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void *)buf, (short)0, (int)region, 0x00020000);
    const unsigned base = lds_u32(sh) + (threadIdx.x >> 6) * 1024u;
    double acc = 0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const unsigned off = lane_off(piece_lanes, region, wave, it, k, lane);
            const unsigned dst = __builtin_amdgcn_readfirstlane(base + (unsigned)k * 4096u);
            asm volatile("s_mov_b32 m0, %1\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %0, %2, 0 offen lds"
                         :
                         : "v"(off), "s"(dst), "s"(rs)
                         : "memory", "m0");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        acc += sh[threadIdx.x].x; // wave-private slice: no barrier needed for this probe
    }
    out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
    const size_t big = 192u << 20;
    double2 *buf;
    double *out;
    (void)hipMalloc(&buf, big);
    (void)hipMemset(buf, 0, big);
    const int wgs = 256 * 8;
    (void)hipMalloc(&out, sizeof(double) * 256 * wgs);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 64;
    constexpr int K = 8;
    const int shapes[] = {64, 32, 16, 8, 6, 1};
    for (unsigned region : {2u << 20, (unsigned)big}) {
        for (int dma = 0; dma < 2; ++dma) {
            for (int pl : shapes) {
                auto go = [&]() {
                    if (dma)
                        gather_dma<K><<<wgs, 256>>>(buf, region, pl, iters, out);
                    else
                        gather_vgpr<K><<<wgs, 256>>>(buf, region, pl, iters, out);
                };
                go();
                (void)hipEventRecord(e0);
                for (int r = 0; r < 5; ++r) go();
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                // bytes delivered to lanes (6-lane pieces: 10 pieces per wave, 4 lanes idle
                // -> count the 60 useful lanes)
                const int used = pl == 6 ? 60 : 64;
                const double bytes = 5.0 * wgs * 4.0 * iters * K * used * 16.0;
                const double tbs = bytes / (ms * 1e-3) / 1e12;
                printf("region %4u MB  %-4s piece %4d B : %7.3f ms  %6.2f TB/s  %6.1f GB/s/CU\n",
                       region >> 20, dma ? "dma" : "vgpr", pl * 16, ms / 5, tbs, tbs * 1e3 / 256);
            }
        }
    }
    return 0;
}
