// The HBM streaming ceiling of this box (not part of the product): what a kernel can move per
// second when it does nothing else, by access form -- the denominator every "fraction of HBM"
// in DESIGN.md is quoted against besides the 8 TB/s spec.
//   read      : 16 B per lane global loads, summed (read-only stream)
//   read_nt   : the same with the non-temporal policy
//   copy      : 16 B per lane load + store (read + write bytes)
//   copy_nt   : the same, non-temporal loads and stores
//   dma       : buffer_load_dwordx4 ... lds (LDS-DMA), one 1-KB piece per wave instruction, into a
//               per-wave LDS ring (read-only stream)
//   dma_nt    : the same with the nt policy (aux bit)
//   memcpy    : hipMemcpyAsync device to device (read + write bytes)
// Every form streams a buffer far larger than the 256 MB Infinity Cache; medians of REPS runs.
// Build: make -C tools/studies stream_ceiling
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef double v2 __attribute__((ext_vector_type(2)));

template <bool NT>
__global__ void __launch_bounds__(256) read_kernel(const v2 *__restrict__ p, long n, double *out) {
    v2 acc = {0, 0};
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) {
        v2 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
        acc += v;
    }
    if (acc.x == 1.2345e300) out[0] = acc.y; // keep the loads
}

template <bool NT>
__global__ void __launch_bounds__(256) copy_kernel(const v2 *__restrict__ p, v2 *__restrict__ q, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256L) {
        if (NT)
            __builtin_nontemporal_store(__builtin_nontemporal_load(p + i), q + i);
        else
            q[i] = p[i];
    }
}

// Several loads per lane before the first use (round 6: the round-5 forms above keep one 16-B
// load per lane in flight between uses, which understates the ceiling -- the library's own block
// transpose copy moved 5.39 TB/s against copy's 4.62): U loads of 16 B per lane, U * 4 KB per
// wave ... issued back to back, then their stores; one-shot grids (no grid-stride loop) or a
// grid-stride loop over U-deep chunks
template <int U, bool NT>
__global__ void __launch_bounds__(256) read_u_kernel(const v2 *__restrict__ p, long n, double *out) {
    v2 acc = {0, 0};
    const long stride = (long)gridDim.x * 256L * U;
    for (long base = blockIdx.x * 256L * U + threadIdx.x; base < n; base += stride) {
        v2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + u * 256L;
            v[u] = i < n ? (NT ? __builtin_nontemporal_load(p + i) : p[i]) : v2{0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc += v[u];
    }
    if (acc.x == 1.2345e300) out[0] = acc.y; // keep the loads
}

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_u_kernel(const v2 *__restrict__ p, v2 *__restrict__ q, long n) {
    const long stride = (long)gridDim.x * 256L * U;
    for (long base = blockIdx.x * 256L * U + threadIdx.x; base < n; base += stride) {
        v2 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + u * 256L;
            if (i < n) v[u] = NT ? __builtin_nontemporal_load(p + i) : p[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long i = base + u * 256L;
            if (i < n) {
                if (NT)
                    __builtin_nontemporal_store(v[u], q + i);
                else
                    q[i] = v[u];
            }
        }
    }
}

// LDS-DMA stream: each wave moves consecutive 1-KB pieces into a RING-slot ring of its own,
// RING - 1 pieces in flight past the one waited for
template <int AUX, int RING = 4>
__global__ void __launch_bounds__(256) dma_kernel(const v2 *__restrict__ p, long n16, double *out) {
    __shared__ v2 ring[4 * RING * 64];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    const long waves = (long)gridDim.x * 4, gw = blockIdx.x * 4L + wave;
    const long pieces = n16 / 64;
    const unsigned base = (unsigned)(size_t)(const __attribute__((address_space(3))) void *)(ring + wave * RING * 64);
    int slot = 0;
    for (long pc = gw; pc < pieces; pc += waves) {
        // a buffer descriptor covers < 2 GiB: rebase every piece (pieces stay inside it)
        const v2 *src = p + __builtin_amdgcn_readfirstlane((int)(pc >> 20)) * (64L << 20);
        const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void *)src, (short)0, 0x7fffffff, 0x00020000);
        const unsigned dst = base + slot * 1024;
        const unsigned off = (unsigned)((pc & ((1L << 20) - 1)) * 1024 + lane * 16);
        if (AUX)
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen nt lds"
                         :: "v"(off), "s"(dst), "s"(r) : "memory", "m0");
        else
            asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %2, 0 offen lds"
                         :: "v"(off), "s"(dst), "s"(r) : "memory", "m0");
        slot = (slot + 1) % RING;
        if (RING == 4) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
        else if (RING == 8) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ring[lane].x == 1.2345e300) out[0] = 1; // keep the ring live
}

int main(int argc, char **argv) {
    const long bytes = (argc > 1 ? atol(argv[1]) : 2048) << 20; // MiB per buffer
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    const long n = bytes / 16;
    v2 *a, *b;
    double *out;
    (void)hipMalloc(&a, bytes);
    (void)hipMalloc(&b, bytes);
    (void)hipMalloc(&out, 64);
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 2, bytes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 256;
    auto time = [&](const char *name, double moved, auto f) {
        std::vector<float> t;
        f();
        (void)hipDeviceSynchronize();
        for (int r = 0; r < reps; ++r) {
            (void)hipEventRecord(e0, 0);
            f();
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        const double med = t[t.size() / 2], best = t.front();
        std::printf("%-9s %8.3f ms median  %6.3f TB/s median  %6.3f TB/s best  (%.2f of 8 TB/s)\n", name,
                    med, moved / med / 1e9, moved / best / 1e9, moved / med / 1e9 / 8.0);
    };
    const int blocks = cus * 16;
    time("read", bytes, [&] { read_kernel<false><<<blocks, 256>>>(a, n, out); });
    time("read_nt", bytes, [&] { read_kernel<true><<<blocks, 256>>>(a, n, out); });
    time("copy", 2.0 * bytes, [&] { copy_kernel<false><<<blocks, 256>>>(a, b, n); });
    time("copy_nt", 2.0 * bytes, [&] { copy_kernel<true><<<blocks, 256>>>(a, b, n); });
    time("dma", bytes, [&] { dma_kernel<0><<<cus * 8, 256>>>(a, n, out); });
    time("dma_nt", bytes, [&] { dma_kernel<1><<<cus * 8, 256>>>(a, n, out); });
    time("memcpy", 2.0 * bytes, [&] { (void)hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); });
    // round 6: several loads per lane in flight; one-shot grids (blocks = n / (256 U)) and
    // persistent ones (cus * 8 blocks, grid-stride over U-deep chunks)
    const long one4 = (n + 1023) / 1024, one8 = (n + 2047) / 2048;
    time("read_u4", bytes, [&] { read_u_kernel<4, false><<<one4, 256>>>(a, n, out); });
    time("read_u8", bytes, [&] { read_u_kernel<8, false><<<one8, 256>>>(a, n, out); });
    time("read_u8nt", bytes, [&] { read_u_kernel<8, true><<<one8, 256>>>(a, n, out); });
    time("read_u8p", bytes, [&] { read_u_kernel<8, false><<<cus * 8, 256>>>(a, n, out); });
    time("copy_u4", 2.0 * bytes, [&] { copy_u_kernel<4, false><<<one4, 256>>>(a, b, n); });
    time("copy_u8", 2.0 * bytes, [&] { copy_u_kernel<8, false><<<one8, 256>>>(a, b, n); });
    time("copy_u4nt", 2.0 * bytes, [&] { copy_u_kernel<4, true><<<one4, 256>>>(a, b, n); });
    time("copy_u8nt", 2.0 * bytes, [&] { copy_u_kernel<8, true><<<one8, 256>>>(a, b, n); });
    time("copy_u4p", 2.0 * bytes, [&] { copy_u_kernel<4, false><<<cus * 8, 256>>>(a, b, n); });
    time("copy_u8p", 2.0 * bytes, [&] { copy_u_kernel<8, false><<<cus * 4, 256>>>(a, b, n); });
    time("dma_r8", bytes, [&] { dma_kernel<0, 8><<<cus * 8, 256>>>(a, n, out); });
    time("dma_r8nt", bytes, [&] { dma_kernel<1, 8><<<cus * 8, 256>>>(a, n, out); });
    time("dma_r16nt", bytes, [&] { dma_kernel<1, 16><<<cus * 4, 256>>>(a, n, out); });
    time("dma_r16", bytes, [&] { dma_kernel<0, 16><<<cus * 4, 256>>>(a, n, out); });
    // fewer waves per CU, each with more pieces in flight
    time("dma_r8nt_w4", bytes, [&] { dma_kernel<1, 8><<<cus * 1, 256>>>(a, n, out); });
    time("dma_r8nt_w8", bytes, [&] { dma_kernel<1, 8><<<cus * 2, 256>>>(a, n, out); });
    time("dma_r16nt_w8", bytes, [&] { dma_kernel<1, 16><<<cus * 2, 256>>>(a, n, out); });
    time("dma_r4nt_w16", bytes, [&] { dma_kernel<1, 4><<<cus * 4, 256>>>(a, n, out); });
    return 0;
}
