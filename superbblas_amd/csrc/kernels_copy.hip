// Strided N-D box copy / permute kernels (the `copy()` hot path of superbblas).
//
// Reference algorithm: local_copy -> copy_normalize -> get_permutation -> copy_n_blocking
// (tensor.h:701-800, 815-961, 978-1037; copy_n.h:584-950).  The reference materialises two
// int32 index vectors (one per side) and runs a thrust gather/scatter over `blocking`-element
// runs.  Here the offsets are computed arithmetically inside the kernel (no index vectors, no
// extra HBM traffic), and when the fastest destination dimension is not the fastest source
// dimension the copy goes through an LDS tile so both the reads and the writes are long
// contiguous runs (a tiled transpose over the normalised dimensions).
//
// Host-side normalisation (launch_box_copy):
//   1. drop size-1 dims, sort by destination stride, merge dims contiguous on both sides;
//   2. the leading dim contiguous on both sides becomes the run R (an "item" of R elements);
//   3. V = the chain of dims contiguous in the destination from stride R, U = the chain of dims
//      contiguous in the source
//      starting at stride R; everything else is an outer dim handled by the grid;
//   4. if U is empty the direct kernel (destination-ordered gather) is used.
#include "elem_ops.h"
#include "sbx_internal.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <numeric>
#include <type_traits>
#include <unordered_map>

namespace sbx {
CopyTune g_copy_tune;
namespace {

/// Unsigned 32-bit division by a runtime constant (mul-hi + shift)
struct FastDiv {
    uint32_t d, m, s;
    FastDiv() : d(1), m(0), s(0) {}
    explicit FastDiv(uint32_t d_) : d(d_) {
        if (d == 0) throw Error("FastDiv: zero divisor");
        s = 0;
        while ((1ull << s) < d) ++s;
        m = (uint32_t)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
    }
    __device__ __forceinline__ uint32_t div(uint32_t n) const {
        uint64_t t = __umulhi(n, m);
        return (uint32_t)((t + n) >> s);
    }
};

constexpr int MAXD = 12;

template <typename T> struct is_cplx { static constexpr bool value = false; };
template <> struct is_cplx<double2> { static constexpr bool value = true; };
template <> struct is_cplx<float2> { static constexpr bool value = true; };

// value conversions S -> D
template <typename D, typename S> __device__ __forceinline__ D conv(S v) { return (D)v; }
template <> __device__ __forceinline__ double2 conv<double2, double2>(double2 v) { return v; }
template <> __device__ __forceinline__ float2 conv<float2, float2>(float2 v) { return v; }
template <> __device__ __forceinline__ double2 conv<double2, float2>(float2 v) {
    return double2{(double)v.x, (double)v.y};
}
template <> __device__ __forceinline__ float2 conv<float2, double2>(double2 v) {
    return float2{(float)v.x, (float)v.y};
}
// real -> complex (blas.h:57-65 instantiates TREAL -> QCOMPLEX, never complex -> real)
template <> __device__ __forceinline__ double2 conv<double2, double>(double v) { return double2{v, 0}; }
template <> __device__ __forceinline__ double2 conv<double2, float>(float v) { return double2{(double)v, 0}; }
template <> __device__ __forceinline__ float2 conv<float2, float>(float v) { return float2{v, 0}; }
template <> __device__ __forceinline__ float2 conv<float2, double>(double v) { return float2{(float)v, 0}; }

struct Alpha {
    double re, im;
    int one; // 1: alpha == 1, no multiplication (bit-exact data movement); 2: alpha == 0, the
             // element is +0 (the reference zero-fills, copy_n.h:435-438: no 0 * v, no -0.0)
};

// alpha * v in the SOURCE type, then converted (the reference's copy_n computes alpha * v[i]
// with alpha of type elem<T>::type and v of the source type T, copy_n.h:147-244): a real source
// is scaled by the real part of alpha, so a real -> complex copy has a +0 imaginary part; the
// complex product is formed with separately rounded products (no FMA contraction), as the
// reference's C-complex multiply on the CPU
template <typename S> __device__ __forceinline__ S scale(S v, const Alpha &a) {
    return a.one == 1 ? v : a.one == 2 ? S{} : (S)(v * (S)a.re);
}
template <> __device__ __forceinline__ double2 scale<double2>(double2 v, const Alpha &a) {
#pragma clang fp contract(off)
    if (a.one == 1) return v;
    if (a.one == 2) return double2{0, 0};
    return double2{a.re * v.x - a.im * v.y, a.re * v.y + a.im * v.x};
}
template <> __device__ __forceinline__ float2 scale<float2>(float2 v, const Alpha &a) {
#pragma clang fp contract(off)
    if (a.one == 1) return v;
    if (a.one == 2) return float2{0, 0};
    const float ar = (float)a.re, ai = (float)a.im;
    return float2{ar * v.x - ai * v.y, ar * v.y + ai * v.x};
}
template <> __device__ __forceinline__ int scale<int>(int v, const Alpha &a) {
    return a.one == 2 ? 0 : v;
}
template <> __device__ __forceinline__ unsigned long scale<unsigned long>(unsigned long v, const Alpha &a) {
    return a.one == 2 ? 0ul : v;
}
/// the element written for source value v
template <typename D, typename S> __device__ __forceinline__ D xform(S v, const Alpha &a) {
    return conv<D, S>(scale<S>(v, a));
}
template <typename D> __device__ __forceinline__ D add(D a, D b) { return a + b; }
template <> __device__ __forceinline__ double2 add<double2>(double2 a, double2 b) {
    return double2{a.x + b.x, a.y + b.y};
}
template <> __device__ __forceinline__ float2 add<float2>(float2 a, float2 b) {
    return float2{a.x + b.x, a.y + b.y};
}

template <bool ADD, typename D> __device__ __forceinline__ void put(D *p, D v) {
    if constexpr (ADD)
        *p = add<D>(*p, v);
    else
        *p = v;
}

struct DirectArgs {
    int nd;
    uint32_t total;
    FastDiv size[MAXD];
    long sst[MAXD], dst[MAXD];
    const void *src;
    void *dstp;
    Alpha alpha;
};

// Destination-ordered gather: element idx is decoded in destination order (dim 0 fastest)
template <typename S, typename D, bool ADD>
__global__ void __launch_bounds__(256) copy_direct_kernel(const DirectArgs p) {
    const S *__restrict__ src = (const S *)p.src;
    D *__restrict__ dst = (D *)p.dstp;
    for (uint32_t idx = blockIdx.x * 256u + threadIdx.x; idx < p.total; idx += gridDim.x * 256u) {
        uint32_t rem = idx;
        long so = 0, doff = 0;
#pragma unroll
        for (int i = 0; i < MAXD; ++i) {
            if (i >= p.nd) break;
            const uint32_t q = p.size[i].div(rem);
            const uint32_t c = rem - q * p.size[i].d;
            rem = q;
            so += (long)c * p.sst[i];
            doff += (long)c * p.dst[i];
        }
        put<ADD, D>(dst + doff, xform<D, S>(src[so], p.alpha));
    }
}

// Masked destination-ordered gather (copy with MaskType masks, tensor.h:1019-1027): an element
// is moved only where the given source and destination masks are both nonzero
template <typename S, typename D, bool ADD>
__global__ void __launch_bounds__(256) copy_masked_kernel(const DirectArgs p,
                                                          const float *__restrict__ smask,
                                                          const float *__restrict__ dmask) {
    const S *__restrict__ src = (const S *)p.src;
    D *__restrict__ dst = (D *)p.dstp;
    for (uint32_t idx = blockIdx.x * 256u + threadIdx.x; idx < p.total; idx += gridDim.x * 256u) {
        uint32_t rem = idx;
        long so = 0, doff = 0;
#pragma unroll
        for (int i = 0; i < MAXD; ++i) {
            if (i >= p.nd) break;
            const uint32_t q = p.size[i].div(rem);
            const uint32_t c = rem - q * p.size[i].d;
            rem = q;
            so += (long)c * p.sst[i];
            doff += (long)c * p.dst[i];
        }
        if ((smask && smask[so] == 0.f) || (dmask && dmask[doff] == 0.f)) continue;
        put<ADD, D>(dst + doff, xform<D, S>(src[so], p.alpha));
    }
}

// Contiguous copy of `total` elements (both sides dense); streaming stores when `nt`
template <typename S, typename D, bool ADD>
__global__ void __launch_bounds__(256) copy_contig_kernel(const S *__restrict__ src,
                                                           D *__restrict__ dst, long total,
                                                           Alpha alpha, int nt) {
    for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256L) {
        const D v = xform<D, S>(src[idx], alpha);
        if (!ADD && nt)
            store_nt(dst + idx, v);
        else
            put<ADD, D>(dst + idx, v);
    }
}

/// LDS tile capacity in elements: 24 KB of tile per workgroup whatever the element size
template <typename D> constexpr int tile_elems() { return (int)(24576 / sizeof(D)) > 3072 ? 3072 : (int)(24576 / sizeof(D)); }

struct TiledArgs {
    uint32_t R, TU, TV;     // run length, tile sizes (items)
    uint32_t NU, NV;        // extents of the U and V chains (flattened)
    FastDiv fR, fTU, fTV;   // divisors
    FastDiv fRTU, fRTV;     // R*TU, R*TV
    uint32_t ntu, ntv;      // number of tiles along U and V
    uint32_t lr, lw;        // log2 of the lanes per tile row in the read / write phase
    uint32_t lr2, lw2;      // ... for the paired (16-byte) forms of the phases
    int nt;                 // non-temporal stores
    int nu, nv;             // dims in the U chain (source-contiguous) / V chain (dest-contiguous)
    FastDiv usize[MAXD], vsize[MAXD];
    long usst[MAXD], udst[MAXD], vsst[MAXD], vdst[MAXD];
    int nw;                 // outer dims
    FastDiv wsize[MAXD];
    long wsst[MAXD], wdst[MAXD];
    const void *src;
    void *dstp;
    Alpha alpha;
};

/// Offsets of item `idx` of a chain of dims (fastest first), unrolled for short chains
__device__ __forceinline__ void chain_offsets4(uint32_t idx, int n, const FastDiv *size,
                                               const long *sst, const long *dst, long &so,
                                               long &doff) {
    so = 0;
    doff = 0;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
        if (i >= n) break;
        const uint32_t q = size[i].div(idx);
        const uint32_t c = idx - q * size[i].d;
        idx = q;
        so += (long)c * sst[i];
        doff += (long)c * dst[i];
    }
}

// Row-mapped single-pass form: in the read phase lane l of a wave owns the positions l, l+64, ...
// of a tile row (a source-contiguous run of R*TU elements) and the wave walks the rows v = wave,
// wave+4, ...; the write phase does the same over destination rows.  A lane's (u, r) split and
// offset base are computed once, so an element costs one LDS offset read (wave-uniform), one
// global access and one LDS access.  The u and v offset tables are filled by different waves.
// VR / VW = 2 (8-byte source / destination elements): the read / write phase moves two elements per lane
// (one 16-byte access): a tile row is then one contiguous, 16-byte aligned run of an even number
// of elements on that side (checked by the launcher), and the lane count per access halves
// (complex<float> transposes were bound by 8-byte lane accesses: chain redistribution 3.3 TB/s)
template <typename D> struct alignas(16) Pair { D a, b; };
template <typename S, typename D, bool ADD, int KR, int VR = 1, int VW = 1>
__global__ void __launch_bounds__(256) copy_tiled3_kernel(const TiledArgs p) {
    __shared__ D tile[tile_elems<D>() + 64];
    __shared__ long su[256], du[256], sv[256], dv[256];
    const S *__restrict__ src = (const S *)p.src;
    D *__restrict__ dst = (D *)p.dstp;
    uint32_t b = blockIdx.x;
    const uint32_t tu = b % p.ntu;
    b /= p.ntu;
    const uint32_t tv = b % p.ntv;
    uint32_t w = b / p.ntv;
    long sbase = 0, dbase = 0;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
        if (i >= p.nw) break;
        const uint32_t q = p.wsize[i].div(w);
        const uint32_t c = w - q * p.wsize[i].d;
        w = q;
        sbase += (long)c * p.wsst[i];
        dbase += (long)c * p.wdst[i];
    }
    const uint32_t u0 = tu * p.TU, v0 = tv * p.TV;
    const uint32_t nu_t = min(p.TU, p.NU - u0), nv_t = min(p.TV, p.NV - v0);
    const uint32_t t = threadIdx.x;
    if (t < 128) {
        if (t < nu_t) chain_offsets4(u0 + t, p.nu, p.usize, p.usst, p.udst, su[t], du[t]);
        if (t + 128 < nu_t) chain_offsets4(u0 + t + 128, p.nu, p.usize, p.usst, p.udst, su[t + 128], du[t + 128]);
    } else {
        const uint32_t v = t - 128;
        if (v < nv_t) chain_offsets4(v0 + v, p.nv, p.vsize, p.vsst, p.vdst, sv[v], dv[v]);
        if (v + 128 < nv_t) chain_offsets4(v0 + v + 128, p.nv, p.vsize, p.vsst, p.vdst, sv[v + 128], dv[v + 128]);
    }
    __syncthreads();
    const uint32_t lane = t & 63, wave = t >> 6;
    const uint32_t ld = p.TU * p.R + 1;
    // read phase: rows = v (nv_t of them), row width R*nu_t; 2^lr lanes per row, so a wave
    // covers 64 >> lr rows per step and a thread keeps KR rows' loads in flight
    if constexpr (VR == 2) {
        // pairs of a contiguous source run: element offset su[0] + pos in the row of v
        const uint32_t wr2 = p.R * nu_t / 2, lpr = 1u << p.lr2;
        const uint32_t step = 4u * (64u >> p.lr2);
        const uint32_t vfirst = wave * (64u >> p.lr2) + (lane >> p.lr2);
        for (uint32_t pp = lane & (lpr - 1); pp < wr2; pp += lpr) {
            const uint32_t pos = 2 * pp;
            const long base = sbase + su[0] + pos;
            for (uint32_t vb = vfirst; vb < nv_t; vb += step * KR) {
                Pair<S> val[KR];
#pragma unroll
                for (int k = 0; k < KR; ++k) {
                    const uint32_t v = vb + step * k;
                    val[k] = *(const Pair<S> *)(src + base + sv[v < nv_t ? v : vb]);
                }
#pragma unroll
                for (int k = 0; k < KR; ++k) {
                    const uint32_t v = vb + step * k;
                    if (v < nv_t) {
                        tile[v * ld + pos] = xform<D, S>(val[k].a, p.alpha);
                        tile[v * ld + pos + 1] = xform<D, S>(val[k].b, p.alpha);
                    }
                }
            }
        }
    } else {
        const uint32_t wr = p.R * nu_t, lpr = 1u << p.lr;
        const uint32_t step = 4u * (64u >> p.lr);
        const uint32_t vfirst = wave * (64u >> p.lr) + (lane >> p.lr);
        for (uint32_t pos = lane & (lpr - 1); pos < wr; pos += lpr) {
            const uint32_t u = p.fR.div(pos), r = pos - u * p.R;
            const long base = sbase + su[u] + r;
            for (uint32_t vb = vfirst; vb < nv_t; vb += step * KR) {
                D val[KR];
#pragma unroll
                for (int k = 0; k < KR; ++k) {
                    const uint32_t v = vb + step * k;
                    val[k] = xform<D, S>(src[base + sv[v < nv_t ? v : vb]], p.alpha);
                }
#pragma unroll
                for (int k = 0; k < KR; ++k) {
                    const uint32_t v = vb + step * k;
                    if (v < nv_t) tile[v * ld + pos] = val[k];
                }
            }
        }
    }
    __syncthreads();
    // write phase: rows = u (nu_t of them), row width R*nv_t
    if constexpr (VW == 2) {
        // pairs of a contiguous destination run: element offset dv[0] + pos in the row of u
        const uint32_t ww2 = p.R * nv_t / 2, lpr = 1u << p.lw2;
        const uint32_t step = 4u * (64u >> p.lw2);
        const uint32_t ufirst = wave * (64u >> p.lw2) + (lane >> p.lw2);
        for (uint32_t pp = lane & (lpr - 1); pp < ww2; pp += lpr) {
            const uint32_t pos = 2 * pp;
            const uint32_t va = p.fR.div(pos), ra = pos - va * p.R;
            const uint32_t vb = p.fR.div(pos + 1), rb = pos + 1 - vb * p.R;
            const long base = dbase + dv[0] + pos;
            const uint32_t la = va * ld + ra, lb = vb * ld + rb;
            for (uint32_t u = ufirst; u < nu_t; u += step) {
                const Pair<D> val{tile[la + u * p.R], tile[lb + u * p.R]};
                if (p.nt)
                    store_nt((Pair<D> *)(dst + base + du[u]), val);
                else
                    *(Pair<D> *)(dst + base + du[u]) = val;
            }
        }
        return;
    }
    {
        const uint32_t ww = p.R * nv_t, lpr = 1u << p.lw;
        const uint32_t step = 4u * (64u >> p.lw);
        const uint32_t ufirst = wave * (64u >> p.lw) + (lane >> p.lw);
        for (uint32_t pos = lane & (lpr - 1); pos < ww; pos += lpr) {
            const uint32_t v = p.fR.div(pos), r = pos - v * p.R;
            const long base = dbase + dv[v] + r;
            const uint32_t lb = v * ld + r;
            for (uint32_t u = ufirst; u < nu_t; u += step)
            {
                const D val = tile[lb + u * p.R];
                if (!ADD && p.nt)
                    store_nt(dst + base + du[u], val);
                else
                    put<ADD, D>(dst + base + du[u], val);
            }
        }
    }
}

// Site-block transpose (round 3): the copies whose source is one contiguous run over
// [R, the U chain, a dimension V1] and whose destination is contiguous over [R, V1] -- a transpose
// of V1 against the U chain in items of R elements, e.g. the config-2p permute xyztsc -> slice n
// of tnsxyzc (R = c, U = (s, t), V1 = xyz).  A workgroup takes QT items of V1 with ALL of U: its
// source is one contiguous run of QT*NU*R elements, loaded coalesced with every load of a thread
// in flight at once, transposed through LDS (one element of padding per V1 item) and written as
// NU runs of QT*R destination elements.  Against the general tile kernel (a tile row spans only
// part of U, offset tables per element, rows walked in several dependent rounds) the config-2p
// slice loop goes 5.2 -> 3.5 us per slice (tools/permute_micro.hip).
/// Destinations from this size are written with streaming (non-temporal) stores: written once,
/// not re-read by the kernel.  4 MB: the config-2p slice of complex<float> (6.3 MB written)
/// measured 3.68 -> 3.98-4.10 TB/s with them, and 4.7-6.3 MB block / tile copies 2-6 % faster
/// (tools/studies/copy_shapes.py COPY_MID); it was 8 MB.
constexpr long NT_MIN_BYTES = 4L << 20;
constexpr int TRANS_EMAX = 1536; // elements per tile
constexpr int TRANS_KMAX = TRANS_EMAX / 256;
/// block transpose tile (elements): 24 KB of 16-byte elements, 3072 smaller ones (12 per thread)
template <typename D> constexpr int btrans_emax() { return sizeof(D) >= 16 ? 1536 : 3072; }
struct TransArgs {
    uint32_t R, NU, QT, NV1;  // run, U chain items, V1 items per tile, V1 extent
    uint32_t ntv;             // tiles along V1
    FastDiv fNUR, fQTR, fR;   // NU*R, QT*R, R
    // thread strides of the two phases, as whole steps: 256 = qi*NU*R + ri (loads), 256 =
    // qo*QT*R + ro and ro = qr*R + rr (stores)
    uint32_t qi, ri, qo, ro, qr, rr;
    uint32_t qi2, ri2, qo2, ro2, qr2, rr2; // the same for 512 (paired phases)
    int pr, pw;                            // the planner allows paired reads / writes
    long ssv, dsv;            // V1 strides (source NU*R, destination R)
    int nu;                   // U chain dims (source order, fastest first)
    FastDiv usize[MAXD];
    long udst[MAXD];
    int nw;                   // outer dims
    FastDiv wsize[MAXD];
    long wsst[MAXD], wdst[MAXD];
    int nt;                   // non-temporal stores
    const void *src;
    void *dstp;
    Alpha alpha;
};

// A1: alpha == 1 (plain data movement, no scaling code); FULL (uniform per workgroup): the tile
// fills every thread's KMAX elements on both phases (no per-element guards); PR / PW (8-byte
// elements): the loads / stores move two consecutive elements per lane (one 16-byte access; the
// planner checks that the runs are even and their starts even, the launch that the pointers are
// 16-byte aligned)
template <typename S, typename D, bool ADD, bool A1, bool FULL, bool PR, bool PW>
__device__ __forceinline__ void trans_body(const TransArgs &p, D *tile, const long *du, const S *s0,
                                           D *d0, uint32_t qt, uint32_t E) {
    const uint32_t t = threadIdx.x, NUR = p.NU * p.R, LD = NUR + 1;
    constexpr int KR = PR ? TRANS_KMAX / 2 : TRANS_KMAX;
    constexpr uint32_t ER = PR ? 2 : 1; // elements per lane access
    S r[KR][ER];
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        const uint32_t j = ER * (t + 256 * k);
        if (FULL || j < E) {
            if constexpr (PR) {
                const Pair<S> v = *(const Pair<S> *)(s0 + j);
                r[k][0] = v.a;
                r[k][ER - 1] = v.b;
            } else {
                r[k][0] = s0[j];
            }
        }
    }
    // element j of the run sits at (item, e) = divmod(j, NU*R), stepped incrementally
    uint32_t item = p.fNUR.div(ER * t), e = ER * t - item * NUR;
#pragma unroll
    for (int k = 0; k < KR; ++k) {
        if (FULL || ER * (t + 256 * k) < E) {
#pragma unroll
            for (uint32_t h = 0; h < ER; ++h) {
                // the pair's second element: e + 1 < NU*R (NU*R even, e even)
                tile[item * LD + e + h] = A1 ? conv<D, S>(r[k][h]) : xform<D, S>(r[k][h], p.alpha);
            }
        }
        item += PR ? p.qi2 : p.qi;
        e += PR ? p.ri2 : p.ri;
        if (e >= NUR) {
            e -= NUR;
            ++item;
        }
    }
    __syncthreads();
    // the destination: for each U item a run of QT*R elements (items v0.. of V1, R each) at
    // d0 + du[u] + x (V1's destination stride is R); thread t writes positions EW*t, EW*(t + 256),
    // ... of the U-major order
    constexpr int KW = PW ? TRANS_KMAX / 2 : TRANS_KMAX;
    constexpr uint32_t EW = PW ? 2 : 1;
    const uint32_t QTR = p.QT * p.R;
    uint32_t u = p.fQTR.div(EW * t), x = EW * t - u * QTR;
    uint32_t it = p.fR.div(x), c = x - it * p.R;
#pragma unroll
    for (int k = 0; k < KW; ++k) {
        if (FULL || (u < p.NU && it < qt)) {
            D *q = d0 + du[u] + x;
            const D v0 = tile[it * LD + u * p.R + c];
            if constexpr (PW) {
                // the pair's second element: position x + 1 of the same U item (QT*R even)
                const uint32_t it1 = c + 1 == p.R ? it + 1 : it, c1 = c + 1 == p.R ? 0 : c + 1;
                if (FULL || it1 < qt) {
                    const Pair<D> v{v0, tile[it1 * LD + u * p.R + c1]};
                    if (p.nt)
                        store_nt((Pair<D> *)q, v);
                    else
                        *(Pair<D> *)q = v;
                } else if (p.nt) {
                    store_nt(q, v0);
                } else {
                    *q = v0;
                }
            } else if (!ADD && p.nt) {
                store_nt(q, v0);
            } else {
                put<ADD, D>(q, v0);
            }
        }
        u += PW ? p.qo2 : p.qo;
        x += PW ? p.ro2 : p.ro;
        it += PW ? p.qr2 : p.qr;
        c += PW ? p.rr2 : p.rr;
        if (c >= p.R) {
            c -= p.R;
            ++it;
        }
        if (x >= QTR) {
            x -= QTR;
            it -= p.QT;
            ++u;
        }
    }
}

template <typename S, typename D, bool ADD, bool A1, bool PR, bool PW>
__global__ void __launch_bounds__(256) copy_trans_kernel(const TransArgs p) {
    __shared__ D tile[TRANS_EMAX + 256];
    __shared__ long du[256];
    uint32_t b = blockIdx.x;
    const uint32_t tv = b % p.ntv;
    uint32_t w = b / p.ntv;
    long sbase = 0, dbase = 0;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
        if (i >= p.nw) break;
        const uint32_t q = p.wsize[i].div(w);
        const uint32_t c = w - q * p.wsize[i].d;
        w = q;
        sbase += (long)c * p.wsst[i];
        dbase += (long)c * p.wdst[i];
    }
    const uint32_t t = threadIdx.x, v0 = tv * p.QT;
    const uint32_t qt = min(p.QT, p.NV1 - v0), E = qt * p.NU * p.R;
    if (t < p.NU) {
        // destination offset of U item t (the U chain's dims, fastest first)
        uint32_t idx = t;
        long o = 0;
#pragma unroll
        for (int i = 0; i < MAXD; ++i) {
            if (i >= p.nu) break;
            const uint32_t q = p.usize[i].div(idx);
            o += (long)(idx - q * p.usize[i].d) * p.udst[i];
            idx = q;
        }
        du[t] = o;
    }
    // the tile's source: one contiguous run of E elements
    const S *s0 = (const S *)p.src + sbase + (long)v0 * p.ssv;
    D *d0 = (D *)p.dstp + dbase + (long)v0 * p.dsv;
    if (E == 256 * TRANS_KMAX && p.NU * p.QT * p.R == 256 * TRANS_KMAX)
        trans_body<S, D, ADD, A1, true, PR, PW>(p, tile, du, s0, d0, qt, E);
    else
        trans_body<S, D, ADD, A1, false, PR, PW>(p, tile, du, s0, d0, qt, E);
}

// Block transpose (round 3): a tile of QT items of a dimension V1 with all NU items of a set U
// of dims, U = SI + SO = DI + DO where SI (DI) are the dims contiguous in the source (destination)
// from the run R: the source holds runs of R*|SI| elements (longer when V1 follows SI), the
// destination runs of R*|DI| elements (longer when V1 follows DI).  Loads walk the source order
// (run, V1, SO), stores the destination order (run, V1, DO); the LDS tile is [V1 item][U item in
// source order][R] and a table maps a destination-order U item to it.  Covers the three-way
// transposes the site-block kernel does not (the chain's tnsxyzc -> pxyztscn: V1 = xyz, SI = c,
// DI = (n, c, s)).  Every index is stepped incrementally (mixed-radix digits, 256 per step).
struct BtransArgs {
    uint32_t R, NU, QT, NV1, ntv;
    uint32_t RS, NSO, RD, NDI, NDO; // source run R*|SI|, SO items; destination run R*|DI|, DI / DO items
    long ssv, dsv;                  // V1 strides
    uint32_t la, lv, lo;            // 256 in the load radix (RS, QT, NSO)
    uint32_t sr, sd, sv, so;        // 256 in the store radix (R, NDI, QT, NDO)
    uint32_t sr2, sd2, sv2, so2;    // 512 in the store radix (paired stores)
    int pw;                         // the planner allows paired stores (8-byte elements)
    int nso, ndo, nud;
    FastDiv sosize[MAXD], dosize[MAXD], udsize[MAXD];
    long sost[MAXD], dost[MAXD];
    uint32_t ucmul[MAXD];           // U dims in destination order (DI then DO): canonical multipliers
    int nw;
    FastDiv wsize[MAXD];
    long wsst[MAXD], wdst[MAXD];
    int nt;
    const void *src;
    void *dstp;
    Alpha alpha;
};

template <typename S, typename D, bool ADD, bool A1, bool PW>
__global__ void __launch_bounds__(256) copy_btrans_kernel(const BtransArgs p) {
    constexpr int BE = btrans_emax<D>(), BK = BE / 256;
    __shared__ D tile[BE + 256];
    __shared__ long so_off[256], do_off[256];
    __shared__ uint16_t ucan[256];
    uint32_t b = blockIdx.x;
    const uint32_t tv = b % p.ntv;
    uint32_t w = b / p.ntv;
    long sbase = 0, dbase = 0;
#pragma unroll
    for (int i = 0; i < MAXD; ++i) {
        if (i >= p.nw) break;
        const uint32_t q = p.wsize[i].div(w);
        const uint32_t c = w - q * p.wsize[i].d;
        w = q;
        sbase += (long)c * p.wsst[i];
        dbase += (long)c * p.wdst[i];
    }
    const uint32_t t = threadIdx.x, v0 = tv * p.QT;
    const uint32_t qt = min(p.QT, p.NV1 - v0);
    if (t < p.NSO) {
        uint32_t idx = t;
        long o = 0;
#pragma unroll
        for (int i = 0; i < MAXD; ++i) {
            if (i >= p.nso) break;
            const uint32_t q = p.sosize[i].div(idx);
            o += (long)(idx - q * p.sosize[i].d) * p.sost[i];
            idx = q;
        }
        so_off[t] = o;
    }
    if (t < p.NDO) {
        uint32_t idx = t;
        long o = 0;
#pragma unroll
        for (int i = 0; i < MAXD; ++i) {
            if (i >= p.ndo) break;
            const uint32_t q = p.dosize[i].div(idx);
            o += (long)(idx - q * p.dosize[i].d) * p.dost[i];
            idx = q;
        }
        do_off[t] = o;
    }
    if (t < p.NU) {
        uint32_t idx = t, uc = 0;
#pragma unroll
        for (int i = 0; i < MAXD; ++i) {
            if (i >= p.nud) break;
            const uint32_t q = p.udsize[i].div(idx);
            uc += (idx - q * p.udsize[i].d) * p.ucmul[i];
            idx = q;
        }
        ucan[t] = (uint16_t)uc;
    }
    __syncthreads();
    const S *s0 = (const S *)p.src + sbase + (long)v0 * p.ssv;
    D *d0 = (D *)p.dstp + dbase + (long)v0 * p.dsv;
    const uint32_t LD = p.NU * p.R + 1, E = p.RS * p.QT * p.NSO;
    // loads in the source order (a in the run, v, so); every load of a thread in flight at once
    S r[BK];
    {
        uint32_t a = t, v = 0, o = 0;
        // t < 256: its digits (a, v, o) by two divisions, then the step carries
        v = p.RS > t ? 0 : t / p.RS;
        a = t - v * p.RS;
        o = v / p.QT;
        v -= o * p.QT;
        const uint32_t a0 = a, v0_ = v, o0 = o;
#pragma unroll
        for (int k = 0; k < BK; ++k) {
            if (t + 256 * k < E && v < qt) r[k] = s0[a + (long)v * p.ssv + so_off[o < p.NSO ? o : 0]];
            a += p.la;
            v += p.lv;
            o += p.lo;
            if (a >= p.RS) {
                a -= p.RS;
                ++v;
            }
            if (v >= p.QT) {
                v -= p.QT;
                ++o;
            }
        }
        a = a0;
        v = v0_;
        o = o0;
#pragma unroll
        for (int k = 0; k < BK; ++k) {
            if (t + 256 * k < E && v < qt)
                tile[v * LD + o * p.RS + a] = A1 ? conv<D, S>(r[k]) : xform<D, S>(r[k], p.alpha);
            a += p.la;
            v += p.lv;
            o += p.lo;
            if (a >= p.RS) {
                a -= p.RS;
                ++v;
            }
            if (v >= p.QT) {
                v -= p.QT;
                ++o;
            }
        }
    }
    __syncthreads();
    // PW (8-byte elements, even destination runs, 16-byte aligned): two consecutive positions per
    // lane, one 16-byte store (the second element is in the same run: runs and starts are even)
    if constexpr (PW) {
        const uint32_t t2 = 2 * t;
        uint32_t x = t2 / p.R, c = t2 - x * p.R;
        uint32_t v = x / p.NDI, di = x - v * p.NDI;
        uint32_t o = v / p.QT;
        v -= o * p.QT;
        const uint32_t ES = p.RD * p.QT * p.NDO;
#pragma unroll
        for (int k = 0; k < BK / 2; ++k) {
            if (t2 + 512 * k < ES && v < qt) {
                uint32_t c1 = c + 1, di1 = di;
                if (c1 == p.R) {
                    c1 = 0;
                    ++di1;
                }
                const Pair<D> val{tile[v * LD + ucan[o * p.NDI + di] * p.R + c],
                                  tile[v * LD + ucan[o * p.NDI + di1] * p.R + c1]};
                Pair<D> *q = (Pair<D> *)(d0 + (di * p.R + c) + (long)v * p.dsv + do_off[o]);
                if (p.nt)
                    store_nt(q, val);
                else
                    *q = val;
            }
            c += p.sr2;
            di += p.sd2;
            v += p.sv2;
            o += p.so2;
            if (c >= p.R) {
                c -= p.R;
                ++di;
            }
            if (di >= p.NDI) {
                di -= p.NDI;
                ++v;
            }
            if (v >= p.QT) {
                v -= p.QT;
                ++o;
            }
        }
        return;
    }
    // stores in the destination order (c in R, di, v, do)
    {
        uint32_t x = t / p.R, c = t - x * p.R;
        uint32_t v = x / p.NDI, di = x - v * p.NDI;
        uint32_t o = v / p.QT;
        v -= o * p.QT;
        const uint32_t ES = p.RD * p.QT * p.NDO;
#pragma unroll
        for (int k = 0; k < BK; ++k) {
            if (t + 256 * k < ES && v < qt) {
                const uint32_t uc = ucan[o * p.NDI + di];
                const D val = tile[v * LD + uc * p.R + c];
                D *q = d0 + (di * p.R + c) + (long)v * p.dsv + do_off[o];
                if (!ADD && p.nt)
                    store_nt(q, val);
                else
                    put<ADD, D>(q, val);
            }
            c += p.sr;
            di += p.sd;
            v += p.sv;
            o += p.so;
            if (c >= p.R) {
                c -= p.R;
                ++di;
            }
            if (di >= p.NDI) {
                di -= p.NDI;
                ++v;
            }
            if (v >= p.QT) {
                v -= p.QT;
                ++o;
            }
        }
    }
}

template <typename T> struct DT;
template <> struct DT<float> { static constexpr int v = SBX_FLOAT; };
template <> struct DT<double> { static constexpr int v = SBX_DOUBLE; };
template <> struct DT<float2> { static constexpr int v = SBX_CFLOAT; };
template <> struct DT<double2> { static constexpr int v = SBX_CDOUBLE; };
template <> struct DT<int> { static constexpr int v = SBX_INT; };
template <> struct DT<unsigned long> { static constexpr int v = SBX_SIZE_T; };

struct Norm {
    std::vector<long> size, ss, ds;
};

Norm normalize(const BoxCopyDesc &d) {
    Norm n;
    const std::size_t nd = d.size.size();
    std::vector<int> idx;
    for (std::size_t i = 0; i < nd; ++i)
        if (d.size[i] != 1) idx.push_back((int)i);
    std::stable_sort(idx.begin(), idx.end(), [&](int a, int b) {
        if (d.dst_stride[a] != d.dst_stride[b]) return d.dst_stride[a] < d.dst_stride[b];
        return d.src_stride[a] < d.src_stride[b];
    });
    for (int i : idx) {
        if (!n.size.empty()) {
            const long s = n.size.back();
            if (n.ss.back() * s == d.src_stride[i] && n.ds.back() * s == d.dst_stride[i]) {
                n.size.back() *= d.size[i];
                continue;
            }
        }
        n.size.push_back(d.size[i]);
        n.ss.push_back(d.src_stride[i]);
        n.ds.push_back(d.dst_stride[i]);
    }
    if (n.size.empty()) {
        n.size.push_back(1);
        n.ss.push_back(1);
        n.ds.push_back(1);
    }
    return n;
}

/// A prepared box-copy launch: everything but the pointers and alpha, which are patched per call
/// (the launch cache below keys it on the box shape, element types and tuning switches; the
/// reference caches its permutation index vectors the same way, tensor.h:919-961)
struct CopyLaunch {
    enum Kind { MASKED, CONTIG, DIRECT, TILED3, TRANS, BTRANS } kind = DIRECT;
    DirectArgs da{};
    TiledArgs ta{};
    TransArgs tr{};
    BtransArgs bt{};
    long total = 0, blocks = 0;
    int nt = 0;
    int vr = 0, vw = 0; // tiled: the shape allows paired reads / writes (pointers checked per call)
    void (*run)(const CopyLaunch &, const void *, void *, const Alpha &, const float *,
                const float *, hipStream_t) = nullptr;
};

template <typename S, typename D, bool ADD>
void run_launch(const CopyLaunch &l, const void *src, void *dst, const Alpha &alpha,
                const float *smask, const float *dmask, hipStream_t stream) {
    KernelTimer timer("copy", stream);
    const dim3 grid((unsigned)l.blocks), block(256);
    g_copy_tune.last_pair = 0;
    switch (l.kind) {
    case CopyLaunch::MASKED: {
        DirectArgs a = l.da;
        a.src = src;
        a.dstp = dst;
        a.alpha = alpha;
        hipLaunchKernelGGL((copy_masked_kernel<S, D, ADD>), grid, block, 0, stream, a, smask, dmask);
        break;
    }
    case CopyLaunch::CONTIG:
        hipLaunchKernelGGL((copy_contig_kernel<S, D, ADD>), grid, block, 0, stream, (const S *)src,
                           (D *)dst, l.total, alpha, l.nt);
        break;
    case CopyLaunch::DIRECT: {
        DirectArgs a = l.da;
        a.src = src;
        a.dstp = dst;
        a.alpha = alpha;
        hipLaunchKernelGGL((copy_direct_kernel<S, D, ADD>), grid, block, 0, stream, a);
        break;
    }
    case CopyLaunch::TRANS: {
        TransArgs a = l.tr;
        a.src = src;
        a.dstp = dst;
        a.alpha = alpha;
        const bool pr = a.pr && ((size_t)src & 15) == 0, pw = a.pw && ((size_t)dst & 15) == 0;
        g_copy_tune.last_pair = 4 | (pr ? 1 : 0) | (pw ? 2 : 0);
        auto go = [&](auto a1, auto pr_, auto pw_) {
            hipLaunchKernelGGL((copy_trans_kernel<S, D, ADD, decltype(a1)::value, decltype(pr_)::value,
                                                  decltype(pw_)::value>),
                               grid, block, 0, stream, a);
        };
        using T_ = std::true_type;
        using F_ = std::false_type;
        constexpr bool CR = sizeof(S) == 8, CW = sizeof(D) == 8 && !ADD;
        if (alpha.one == 1) {
            if constexpr (CR && CW) {
                if (pr && pw) { go(T_{}, T_{}, T_{}); break; }
            }
            if constexpr (CR) {
                if (pr) { go(T_{}, T_{}, F_{}); break; }
            }
            if constexpr (CW) {
                if (pw) { go(T_{}, F_{}, T_{}); break; }
            }
            go(T_{}, F_{}, F_{});
        } else {
            if constexpr (CR && CW) {
                if (pr && pw) { go(F_{}, T_{}, T_{}); break; }
            }
            if constexpr (CR) {
                if (pr) { go(F_{}, T_{}, F_{}); break; }
            }
            if constexpr (CW) {
                if (pw) { go(F_{}, F_{}, T_{}); break; }
            }
            go(F_{}, F_{}, F_{});
        }
        break;
    }
    case CopyLaunch::BTRANS: {
        BtransArgs a = l.bt;
        a.src = src;
        a.dstp = dst;
        a.alpha = alpha;
        constexpr bool CW = sizeof(D) == 8 && !ADD;
        const bool pw = CW && a.pw && ((size_t)dst & 15) == 0;
        g_copy_tune.last_pair = 8 | (pw ? 2 : 0);
        if (alpha.one == 1) {
            if constexpr (CW) {
                if (pw) {
                    hipLaunchKernelGGL((copy_btrans_kernel<S, D, ADD, true, CW>), grid, block, 0, stream, a);
                    break;
                }
            }
            hipLaunchKernelGGL((copy_btrans_kernel<S, D, ADD, true, false>), grid, block, 0, stream, a);
        } else {
            if constexpr (CW) {
                if (pw) {
                    hipLaunchKernelGGL((copy_btrans_kernel<S, D, ADD, false, CW>), grid, block, 0, stream, a);
                    break;
                }
            }
            hipLaunchKernelGGL((copy_btrans_kernel<S, D, ADD, false, false>), grid, block, 0, stream, a);
        }
        break;
    }
    case CopyLaunch::TILED3: {
        g_copy_tune.last_pair = 0;
        TiledArgs a = l.ta;
        a.src = src;
        a.dstp = dst;
        a.alpha = alpha;
        constexpr bool PS = sizeof(S) == 8, PD = sizeof(D) == 8 && !ADD;
        if constexpr (PS || PD) {
            const bool vr = PS && l.vr && ((size_t)src & 15) == 0;
            const bool vw = PD && l.vw && ((size_t)dst & 15) == 0;
            g_copy_tune.last_pair = (vr ? 1 : 0) | (vw ? 2 : 0);
            if constexpr (PS && PD) {
                if (vr && vw) {
                    hipLaunchKernelGGL((copy_tiled3_kernel<S, D, ADD, 4, 2, 2>), grid, block, 0, stream, a);
                    break;
                }
            }
            if constexpr (PS) {
                if (vr) {
                    hipLaunchKernelGGL((copy_tiled3_kernel<S, D, ADD, 4, 2, 1>), grid, block, 0, stream, a);
                    break;
                }
            }
            if constexpr (PD) {
                if (vw) {
                    hipLaunchKernelGGL((copy_tiled3_kernel<S, D, ADD, 4, 1, 2>), grid, block, 0, stream, a);
                    break;
                }
            }
            hipLaunchKernelGGL((copy_tiled3_kernel<S, D, ADD, 4>), grid, block, 0, stream, a);
        } else {
            hipLaunchKernelGGL((copy_tiled3_kernel<S, D, ADD, 4>), grid, block, 0, stream, a);
        }
        break;
    }
    }
    SBX_HIP_CHECK(hipGetLastError());
}

/// The site-block transpose (copy_trans_kernel) when the normalised box has the shape it takes:
/// a dim V1 of destination stride R whose source stride is R * NU, NU the product of a chain of
/// dims whose source strides run R, R*u0, ... up to it (the U chain; at most 256 items and at
/// least two V1 items per tile)
constexpr long BTRANS_MIN_RUN = 128; // bytes: the shortest run either transpose kernel takes
template <typename S, typename D, bool ADD>
bool prepare_trans(CopyLaunch &l, const Norm &n, int first, long R, long total) {
    const int nd = (int)n.size.size();
    int v1 = -1;
    for (int i = first; i < nd; ++i)
        if (n.ds[i] == R && n.size[i] > 1) v1 = i;
    if (v1 < 0 || n.ss[v1] % R) return false;
    const long NU = n.ss[v1] / R;
    if (NU < 2 || NU > 256 || NU * R * 2 > TRANS_EMAX) return false;
    std::vector<bool> used(nd, false);
    for (int i = 0; i < first; ++i) used[i] = true;
    used[v1] = true;
    std::vector<int> U;
    long want = R;
    while (want < n.ss[v1]) {
        int f = -1;
        for (int i = first; i < nd; ++i)
            if (!used[i] && n.ss[i] == want) f = i;
        if (f < 0) return false;
        U.push_back(f);
        used[f] = true;
        want *= n.size[f];
    }
    if (want != n.ss[v1] || (int)U.size() > MAXD) return false;
    TransArgs &a = l.tr;
    // (at most 256 items: the tile's padding, one element per item, must fit its 256 spare slots)
    const long QT = std::min({n.size[v1], 256L, (long)TRANS_EMAX / (NU * R)});
    if (QT * (NU * R + 1) > TRANS_EMAX + 256) throw Error("copy: internal transpose tile sizing error");
    // destination runs of QT*R elements: at least BTRANS_MIN_RUN bytes (a 3-item V1 against a
    // 12-item U measured 10x slower than the tile kernel)
    if (QT * R * (long)sizeof(D) < BTRANS_MIN_RUN) return false;
    a.R = (uint32_t)R;
    a.NU = (uint32_t)NU;
    a.QT = (uint32_t)QT;
    a.NV1 = (uint32_t)n.size[v1];
    a.ntv = (uint32_t)((n.size[v1] + QT - 1) / QT);
    a.fNUR = FastDiv((uint32_t)(NU * R));
    a.fQTR = FastDiv((uint32_t)(QT * R));
    a.fR = FastDiv((uint32_t)R);
    a.qi = (uint32_t)(256 / (NU * R));
    a.ri = (uint32_t)(256 % (NU * R));
    a.qo = (uint32_t)(256 / (QT * R));
    a.ro = (uint32_t)(256 % (QT * R));
    a.qr = a.ro / (uint32_t)R;
    a.rr = a.ro % (uint32_t)R;
    a.qi2 = (uint32_t)(512 / (NU * R));
    a.ri2 = (uint32_t)(512 % (NU * R));
    a.qo2 = (uint32_t)(512 / (QT * R));
    a.ro2 = (uint32_t)(512 % (QT * R));
    a.qr2 = a.ro2 / (uint32_t)R;
    a.rr2 = a.ro2 % (uint32_t)R;
    a.ssv = n.ss[v1];
    a.dsv = n.ds[v1];
    a.nu = (int)U.size();
    for (std::size_t k = 0; k < U.size(); ++k) {
        a.usize[k] = FastDiv((uint32_t)n.size[U[k]]);
        a.udst[k] = n.ds[U[k]];
    }
    long NW = 1;
    int nw = 0;
    for (int i = first; i < nd; ++i) {
        if (used[i]) continue;
        if (nw == MAXD) return false;
        a.wsize[nw] = FastDiv((uint32_t)n.size[i]);
        a.wsst[nw] = n.ss[i];
        a.wdst[nw] = n.ds[i];
        NW *= n.size[i];
        ++nw;
    }
    a.nw = nw;
    a.nt = g_copy_tune.nt > 0 || (g_copy_tune.nt == 0 && total * (long)sizeof(D) >= NT_MIN_BYTES);
    // paired 16-byte accesses for 8-byte elements: even runs with even starts on that side
    bool ws_even = true, wd_even = true, ud_even = true;
    for (int i = 0; i < nw; ++i) {
        ws_even = ws_even && a.wsst[i] % 2 == 0;
        wd_even = wd_even && a.wdst[i] % 2 == 0;
    }
    for (int k = 0; k < a.nu; ++k) ud_even = ud_even && a.udst[k] % 2 == 0;
    // (a 16-byte destination element: single reads measured faster, cf2cd 4.83 -> 5.01 TB/s)
    a.pr = sizeof(S) == 8 && sizeof(D) == 8 && g_copy_tune.pair >= 0 && (NU * R) % 2 == 0 && ws_even;
    a.pw = sizeof(D) == 8 && !ADD && g_copy_tune.pair >= 0 && (QT * R) % 2 == 0 && ud_even && wd_even;
    const long blocks = (long)a.ntv * NW;
    if (blocks >= (1L << 31)) return false;
    l.kind = CopyLaunch::TRANS;
    l.blocks = blocks;
    static const bool debug = getenv("SBX_COPY_DEBUG") != nullptr;
    if (debug)
        std::fprintf(stderr, "copy_trans: R=%ld NU=%ld V1=%ld QT=%ld nu=%d nw=%d blocks=%ld\n", R, NU,
                     n.size[v1], QT, a.nu, nw, blocks);
    return true;
}

/// The block transpose (copy_btrans_kernel): over every choice of V1, U = the source chain SI
/// and the destination chain DI from the run R (at most 256 items, the source and destination
/// runs as long as possible); taken when both runs reach `BTRANS_MIN_RUN` bytes
template <typename S, typename D, bool ADD>
bool prepare_btrans(CopyLaunch &l, const Norm &n0, int first, long R, long total) {
    struct Plan {
        Norm n;
        int v1 = -1;
        std::vector<int> si, di;
        long score = 0;
    } best;
    constexpr long EMAX = btrans_emax<D>();
    const long cap0 = std::min(256L, EMAX / (2 * R));
    // (runs too long for two items per tile: nothing to transpose here -- and cap0 = 0 would never
    // end the halving loop below, which hung the chain's halo copies with 4.6K-element runs)
    if (cap0 < 2) return false;
    // V1 items per tile: as many as fit, rounded so that runs continuing over V1 (source first)
    // are whole 128-B lines (the chain redistribution's 240-B source runs read 1.47x their bytes)
    auto qt_of = [&](long nv1, long NU, long rs, long ssv, long rd, long dsv) {
        long QT = std::min(nv1, std::min(256L, EMAX / (NU * R)));
        auto round_to = [&](long run_bytes) {
            const long qa = 128 / std::gcd(run_bytes, 128L);
            if (QT >= qa && QT < nv1) QT = QT / qa * qa;
        };
        if (ssv == rs) round_to(rs * (long)sizeof(S));
        else if (dsv == rd) round_to(rd * (long)sizeof(D));
        return QT;
    };
    const int nd0 = (int)n0.size.size();
    // chain caps: whole dims first, then (16-byte elements) inner factors of a dim (split) so
    // that a tile holds more V1 items -- longer runs on V1's side (the whole-tensor complex<double>
    // permute 335 -> 310 us); for smaller elements the split plans measured slower than the tile
    // kernel's paired accesses (profiles/r03_copy_btrans.txt)
    const long cap_min = std::max(2L, sizeof(D) >= 16 ? 8L : cap0);
    for (long cap = cap0; cap >= cap_min; cap /= 2)
    for (int v1 = first; v1 < nd0; ++v1) {
        if (n0.size[v1] < 2) continue;
        Norm n = n0;
        // `other`: the chain built before this one; a dim of it may be split here only when it is
        // that chain's last dim (splitting an inner one would break its run of strides)
        auto chain = [&](bool dst_side, std::vector<int> &c, std::vector<bool> &used,
                         const std::vector<int> *other) {
            long want = R, prod = 1;
            while ((int)n.size.size() <= MAXD) {
                int f = -1;
                for (int i = first; i < (int)n.size.size(); ++i)
                    if (!used[i] && (dst_side ? n.ds[i] : n.ss[i]) == want && n.size[i] > 1) f = i;
                if (f < 0) break;
                if (prod * n.size[f] > cap) {
                    if (sizeof(D) < 16) break; // (no split plans for smaller elements, above)
                    if (other && std::find(other->begin(), other->end(), f) != other->end() &&
                        other->back() != f)
                        break;
                    long d = 1; // the largest inner factor that fits
                    for (long q = 2; q <= cap / prod; ++q)
                        if (n.size[f] % q == 0) d = q;
                    if (d < 2) break;
                    n.size.push_back(n.size[f] / d);
                    n.ss.push_back(n.ss[f] * d);
                    n.ds.push_back(n.ds[f] * d);
                    n.size[f] = d;
                    used.push_back(false);
                }
                c.push_back(f);
                used[f] = true;
                prod *= n.size[f];
                want *= n.size[f];
                if (prod >= cap) break;
            }
        };
        std::vector<int> si, di;
        std::vector<bool> us(n.size.size(), false), ud(n.size.size(), false);
        us[v1] = ud[v1] = true;
        chain(false, si, us, nullptr);
        ud.resize(n.size.size(), false);
        chain(true, di, ud, &si);
        const int nd = (int)n.size.size();
        if (nd > MAXD) continue;
        // both chains must still be runs: strides R, R*s0, R*s0*s1, ... on their side (a split
        // made by the later chain changes the sizes the earlier one was built from)
        auto is_run = [&](const std::vector<int> &c, const std::vector<long> &st) {
            long want = R;
            for (int i : c) {
                if (st[i] != want) return false;
                want *= n.size[i];
            }
            return true;
        };
        if (!is_run(si, n.ss) || !is_run(di, n.ds)) continue;
        auto nu_of = [&]() {
            std::vector<bool> in(nd, false);
            long nu = 1;
            for (int i : si) in[i] = true;
            for (int i : di) in[i] = true;
            for (int i = 0; i < nd; ++i)
                if (in[i]) nu *= n.size[i];
            return nu;
        };
        // too many U items: drop the outermost dim of the longer chain (it becomes an outer dim)
        while (nu_of() > cap0 && !(si.empty() && di.empty())) {
            long ps = 1, pd = 1;
            for (int i : si) ps *= n.size[i];
            for (int i : di) pd *= n.size[i];
            if (ps >= pd) si.pop_back();
            else di.pop_back();
        }
        const long NU = nu_of();
        if (NU < 2 || NU > cap0) continue;
        long rs = R, rd = R;
        for (int i : si) rs *= n.size[i];
        for (int i : di) rd *= n.size[i];
        const long QT = qt_of(n.size[v1], NU, rs, n.ss[v1], rd, n.ds[v1]);
        const long srun = n.ss[v1] == rs ? rs * QT : rs, drun = n.ds[v1] == rd ? rd * QT : rd;
        const long score = std::min(srun * (long)sizeof(S), drun * (long)sizeof(D));
        if (score > best.score) {
            best.n = n;
            best.v1 = v1;
            best.si = si;
            best.di = di;
            best.score = score;
        }
    }
    if (best.v1 < 0 || best.score < BTRANS_MIN_RUN) return false;
    const Norm &n = best.n;
    const int nd = (int)n.size.size();
    const int v1 = best.v1;
    std::vector<bool> inU(nd, false), inSI(nd, false), inDI(nd, false);
    for (int i : best.si) inU[i] = inSI[i] = true;
    for (int i : best.di) inU[i] = inDI[i] = true;
    // SO / DO: the rest of U, by source / destination stride
    std::vector<int> so, dO;
    for (int i = first; i < nd; ++i) {
        if (inU[i] && !inSI[i]) so.push_back(i);
        if (inU[i] && !inDI[i]) dO.push_back(i);
    }
    std::sort(so.begin(), so.end(), [&](int a, int b) { return n.ss[a] < n.ss[b]; });
    std::sort(dO.begin(), dO.end(), [&](int a, int b) { return n.ds[a] < n.ds[b]; });
    if ((int)so.size() > MAXD || (int)dO.size() > MAXD || (int)(best.di.size() + dO.size()) > MAXD)
        return false;
    BtransArgs &a = l.bt;
    long NU = 1, NSI = 1, NSO = 1, NDI = 1, NDO = 1;
    for (int i = 0; i < nd; ++i)
        if (inU[i]) NU *= n.size[i];
    for (int i : best.si) NSI *= n.size[i];
    for (int i : so) NSO *= n.size[i];
    for (int i : best.di) NDI *= n.size[i];
    for (int i : dO) NDO *= n.size[i];
    const long QT = qt_of(n.size[v1], NU, R * NSI, n.ss[v1], R * NDI, n.ds[v1]);
    if (QT > 256 || QT * (NU * R + 1) > EMAX + 256) throw Error("copy: internal block transpose tile sizing error");
    a.R = (uint32_t)R;
    a.NU = (uint32_t)NU;
    a.QT = (uint32_t)QT;
    a.NV1 = (uint32_t)n.size[v1];
    a.ntv = (uint32_t)((n.size[v1] + QT - 1) / QT);
    a.RS = (uint32_t)(R * NSI);
    a.NSO = (uint32_t)NSO;
    a.RD = (uint32_t)(R * NDI);
    a.NDI = (uint32_t)NDI;
    a.NDO = (uint32_t)NDO;
    a.ssv = n.ss[v1];
    a.dsv = n.ds[v1];
    {
        const long q1 = 256 / (R * NSI);
        a.la = (uint32_t)(256 % (R * NSI));
        a.lv = (uint32_t)(q1 % QT);
        a.lo = (uint32_t)(q1 / QT);
        const long p1 = 256 / R, p2 = p1 / NDI;
        a.sr = (uint32_t)(256 % R);
        a.sd = (uint32_t)(p1 % NDI);
        a.sv = (uint32_t)(p2 % QT);
        a.so = (uint32_t)(p2 / QT);
        const long e1 = 512 / R, e2 = e1 / NDI;
        a.sr2 = (uint32_t)(512 % R);
        a.sd2 = (uint32_t)(e1 % NDI);
        a.sv2 = (uint32_t)(e2 % QT);
        a.so2 = (uint32_t)(e2 / QT);
    }
    a.nso = (int)so.size();
    for (std::size_t k = 0; k < so.size(); ++k) {
        a.sosize[k] = FastDiv((uint32_t)n.size[so[k]]);
        a.sost[k] = n.ss[so[k]];
    }
    a.ndo = (int)dO.size();
    for (std::size_t k = 0; k < dO.size(); ++k) {
        a.dosize[k] = FastDiv((uint32_t)n.size[dO[k]]);
        a.dost[k] = n.ds[dO[k]];
    }
    // canonical U index = SI digits (fastest first) then SO digits; its multiplier per dim
    std::vector<long> cmul(nd, 0);
    {
        long m = 1;
        for (int i : best.si) {
            cmul[i] = m;
            m *= n.size[i];
        }
        for (int i : so) {
            cmul[i] = m;
            m *= n.size[i];
        }
    }
    std::vector<int> ud = best.di;
    ud.insert(ud.end(), dO.begin(), dO.end());
    a.nud = (int)ud.size();
    for (std::size_t k = 0; k < ud.size(); ++k) {
        a.udsize[k] = FastDiv((uint32_t)n.size[ud[k]]);
        a.ucmul[k] = (uint32_t)cmul[ud[k]];
    }
    long NW = 1;
    int nw = 0;
    for (int i = first; i < nd; ++i) {
        if (inU[i] || i == v1) continue;
        if (nw == MAXD) return false;
        a.wsize[nw] = FastDiv((uint32_t)n.size[i]);
        a.wsst[nw] = n.ss[i];
        a.wdst[nw] = n.ds[i];
        NW *= n.size[i];
        ++nw;
    }
    a.nw = nw;
    a.nt = g_copy_tune.nt > 0 || (g_copy_tune.nt == 0 && total * (long)sizeof(D) >= NT_MIN_BYTES);
    // paired stores: even destination runs whose starts are even (V1, DO and outer strides)
    bool d_even = a.RD % 2 == 0 && a.dsv % 2 == 0;
    for (int k = 0; k < a.ndo; ++k) d_even = d_even && a.dost[k] % 2 == 0;
    for (int k = 0; k < nw; ++k) d_even = d_even && a.wdst[k] % 2 == 0;
    a.pw = sizeof(D) == 8 && !ADD && g_copy_tune.pair >= 0 && d_even;
    // 8-byte destinations without paired stores: the tile kernel's paired accesses measured
    // faster (the chain's operand reorder pXYZTSCn -> TSnpXYZC, odd runs: 121 vs 116 us)
    if (sizeof(D) == 8 && !a.pw && g_copy_tune.pair >= 0 && g_copy_tune.btrans == 0) return false;
    const long blocks = (long)a.ntv * NW;
    if (blocks >= (1L << 31)) return false;
    l.kind = CopyLaunch::BTRANS;
    l.blocks = blocks;
    static const bool debug = getenv("SBX_COPY_DEBUG") != nullptr;
    if (debug)
        std::fprintf(stderr, "copy_btrans: R=%ld NU=%ld (SI %ld SO %ld DI %ld DO %ld) V1=%ld QT=%ld nw=%d "
                     "blocks=%ld runs %ld B\n", R, NU, NSI, NSO, NDI, NDO, n.size[v1], QT, nw, blocks,
                     best.score);
    return true;
}

template <typename S, typename D, bool ADD>
CopyLaunch prepare_pair(bool masked, Norm n, long total) {
    CopyLaunch l;
    l.run = run_launch<S, D, ADD>;
    l.total = total;
    if (masked) {
        if (total >= (1L << 32) - 1) throw Error("copy: masked boxes of 2^32 elements or more are not supported");
        if ((int)n.size.size() > MAXD) throw Error("copy: too many non-mergeable dimensions");
        DirectArgs &a = l.da;
        a.nd = (int)n.size.size();
        a.total = (uint32_t)total;
        for (int i = 0; i < a.nd; ++i) {
            a.size[i] = FastDiv((uint32_t)n.size[i]);
            a.sst[i] = n.ss[i];
            a.dst[i] = n.ds[i];
        }
        l.kind = CopyLaunch::MASKED;
        l.blocks = std::min((total + 255) / 256, 8192L);
        return l;
    }
    // Fully contiguous on both sides
    if (n.size.size() == 1 && n.ss[0] == 1 && n.ds[0] == 1) {
        l.kind = CopyLaunch::CONTIG;
        l.blocks = std::min((total + 255) / 256, 8192L);
        l.nt = g_copy_tune.nt > 0 || (g_copy_tune.nt == 0 && total * (long)sizeof(D) >= NT_MIN_BYTES);
        return l;
    }
    if (total >= (1L << 32) - 1) throw Error("copy: boxes with 2^32 elements or more are not supported yet");
    const int nd = (int)n.size.size();
    if (nd > MAXD) throw Error("copy: too many non-mergeable dimensions");

    // Run R: leading dim contiguous in both
    int first = 0;
    long R = 1;
    if (n.ss[0] == 1 && n.ds[0] == 1) {
        R = n.size[0];
        first = 1;
    }
    if (g_copy_tune.trans >= 0 && prepare_trans<S, D, ADD>(l, n, first, R, total)) return l;
    if (g_copy_tune.btrans >= 0 && prepare_btrans<S, D, ADD>(l, n, first, R, total)) return l;
    // V chain: dims contiguous in the destination from stride R (destination order);
    // U chain: dims contiguous in the source from stride R, not in V.  Both are capped so that a
    // tile holds a few hundred items on each side.
    constexpr long CHAIN_MAX = 256;
    // a chain may take only the inner part of a dimension: split size = inner * outer
    auto split_dim = [&](int i, long inner) {
        n.size.push_back(n.size[i] / inner);
        n.ss.push_back(n.ss[i] * inner);
        n.ds.push_back(n.ds[i] * inner);
        n.size[i] = inner;
    };
    auto best_divisor = [](long size, long cap) {
        long best = 1;
        for (long d = 2; d <= std::min(size, cap); ++d)
            if (size % d == 0) best = d;
        return best;
    };
    std::vector<int> U, Vc;
    std::vector<bool> used(nd, false);
    for (int i = 0; i < first; ++i) used[i] = true;
    auto build_chain = [&](bool dst_side, std::vector<int> &chain, long start) {
        long want = start, prod = 1;
        while (prod < CHAIN_MAX) {
            int found = -1;
            for (int i = 0; i < (int)n.size.size(); ++i)
                if (!used[i] && (dst_side ? n.ds[i] : n.ss[i]) == want) found = i;
            if (found < 0) break;
            if (prod * n.size[found] > CHAIN_MAX) {
                const long d = best_divisor(n.size[found], CHAIN_MAX / prod);
                if (d < 2) break;
                split_dim(found, d);
                used.push_back(false);
            }
            chain.push_back(found);
            used[found] = true;
            prod *= n.size[found];
            want *= n.size[found];
        }
    };
    bool u_contig = false; // the U chain starts at source stride R (its items are one run)
    if (first < nd && R <= 64) {
        const Norm n_keep = n;
        const std::vector<bool> used_keep = used;
        build_chain(true, Vc, R);
        if (!Vc.empty()) build_chain(false, U, R);
        u_contig = !U.empty();
        if (!Vc.empty() && U.empty() && g_copy_tune.order >= 0 && sizeof(S) == 8 &&
            std::is_same<S, D>::value && g_copy_tune.pair >= 0) {
            // the destination chain took the source's contiguous dim (n <-> c <-> xyz transposes:
            // c fastest in the source, second in the destination): with paired 8-byte accesses
            // the source chain goes first, so both phases move whole runs (the chain
            // redistribution tnsxyzc -> pxyztscn, complex<float>)
            Norm n_u = n_keep;
            std::vector<bool> used_u = used_keep;
            std::vector<int> U2, V2;
            std::swap(n, n_u);
            std::swap(used, used_u);
            build_chain(false, U2, R);
            if (!U2.empty()) build_chain(true, V2, R);
            if (!U2.empty() && !V2.empty()) {
                U = U2;
                Vc = V2;
                u_contig = true;
            } else {
                std::swap(n, n_u);
                std::swap(used, used_u);
            }
        }
        if (!Vc.empty() && U.empty()) {
            // the source-contiguous dims went to V: start U at the smallest remaining source
            // stride (reads of a tile then interleave across its V items, still line-complete)
            long smin = -1;
            for (int i = 0; i < (int)n.size.size(); ++i)
                if (!used[i] && (smin < 0 || n.ss[i] < smin)) smin = n.ss[i];
            if (smin > 0) build_chain(false, U, smin);
        }
    }
    const int ndd = (int)n.size.size(); // dims after splits
    if (ndd > MAXD) throw Error("copy: too many non-mergeable dimensions");
    if (Vc.empty() || U.empty()) {
        // Direct destination-ordered gather
        DirectArgs &a = l.da;
        a.nd = ndd;
        a.total = (uint32_t)total;
        for (int i = 0; i < ndd; ++i) {
            a.size[i] = FastDiv((uint32_t)n.size[i]);
            a.sst[i] = n.ss[i];
            a.dst[i] = n.ds[i];
        }
        l.kind = CopyLaunch::DIRECT;
        l.blocks = std::min((total + 255) / 256, 8192L);
        return l;
    }

    static const bool debug = getenv("SBX_COPY_DEBUG") != nullptr; // print the tiling
    TiledArgs &a = l.ta;
    long NU = 1, NV = 1;
    for (int i : U) NU *= n.size[i];
    for (int i : Vc) NV *= n.size[i];
    // Tile sizes: contiguous runs of >= 48 elements on both sides (>= 768 B for 16-byte
    // elements) and ~1.5K elements per workgroup so several workgroups share a CU
    // small copies: smaller tiles so that >= ~1024 workgroups (4 per CU) share the chip
    long budget = std::max(256L, std::min((long)tile_elems<D>(), total / 1024));
    if (g_copy_tune.budget > 0) budget = std::min((long)tile_elems<D>(), g_copy_tune.budget);
    const long run_target = g_copy_tune.run > 0 ? g_copy_tune.run : 48; // elements per contiguous source run of a tile row
    // the LDS image holds TV padded rows of R*TU + 1 elements: TV * (R*TU + 1) <= budget + 64
    const long cap = budget + 64;
    long TU = std::min(std::min(NU, std::max(1L, (run_target + R - 1) / R)), 256L);
    long TV = std::min(std::min(NV, std::max(1L, cap / (R * TU + 1))), 256L);
    if (TV == NV) TU = std::min(std::min(NU, std::max(1L, (cap / TV - 1) / R)), 256L);
    if (g_copy_tune.pair >= 0 && (sizeof(S) == 8 || sizeof(D) == 8) && (R & 1)) {
        // odd runs (c = 3): even tile rows keep the paired 16-byte accesses (below) -- the chain
        // redistribution at a 2048-element budget: TV 43 -> 42, 332 -> 167 us
        if (TV > 1 && TV < NV && (TV & 1)) --TV;
        if (TU > 1 && TU < NU && (TU & 1)) --TU;
    }
    if (R * TU * TV + TV > tile_elems<D>() + 64) throw Error("copy: internal tile sizing error");
    a.R = (uint32_t)R;
    a.TU = (uint32_t)TU;
    a.TV = (uint32_t)TV;
    a.NU = (uint32_t)NU;
    a.NV = (uint32_t)NV;
    a.fR = FastDiv((uint32_t)R);
    a.fTU = FastDiv((uint32_t)TU);
    a.fTV = FastDiv((uint32_t)TV);
    a.fRTU = FastDiv((uint32_t)(R * TU));
    a.fRTV = FastDiv((uint32_t)(R * TV));
    // lanes per tile row: the smallest power of two >= the row width, at most a wave
    auto lanes_log2 = [](long width) {
        uint32_t l2 = 0;
        while (l2 < 6 && (1L << l2) < width) ++l2;
        return l2;
    };
    // streaming stores for large destinations (written once, not re-read by this kernel):
    // the config-2p slice loop 6.8 -> 4.9 us per slice, the 1.6 GB permute 5.0 -> 5.2 TB/s
    a.nt = g_copy_tune.nt > 0 || (g_copy_tune.nt == 0 && total * (long)sizeof(D) >= NT_MIN_BYTES);
    a.lr = lanes_log2(R * TU);
    a.lw = lanes_log2(R * TV);
    a.lr2 = lanes_log2((R * TU + 1) / 2);
    a.lw2 = lanes_log2((R * TV + 1) / 2);
    a.ntu = (uint32_t)((NU + TU - 1) / TU);
    a.ntv = (uint32_t)((NV + TV - 1) / TV);
    a.nu = (int)U.size();
    for (std::size_t k = 0; k < U.size(); ++k) {
        a.usize[k] = FastDiv((uint32_t)n.size[U[k]]);
        a.usst[k] = n.ss[U[k]];
        a.udst[k] = n.ds[U[k]];
    }
    a.nv = (int)Vc.size();
    for (std::size_t k = 0; k < Vc.size(); ++k) {
        a.vsize[k] = FastDiv((uint32_t)n.size[Vc[k]]);
        a.vsst[k] = n.ss[Vc[k]];
        a.vdst[k] = n.ds[Vc[k]];
    }
    long NW = 1;
    int nw = 0;
    for (int i = first; i < ndd; ++i) {
        if (used[i]) continue;
        a.wsize[nw] = FastDiv((uint32_t)n.size[i]);
        a.wsst[nw] = n.ss[i];
        a.wdst[nw] = n.ds[i];
        NW *= n.size[i];
        ++nw;
    }
    a.nw = nw;
    if (g_copy_tune.pair >= 0 && (sizeof(S) == 8 || sizeof(D) == 8)) {
        // paired accesses: every tile row an even, 16-byte aligned run on that side (element
        // offsets of the row starts even: the other chain's and the outer dims' strides even)
        auto even_strides = [&](const std::vector<int> &dims, bool dst_side) {
            for (int i : dims)
                if (n.size[i] > 1 && ((dst_side ? n.ds[i] : n.ss[i]) & 1)) return false;
            return true;
        };
        std::vector<int> W;
        for (int i = first; i < ndd; ++i)
            if (!used[i]) W.push_back(i);
        const bool rows_u = (R * TU) % 2 == 0 && (R * (NU % TU)) % 2 == 0;
        const bool rows_v = (R * TV) % 2 == 0 && (R * (NV % TV)) % 2 == 0;
        l.vr = sizeof(S) == 8 && u_contig && rows_u && even_strides(Vc, false) && even_strides(W, false);
        l.vw = sizeof(D) == 8 && !ADD && rows_v && even_strides(U, true) && even_strides(W, true);
    }
    const long blocks = (long)a.ntu * a.ntv * NW;
    if (blocks >= (1L << 31)) throw Error("copy: grid too large");
    if (debug) {
        std::fprintf(stderr, "copy_tiled: dims(size/ss/ds)");
        for (int i = 0; i < ndd; ++i) std::fprintf(stderr, " %ld/%ld/%ld", n.size[i], n.ss[i], n.ds[i]);
        std::fprintf(stderr, " | R=%ld NU=%ld NV=%ld TU=%ld TV=%ld nu=%d nv=%d nw=%d blocks=%ld vr=%d vw=%d\n",
                     R, NU, NV, TU, TV, a.nu, a.nv, nw, blocks, l.vr, l.vw);
    }
    l.kind = CopyLaunch::TILED3;
    l.blocks = blocks;
    return l;
}

template <typename S, typename D>
CopyLaunch prepare_sd(bool add, bool masked, const Norm &n, long total) {
    return add ? prepare_pair<S, D, true>(masked, n, total)
               : prepare_pair<S, D, false>(masked, n, total);
}

CopyLaunch prepare_launch(const BoxCopyDesc &d, long total) {
    const Norm n = normalize(d);
    const bool m = d.src_mask || d.dst_mask, a = d.add;
    const int st = d.src_t, dt = d.dst_t;
    if (st == dt) {
        switch (st) {
        case SBX_FLOAT: return prepare_sd<float, float>(a, m, n, total);
        case SBX_DOUBLE: return prepare_sd<double, double>(a, m, n, total);
        case SBX_CFLOAT: return prepare_sd<float2, float2>(a, m, n, total);
        case SBX_CDOUBLE: return prepare_sd<double2, double2>(a, m, n, total);
        case SBX_INT: return prepare_sd<int, int>(a, m, n, total);
        case SBX_SIZE_T: return prepare_sd<unsigned long, unsigned long>(a, m, n, total);
        }
    }
    if (st == SBX_FLOAT && dt == SBX_DOUBLE) return prepare_sd<float, double>(a, m, n, total);
    if (st == SBX_DOUBLE && dt == SBX_FLOAT) return prepare_sd<double, float>(a, m, n, total);
    if (st == SBX_CFLOAT && dt == SBX_CDOUBLE) return prepare_sd<float2, double2>(a, m, n, total);
    if (st == SBX_CDOUBLE && dt == SBX_CFLOAT) return prepare_sd<double2, float2>(a, m, n, total);
    if (st == SBX_FLOAT && dt == SBX_CFLOAT) return prepare_sd<float, float2>(a, m, n, total);
    if (st == SBX_FLOAT && dt == SBX_CDOUBLE) return prepare_sd<float, double2>(a, m, n, total);
    if (st == SBX_DOUBLE && dt == SBX_CFLOAT) return prepare_sd<double, float2>(a, m, n, total);
    if (st == SBX_DOUBLE && dt == SBX_CDOUBLE) return prepare_sd<double, double2>(a, m, n, total);
    if (st == SBX_INT && dt == SBX_SIZE_T) return prepare_sd<int, unsigned long>(a, m, n, total);
    if (st == SBX_SIZE_T && dt == SBX_INT) return prepare_sd<unsigned long, int>(a, m, n, total);
    throw Error("copy: unsupported type conversion");
}

/// Launch cache: prepared launches by box shape, bounded (cleared when it reaches 4096 shapes;
/// the reference caps its plan caches at a fraction of memory, cache.h:21-305)
struct LaunchKeyHash {
    std::size_t operator()(const std::vector<long> &k) const {
        std::size_t h = 1469598103934665603ull;
        for (long v : k) h = (h ^ (std::size_t)v) * 1099511628211ull;
        return h;
    }
};
std::mutex g_launch_mutex;
std::unordered_map<std::vector<long>, CopyLaunch, LaunchKeyHash> &launch_cache() {
    static std::unordered_map<std::vector<long>, CopyLaunch, LaunchKeyHash> c;
    return c;
}

} // namespace

void clear_copy_launch_cache() {
    std::lock_guard<std::mutex> g(g_launch_mutex);
    launch_cache().clear();
}

namespace {
thread_local CopyTape *t_tape = nullptr;
}
void set_copy_tape(CopyTape *t) { t_tape = t; }
CopyTape *current_copy_tape() { return t_tape; }

void replay_launch(const TapeLaunch &tl, const void *src, void *dst, const Scalar &alpha) {
    const CopyLaunch &l = *(const CopyLaunch *)tl.launch.get();
    set_device(tl.device);
    const Alpha a{alpha.re, alpha.im, alpha.is_one() ? 1 : alpha.is_zero() ? 2 : 0};
    l.run(l, src, dst, a, nullptr, nullptr, get_stream(tl.device));
}

void launch_box_copy(const BoxCopyDesc &d, int device) {
    long total = 1;
    for (long s : d.size) total *= s;
    if (total == 0) return;
    // boxes beyond the kernels' 32-bit element indexing (2^31 elements and more -- 32 GB of
    // complex<double> fit in 288 GB of HBM) are copied as slabs of the dimension with the
    // largest destination stride, each slab a separate launch on shifted base pointers
    const long max_elems = g_copy_tune.max_elems > 0 ? g_copy_tune.max_elems : (1L << 31) - 1;
    if (total > max_elems) {
        int k = -1;
        for (int i = 0; i < (int)d.size.size(); ++i)
            if (d.size[i] > 1 && (k < 0 || d.dst_stride[i] > d.dst_stride[k])) k = i;
        const long inner = total / d.size[k];
        const long rows = std::max(1L, max_elems / inner);
        for (long r0 = 0; r0 < d.size[k]; r0 += rows) {
            BoxCopyDesc c = d;
            c.size[k] = std::min(rows, d.size[k] - r0);
            c.src = (const char *)d.src + dtype_size(d.src_t) * r0 * d.src_stride[k];
            c.dst = (char *)d.dst + dtype_size(d.dst_t) * r0 * d.dst_stride[k];
            if (d.src_mask) c.src_mask = d.src_mask + r0 * d.src_stride[k];
            if (d.dst_mask) c.dst_mask = d.dst_mask + r0 * d.dst_stride[k];
            launch_box_copy(c, device);
        }
        return;
    }
    set_device(device);
    hipStream_t s = get_stream(device);
    // key: types, Copy/Add, masks, the box (sizes and both strides), the tuning switches
    const std::size_t nd = d.size.size();
    std::vector<long> key;
    key.reserve(4 + 3 * nd);
    key.push_back(d.src_t | (d.dst_t << 8) | ((long)d.add << 16) |
                  ((long)(d.src_mask != nullptr) << 17) | ((long)(d.dst_mask != nullptr) << 18));
    key.push_back(g_copy_tune.budget);
    key.push_back(g_copy_tune.run);
    key.push_back(16L * g_copy_tune.nt + 256L * g_copy_tune.pair +
                  4096L * g_copy_tune.order + 65536L * g_copy_tune.trans +
                  1048576L * g_copy_tune.btrans);
    for (std::size_t i = 0; i < nd; ++i) {
        key.push_back(d.size[i]);
        key.push_back(d.src_stride[i]);
        key.push_back(d.dst_stride[i]);
    }
    CopyLaunch l;
    bool hit = false;
    {
        std::lock_guard<std::mutex> g(g_launch_mutex);
        auto it = launch_cache().find(key);
        if (it != launch_cache().end()) {
            l = it->second;
            hit = true;
        }
    }
    if (!hit) {
        l = prepare_launch(d, total);
        std::lock_guard<std::mutex> g(g_launch_mutex);
        if (launch_cache().size() >= 4096) launch_cache().clear();
        launch_cache().emplace(std::move(key), l);
    }
    if (CopyTape *t = t_tape) {
        if (d.src_mask || d.dst_mask)
            t->valid = false;
        else
            t->launches.push_back(TapeLaunch{std::make_shared<CopyLaunch>(l), d.src, d.dst,
                                             device, d.alpha});
    }
    const Alpha alpha{d.alpha.re, d.alpha.im, d.alpha.is_one() ? 1 : d.alpha.is_zero() ? 2 : 0};
    l.run(l, d.src, d.dst, alpha, d.src_mask, d.dst_mask, s);
}

int copy_kernel_plan(const BoxCopyDesc &d, long *blocks) {
    long total = 1;
    for (long x : d.size) total *= x;
    if (total == 0) return -1;
    const CopyLaunch l = prepare_launch(d, total);
    if (blocks) *blocks = l.blocks;
    return (int)l.kind;
}

void launch_zero(void *p, std::size_t bytes, int device) {
    if (bytes == 0) return;
    set_device(device);
    SBX_HIP_CHECK(hipMemsetAsync(p, 0, bytes, get_stream(device)));
}

//
// Index-vector gather / scatter of `blocking`-element runs: the reference's low-level
// copy_n / copy_n_blocking with explicit index vectors (copy_n.h:584-740, 898-1050), which the
// library's own copy() never materialises but which callers of superbblas::detail use directly.
// One lane per element of the n * blocking runs; a run's lanes are consecutive, so the accesses
// of a wave are coalesced whenever blocking >= 16 and contiguous for null index vectors.
//
namespace {
template <typename S, typename D, bool ADD>
__global__ void __launch_bounds__(256)
    copy_index_kernel(const S *__restrict__ src, const int *__restrict__ sidx, D *dst,
                      const int *__restrict__ didx, long n, long blocking, Alpha alpha) {
    const long total = n * blocking;
    for (long e = blockIdx.x * 256L + threadIdx.x; e < total; e += (long)gridDim.x * 256L) {
        const long d = e / blocking, r = e - d * blocking;
        const long so = (sidx ? (long)sidx[d] : d * blocking) + r;
        const long wo = (didx ? (long)didx[d] : d * blocking) + r;
        put<ADD, D>(dst + wo, xform<D, S>(src[so], alpha));
    }
}

template <typename S, typename D>
void index_copy_typed(const IndexCopyDesc &c, const Alpha &a, hipStream_t s) {
    const long total = c.n * c.blocking;
    const long blocks = std::max(1L, std::min((total + 255) / 256, 256L * 64));
    if (c.add)
        copy_index_kernel<S, D, true><<<blocks, 256, 0, s>>>((const S *)c.src, c.src_idx,
                                                             (D *)c.dst, c.dst_idx, c.n,
                                                             c.blocking, a);
    else
        copy_index_kernel<S, D, false><<<blocks, 256, 0, s>>>((const S *)c.src, c.src_idx,
                                                              (D *)c.dst, c.dst_idx, c.n,
                                                              c.blocking, a);
    SBX_HIP_CHECK(hipGetLastError());
}
} // namespace

void launch_index_copy(const IndexCopyDesc &c, int device) {
    if (c.n <= 0 || c.blocking <= 0) return;
    set_device(device);
    hipStream_t s = get_stream(device);
    KernelTimer timer("copy", s);
    const Alpha a{c.alpha.re, c.alpha.im, c.alpha.is_one() ? 1 : c.alpha.is_zero() ? 2 : 0};
    const int st = c.src_t, dt = c.dst_t;
    if (st == dt) {
        switch (st) {
        case SBX_FLOAT: return index_copy_typed<float, float>(c, a, s);
        case SBX_DOUBLE: return index_copy_typed<double, double>(c, a, s);
        case SBX_CFLOAT: return index_copy_typed<float2, float2>(c, a, s);
        case SBX_CDOUBLE: return index_copy_typed<double2, double2>(c, a, s);
        case SBX_INT: return index_copy_typed<int, int>(c, a, s);
        case SBX_SIZE_T: return index_copy_typed<unsigned long, unsigned long>(c, a, s);
        }
    }
    if (st == SBX_FLOAT && dt == SBX_DOUBLE) return index_copy_typed<float, double>(c, a, s);
    if (st == SBX_DOUBLE && dt == SBX_FLOAT) return index_copy_typed<double, float>(c, a, s);
    if (st == SBX_CFLOAT && dt == SBX_CDOUBLE) return index_copy_typed<float2, double2>(c, a, s);
    if (st == SBX_CDOUBLE && dt == SBX_CFLOAT) return index_copy_typed<double2, float2>(c, a, s);
    if (st == SBX_FLOAT && dt == SBX_CFLOAT) return index_copy_typed<float, float2>(c, a, s);
    if (st == SBX_FLOAT && dt == SBX_CDOUBLE) return index_copy_typed<float, double2>(c, a, s);
    if (st == SBX_DOUBLE && dt == SBX_CFLOAT) return index_copy_typed<double, float2>(c, a, s);
    if (st == SBX_DOUBLE && dt == SBX_CDOUBLE) return index_copy_typed<double, double2>(c, a, s);
    if (st == SBX_INT && dt == SBX_SIZE_T) return index_copy_typed<int, unsigned long>(c, a, s);
    if (st == SBX_SIZE_T && dt == SBX_INT) return index_copy_typed<unsigned long, int>(c, a, s);
    throw Error("copy_n: unsupported type conversion");
}

} // namespace sbx
