// Batched (complex) GEMM on CDNA4 matrix cores -- the local contraction of superbblas.
//
// Replaces the reference's `xgemm_batch_strided` -> `rocblas_gemm_strided_batched_ex`
// (blas.h:662-810, called from local_contraction_normalized, tensor.h:1567-1597) with a
// hand-written MFMA kernel:
//  * f64 / complex<f64>: v_mfma_f64_16x16x4_f64; f32 / complex<f32>: v_mfma_f32_16x16x4_f32.
//    There is no complex MFMA, so a complex tile product issues 4 real MFMAs
//    (re*re - im*im, re*im + im*re: the 4-multiplication form, which keeps each component's
//    rounding at the level of BLAS zgemm -- pinned against the reference's OpenBLAS output on
//    near-real and wide-range operands, tests/test_gpu_golden.py).  The 3-multiplication (Gauss)
//    form is an opt-in (sbx_tune_set("gemm.m3", 1)): 25 % fewer MFMAs, but a small imaginary
//    part inherits the rounding of the large real products.  Conjugation flips the sign of the
//    imaginary part when the fragment is read.
//  * Operands are staged global -> registers -> LDS (async-stage split: the next K-slab is
//    loaded into registers while the current one is consumed from LDS), in a [row][k] image
//    padded by one element so that the 16-byte fragment reads are bank-conflict free.
//  * The thread -> element map of a stage load follows whichever operand stride is unit
//    (k-contiguous or m/n-contiguous), so both `T` and `N` layouts read coalesced rows.
//  * Split-K over workgroups when the output has too few tiles to fill 256 CUs (the
//    lattice contraction has m = n = 256, k = 12288, batch = 16: only 256 64x64 tiles);
//    the partial slabs are summed in a fixed order by a second kernel, so results are
//    deterministic.
//  * XCD-aware workgroup numbering: the tiles of one (batch, k-split) group are dealt to one
//    XCD so that their shared A/B panels hit that XCD's L2.
#include "sbx_internal.h"

#include <algorithm>
#include <map>
#include <mutex>
#include <cstdint>
#include <type_traits>

namespace sbx {
GemmTune g_gemm_tune;
namespace {

template <typename R> struct Mfma;
template <> struct Mfma<double> {
    typedef double acc_t __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc_t mma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    // C/D map of v_mfma_f64_16x16x4_f64: col = lane&15, row = (lane>>4) + 4*reg
    static __device__ __forceinline__ int row(int lane, int r) { return (lane >> 4) + 4 * r; }
};
template <> struct Mfma<float> {
    typedef float acc_t __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // C/D map of v_mfma_f32_16x16x4_f32: col = lane&15, row = 4*(lane>>4) + reg
    static __device__ __forceinline__ int row(int lane, int r) { return ((lane >> 4) << 2) + r; }
};

template <typename R, bool CPLX> struct Elem;
template <> struct Elem<double, true> { typedef double2 type; };
template <> struct Elem<double, false> { typedef double type; };
template <> struct Elem<float, true> { typedef float2 type; };
template <> struct Elem<float, false> { typedef float type; };

template <typename E> __device__ __forceinline__ E zero_elem() { return E{}; }
[[maybe_unused]] __device__ __forceinline__ double2 conj_if(double2 v, bool c) { return c ? double2{v.x, -v.y} : v; }
__device__ __forceinline__ float2 conj_if(float2 v, bool c) { return c ? float2{v.x, -v.y} : v; }
__device__ __forceinline__ double conj_if(double v, bool) { return v; }
__device__ __forceinline__ float conj_if(float v, bool) { return v; }

/// 16/8/4-byte load through a buffer descriptor: an offset past the descriptor's range returns
/// zero, which is how out-of-tile elements are padded (no per-load branch, so the compiler keeps
/// every stage load in flight behind the MFMAs instead of waiting after each one).
template <typename E> __device__ __forceinline__ E buf_load(__amdgpu_buffer_rsrc_t r, unsigned off);
template <> [[maybe_unused]] __device__ __forceinline__ double2 buf_load<double2>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
    return __builtin_bit_cast(double2, v);
}
template <> __device__ __forceinline__ double buf_load<double>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return __builtin_bit_cast(double, v);
}
template <> __device__ __forceinline__ float2 buf_load<float2>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
    return __builtin_bit_cast(float2, v);
}
template <> __device__ __forceinline__ float buf_load<float>(__amdgpu_buffer_rsrc_t r, unsigned off) {
    auto v = __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
    return __builtin_bit_cast(float, v);
}

struct GemmKArgs {
    long m, n, k, batch;
    const void *a;
    long sa_m, sa_k, sa_b;
    const void *b;
    long sb_k, sb_n, sb_b;
    void *c;
    long sc_m, sc_n, sc_b;
    double alpha_re, alpha_im, beta_re, beta_im;
    int conja, conjb;
    int splits;
    long kchunk;
    void *work;
    unsigned long long *probe; // tools only: workgroup 0 stores s_memtime / s_memrealtime at its start and end
    int probe_all;             // tools only: every workgroup stores s_memrealtime at its start, at the end of
                               // its main loop and at its end in probe[2 + 3 * blockIdx.x ...]
    int tm, tn;
    unsigned a_bytes, b_bytes; // extent of one batch entry of A / B (buffer descriptor range)
    // split label groups: index i of M (N, K) is (i / m_lo, i % m_lo) with strides (sa_m_hi,
    // sa_m), ...; split == 0 when every group is one run (m_lo == m, ...)
    int split;
    long m_lo, n_lo, k_lo;
    long sa_m_hi, sa_k_hi, sb_k_hi, sb_n_hi, sc_m_hi, sc_n_hi;
    // A and B are the same memory with the same M / N and K addressing (a tensor contracted with
    // itself or its conjugate, e.g. the chain's correlator y^H y): a workgroup on a diagonal tile
    // (m0 == n0) stages one slab image and reads both operands' fragments from it
    int same_ab;
    int dma_nt; // the loader waves' slab DMA with the non-temporal policy (gemm.dma_nt)
    // gemm_frag_kernel<., KP = true>: the operand's k pairs are one 16-byte load (8-byte
    // elements, unit k stride, 16-byte aligned rows)
    int pair_a, pair_b;
};

/// Offset of index i of a split group: (i / lo) * s_hi + (i % lo) * s (i < 2^31)
__device__ __forceinline__ long split_off(long i, long lo, long s, long s_hi) {
    const unsigned q = (unsigned)i / (unsigned)lo;
    return (long)q * s_hi + (long)((unsigned)i - q * (unsigned)lo) * s;
}
__device__ __forceinline__ long c_off(const GemmKArgs &p, long gi, long gj) {
    return p.split ? split_off(gi, p.m_lo, p.sc_m, p.sc_m_hi) + split_off(gj, p.n_lo, p.sc_n, p.sc_n_hi)
                   : gi * p.sc_m + gj * p.sc_n;
}

// out = alpha*v (+ beta*old)
template <typename R>
__device__ __forceinline__ void epilogue_store(R *cptr, R vr, R vi, const GemmKArgs &p, bool cplx) {
    if (cplx) {
        R ar = (R)p.alpha_re, ai = (R)p.alpha_im;
        R outr = ar * vr - ai * vi, outi = ar * vi + ai * vr;
        if (p.beta_re != 0 || p.beta_im != 0) {
            R br = (R)p.beta_re, bi = (R)p.beta_im;
            R cr = cptr[0], ci = cptr[1];
            outr += br * cr - bi * ci;
            outi += br * ci + bi * cr;
        }
        cptr[0] = outr;
        cptr[1] = outi;
    } else {
        R out = (R)p.alpha_re * vr;
        if (p.beta_re != 0) out += (R)p.beta_re * cptr[0];
        cptr[0] = out;
    }
}

template <typename R, bool CPLX, bool AK, bool BK, int BM, int BN, int BKK, int WM, int WN>
__global__ void __launch_bounds__(WM *WN * 64) gemm_kernel(const GemmKArgs p) {
    typedef typename Elem<R, CPLX>::type E;
    typedef typename Mfma<R>::acc_t acc_t;
    constexpr int NTH = WM * WN * 64;
    constexpr int LDK = BKK + 1; // padded [row][k] image
    constexpr int EA = BM * BKK / NTH;
    constexpr int EB = BN * BKK / NTH;
    static_assert(EA * NTH == BM * BKK && EB * NTH == BN * BKK, "tile/threads mismatch");
    constexpr int WTM = BM / WM, WTN = BN / WN; // wave tile
    constexpr int MT = WTM / 16, NT = WTN / 16;
    static_assert(MT * 16 == WTM && NT * 16 == WTN && BKK % 4 == 0, "bad wave tile");

    __shared__ E As[BM * LDK];
    __shared__ E Bs[BN * LDK];

    // XCD-aware remap: consecutive logical workgroups share an XCD (bijective form)
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);

    const int ti = wg % p.tm;
    int rest = wg / p.tm;
    const int tj = rest % p.tn;
    rest /= p.tn;
    const int split = rest % p.splits;
    const long bb = rest / p.splits;

    const long m0 = (long)ti * BM, n0 = (long)tj * BN;
    const long k_begin = (long)split * p.kchunk;
    const long k_end = min(p.k, k_begin + p.kchunk);

    const E *__restrict__ A = (const E *)p.a + bb * p.sa_b;
    const E *__restrict__ B = (const E *)p.b + bb * p.sb_b;
    const int tid = threadIdx.x;
    const bool conja = p.conja != 0, conjb = p.conjb != 0;

    E ra[EA], rb[EB];
    // Wave-uniform buffer descriptors of this batch entry (T8/T20 of the CDNA guide)
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, (short)0, (int)p.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB =
        __builtin_amdgcn_make_buffer_rsrc((void *)B, (short)0, (int)p.b_bytes, 0x00020000);
    constexpr unsigned OOB = 0x80000000u; // past any descriptor range: loads return 0
    auto load_stage = [&](long k0) {
#pragma unroll
        for (int i = 0; i < EA; ++i) {
            const int e = tid + NTH * i;
            const int row = AK ? e / BKK : e % BM;
            const int kk = AK ? e % BKK : e / BM;
            const long gi = m0 + row, gk = k0 + kk;
            const bool ok = gi < p.m && gk < k_end;
            const long o = p.split ? split_off(gi, p.m_lo, p.sa_m, p.sa_m_hi) +
                                         split_off(gk, p.k_lo, p.sa_k, p.sa_k_hi)
                                   : gi * p.sa_m + gk * p.sa_k;
            const unsigned off = ok ? (unsigned)(o * sizeof(E)) : OOB;
            ra[i] = buf_load<E>(rsA, off);
        }
#pragma unroll
        for (int i = 0; i < EB; ++i) {
            const int e = tid + NTH * i;
            const int col = BK ? e / BKK : e % BN;
            const int kk = BK ? e % BKK : e / BN;
            const long gj = n0 + col, gk = k0 + kk;
            const bool ok = gj < p.n && gk < k_end;
            const long o = p.split ? split_off(gk, p.k_lo, p.sb_k, p.sb_k_hi) +
                                         split_off(gj, p.n_lo, p.sb_n, p.sb_n_hi)
                                   : gk * p.sb_k + gj * p.sb_n;
            const unsigned off = ok ? (unsigned)(o * sizeof(E)) : OOB;
            rb[i] = buf_load<E>(rsB, off);
        }
    };
    auto store_stage = [&]() {
#pragma unroll
        for (int i = 0; i < EA; ++i) {
            const int e = tid + NTH * i;
            const int row = AK ? e / BKK : e % BM;
            const int kk = AK ? e % BKK : e / BM;
            As[row * LDK + kk] = conj_if(ra[i], conja);
        }
#pragma unroll
        for (int i = 0; i < EB; ++i) {
            const int e = tid + NTH * i;
            const int col = BK ? e / BKK : e % BN;
            const int kk = BK ? e % BKK : e / BN;
            Bs[col * LDK + kk] = conj_if(rb[i], conjb);
        }
    };

    const int lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int frow = wm * WTM + (lane & 15); // fragment row (A) / col (B) in the tile
    const int fcol = wn * WTN + (lane & 15);
    const int kq = lane >> 4;

    acc_t accR[MT][NT], accI[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            accR[i][j] = acc_t{0, 0, 0, 0};
            accI[i][j] = acc_t{0, 0, 0, 0};
        }

    long k0 = k_begin;
    if (k0 < k_end) load_stage(k0);
    for (; k0 < k_end; k0 += BKK) {
        __syncthreads(); // the previous slab is no longer read
        store_stage();
        __syncthreads();
        if (k0 + BKK < k_end) load_stage(k0 + BKK); // in flight while this slab is consumed
#pragma unroll
        for (int kk = 0; kk < BKK; kk += 4) {
            E af[MT], bf[NT];
#pragma unroll
            for (int i = 0; i < MT; ++i) af[i] = As[(frow + 16 * i) * LDK + kk + kq];
#pragma unroll
            for (int j = 0; j < NT; ++j) bf[j] = Bs[(fcol + 16 * j) * LDK + kk + kq];
            if constexpr (CPLX) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(af[i].x, bf[j].x, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].x, bf[j].y, accI[i][j]);
                    }
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(-af[i].y, bf[j].y, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].y, bf[j].x, accI[i][j]);
                    }
            } else {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j)
                        accR[i][j] = Mfma<R>::mma(af[i], bf[j], accR[i][j]);
            }
        }
    }

    // Epilogue
    const int ccol = lane & 15;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long gi = m0 + wm * WTM + 16 * i + Mfma<R>::row(lane, r);
                const long gj = n0 + wn * WTN + 16 * j + ccol;
                if (gi >= p.m || gj >= p.n) continue;
                const R vr = accR[i][j][r];
                const R vi = CPLX ? accI[i][j][r] : R(0);
                if (p.splits == 1) {
                    R *cptr = (R *)((E *)p.c + bb * p.sc_b + c_off(p, gi, gj));
                    epilogue_store<R>(cptr, vr, vi, p, CPLX);
                } else {
                    E *w = (E *)p.work + (((long)split * p.batch + bb) * p.n + gj) * p.m + gi;
                    if constexpr (CPLX)
                        *w = E{vr, vi};
                    else
                        *w = vr;
                }
            }
    if (p.probe && p.probe_all) {
        __syncthreads();
        if (tid == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            p.probe[4 + 3 * bid] = __builtin_amdgcn_s_memrealtime();
        }
    }
}

// ---------------------------------------------------------------------------------------------
// LDS-DMA kernel (buffer_load_dwordx4 ... lds), every element type
//
// Both operands go global -> LDS in 16-byte DMA lanes ("granules": 1 complex<double>, 2 double
// or complex<float>, 4 float) with no VGPR round trip and no ds_write pass.  Per operand the LDS
// image of a BKK-deep K slab is either
//   K-major  [row][BKK k] (operand contiguous along k), the granule column XOR-swizzled on the
//            SOURCE address (the DMA destination is lane-linear) so that the 16 rows of a
//            fragment read (same k) hit 16 different bank groups;
//   M-major  [BKK k][rows] (operand contiguous along m / n), read conflict-free as is.
// Two LDS buffers, one barrier per slab: the DMA of slab s+1 is in flight while slab s feeds the
// MFMAs (the barrier's vmcnt(0) retires it one slab later).  Out-of-range rows/k read zero
// through the buffer descriptor (no branches); a granule never straddles the edge of the
// operand (launcher's precondition).  Conjugation flips the fragment's imaginary sign.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned lds_addr(const void *p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void *)p;
}

template <bool XK, int R, int BKK, int NTH, int ES>
struct DmaOperand {
    static constexpr int EPG = 16 / ES;          // elements per 16-B granule
    static constexpr int GR = BKK / EPG;         // granules per K-major row
    static constexpr int GTOT = R * BKK / EPG;   // granules per slab image
    static constexpr int NI = (GTOT + NTH - 1) / NTH; // DMA lanes per thread per slab
    // a partial last pass is skipped by whole waves (a DMA instruction writes 64 lanes of LDS,
    // out-of-range lanes included): the image must be a whole number of wave passes
    static_assert(GTOT * EPG == R * BKK && GTOT % 64 == 0 && GR >= 1 && (!XK || GR <= 16),
                  "tile/threads mismatch");
    unsigned roff[NI]; // byte offset of this lane's granule at k0 = 0
    int kl[NI];        // first k of the granule within the slab
    bool rok[NI];
    // K-major image: granule swizzle so that 16 consecutive rows read at one k hit distinct
    // 16-B bank groups (a 256-B bank row holds 16/GR image rows)
    static __device__ __forceinline__ int swz(int row) { return (row / (16 / GR)) & (GR - 1); }
    __device__ __forceinline__ void init(int tid, long r0, long nrows, long s_r, long s_k,
                                         bool split = false, long r_lo = 1, long s_r_hi = 0) {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            const int slot = tid + NTH * i; // lane-linear granule slot of this lane
            int r, k;
            if (XK) {
                r = slot / GR;
                k = ((slot % GR) ^ swz(r)) * EPG;
            } else {
                r = (slot % (R / EPG)) * EPG;
                k = slot / (R / EPG);
            }
            const long gr = r0 + r;
            rok[i] = gr < nrows;
            kl[i] = k;
            // split groups: the row part only; the k part is added per slab in issue()
            roff[i] = split ? (unsigned)(split_off(rok[i] ? gr : 0, r_lo, s_r, s_r_hi) * ES)
                            : (unsigned)(((rok[i] ? gr : 0) * s_r + (long)k * s_k) * ES);
        }
    }
    // issue the DMA of slab [k0, k0+BKK) into the image at `lds_base`
    __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, const char *lds_base,
                                          int wave, long k0, long k_end, long s_k,
                                          bool split = false, long k_lo = 1,
                                          long s_k_hi = 0) const {
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (GTOT % NTH && i * NTH + wave * 64 >= GTOT) break; // (wave-uniform)
            const bool ok = rok[i] && (k0 + kl[i] < k_end);
            const unsigned kpart = split ? (unsigned)(split_off(k0 + kl[i], k_lo, s_k, s_k_hi) * ES)
                                         : (unsigned)(k0 * s_k * ES);
            const unsigned off = ok ? roff[i] + kpart : 0x80000000u;
            // inline asm so that hipcc does not wait vmcnt(0) before every ds_read of the
            // other buffer (it cannot tell the DMA target from the buffer being read); the
            // kernel retires the DMA itself with an explicit vmcnt(0) before its barrier
            const unsigned dst = lds_addr(lds_base) + (unsigned)(i * NTH + wave * 64) * 16;
            asm volatile("s_mov_b32 m0, %1\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %0, %2, 0 offen lds"
                         :
                         : "v"(off), "s"(dst), "s"(rs)
                         : "memory", "m0");
        }
    }
    // element index of fragment element (row, k) in the slab image
    static __device__ __forceinline__ int slot(int row, int k) {
        return XK ? row * BKK + (((k / EPG) ^ swz(row)) * EPG + k % EPG) : k * R + row;
    }
};

// Loader-wave DMA of a K-major operand whose rows are one run (no split groups): the first LWT
// threads of the workgroup (LW = LWT / 64 "loader" waves) issue the whole slab image while the
// other waves only read fragments and issue MFMAs.  Lane slot = tid + LWT * i (i < NI), so a
// lane's granule column and swizzle are the same for every i and its state is three registers
// (the per-lane arrays of DmaOperand would cost 6 NI of them).  The image is DmaOperand<true>'s.
template <int R, int BKK, int LWT, int ES> struct DmaRowsK {
    static constexpr int EPG = 16 / ES, GR = BKK / EPG, GTOT = R * BKK / EPG, NI = GTOT / LWT;
    static constexpr int RSTEP = LWT / GR; // rows between a lane's consecutive granules
    static_assert(GTOT % LWT == 0 && LWT % GR == 0 && GR <= 16 && (RSTEP / (16 / GR)) % GR == 0,
                  "loader lane map");
    unsigned off0, step;
    int k, rleft;
    __device__ __forceinline__ void init(int tid, long r0, long nrows, long s_r, long s_k) {
        const int r = tid / GR;
        k = ((tid % GR) ^ ((r / (16 / GR)) & (GR - 1))) * EPG;
        rleft = (int)min(nrows - r0 - r, (long)0x7fffffff);
        off0 = (unsigned)(((r0 + r) * s_r + (long)k * s_k) * ES); // (used only while in range)
        step = (unsigned)((long)RSTEP * s_r * ES);
    }
    // issue granules i in [ib, ie) of slab [k0, k0+BKK) into the image at `lds_base`
    __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, const char *lds_base,
                                          int wave, long k0, long k_end, long s_k, int ib,
                                          int ie, bool nt = false) const {
        const unsigned kpart = (unsigned)(k0 * s_k * ES);
        const bool kok = k0 + k < k_end;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
            if (i < ib || i >= ie) continue;
            const bool ok = kok && RSTEP * i < rleft;
            const unsigned off = ok ? off0 + (unsigned)i * step + kpart : 0x80000000u;
            const unsigned dst = lds_addr(lds_base) + (unsigned)(i * LWT + wave * 64) * 16;
            if (nt)
                asm volatile("s_mov_b32 m0, %1\n\t"
                             "s_nop 0\n\t"
                             "buffer_load_dwordx4 %0, %2, 0 offen nt lds"
                             :
                             : "v"(off), "s"(dst), "s"(rs)
                             : "memory", "m0");
            else
                asm volatile("s_mov_b32 m0, %1\n\t"
                             "s_nop 0\n\t"
                             "buffer_load_dwordx4 %0, %2, 0 offen lds"
                             :
                             : "v"(off), "s"(dst), "s"(rs)
                             : "memory", "m0");
        }
    }
};

struct NoLoader { // (LW == 0: every wave issues its share through DmaOperand)
    static constexpr int NI = 0;
    __device__ void init(int, long, long, long, long) {}
    __device__ void issue(__amdgpu_buffer_rsrc_t, const char *, int, long, long, long, int, int, bool = false) const {}
};

// M3: complex products in the 3-multiplication (Gauss) form, P1 = ar*br, P2 = ai*bi,
// P3 = (ar+ai)*(br+bi), re = P1 - P2, im = P3 - P1 - P2: 3 real MFMAs per complex k-step instead
// of 4 (a third accumulator per tile; the operand sums are one VALU add per fragment element)
// PF: the 4-multiplication path reads the fragments of k-step kk+4 from LDS before issuing the
// MFMAs of k-step kk (a register double buffer), so a wave's LDS latency hides behind its own
// MFMAs, not only behind the other wave of its SIMD
// KG > 1: the workgroup's waves form KG groups of WM x WN; group g takes the k-steps g, g + KG,
// ... of every slab (an intra-workgroup split-K: a 48x48 output in 4 waves of the whole tile, so
// every SIMD of a CU gets the same share and each wave issues 36 MFMAs per 6 fragment reads); the
// groups' partial tiles are summed through LDS in group order at the end (deterministic)
// SH: every tile of the launch is a diagonal tile of a tensor contracted with itself (same_ab,
// one tile row and column): the slab image holds A only, so the double buffer takes half the LDS
// and twice the workgroups fit a CU
// LW > 0: only waves 0..LW-1 issue the slab DMA (K-major operands without split groups), each
// spreading its share over the first SP k-steps of the slab; the other waves issue no DMA
template <typename R, bool CPLX, bool AK, bool BK, int BM, int BN, int BKK, int WM, int WN,
          bool M3 = false, bool PF = false, int KG = 1, bool SH = false, int LW = 0, int SP = 1>
__global__ void __launch_bounds__(WM *WN *KG * 64) gemm_dma_kernel(const GemmKArgs p) {
    typedef typename Elem<R, CPLX>::type E;
    typedef typename Mfma<R>::acc_t acc_t;
    constexpr int ES = (int)sizeof(E);
    constexpr int NTH = WM * WN * KG * 64;
    static_assert(KG == 1 || (!M3 && !PF && BKK % (4 * KG) == 0), "k-groups: 4M form only");
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int MT = WTM / 16, NT = WTN / 16;
    constexpr int SLAB = (BM + (SH ? 0 : BN)) * BKK; // elements per slab (A then B)
    static_assert(!SH || (AK == BK && BM == BN), "shared image: A and B laid out alike");
    static_assert(MT * 16 == WTM && NT * 16 == WTN, "bad wave tile");
    typedef DmaOperand<AK, BM, BKK, NTH, ES> OpA;
    typedef DmaOperand<BK, BN, BKK, NTH, ES> OpB;
    static_assert(LW == 0 || (AK && BK && !SH && KG == 1 && !PF), "loader waves: K-major operands");
    typedef typename std::conditional<(LW > 0), DmaRowsK<BM, BKK, LW * 64, ES>, NoLoader>::type LdA;
    typedef typename std::conditional<(LW > 0), DmaRowsK<BN, BKK, LW * 64, ES>, NoLoader>::type LdB;
    static_assert(LW == 0 || BKK / 4 >= SP, "loader spread: SP k-steps per slab at most");
    // the double buffer, also the k-groups' reduction area at the end
    constexpr int LDS_E = KG > 1 && BM * BN > 2 * SLAB ? BM * BN : 2 * SLAB;
    __shared__ __attribute__((aligned(16))) E lds[LDS_E]; // the only LDS object

    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    const int ti = wg % p.tm;
    int rest = wg / p.tm;
    const int tj = rest % p.tn;
    rest /= p.tn;
    const int split = rest % p.splits;
    const long bb = rest / p.splits;
    const long m0 = (long)ti * BM, n0 = (long)tj * BN;
    const long k_begin = (long)split * p.kchunk;
    const long k_end = min(p.k, k_begin + p.kchunk);

    const E *A = (const E *)p.a + bb * p.sa_b;
    const E *B = (const E *)p.b + bb * p.sb_b;
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, (short)0, (int)p.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB =
        __builtin_amdgcn_make_buffer_rsrc((void *)B, (short)0, (int)p.b_bytes, 0x00020000);

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    unsigned long long clk0 = 0, rt0 = 0;
    if (p.probe && (bid == 0 || p.probe_all > 0)) {
        clk0 = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
    }
    OpA da;
    OpB db;
    LdA la;
    LdB lb;
    const bool spl = p.split != 0;
    if constexpr (LW == 0) {
        da.init(tid, m0, p.m, p.sa_m, p.sa_k, spl, p.m_lo, p.sa_m_hi);
        db.init(tid, n0, p.n, p.sb_n, p.sb_k, spl, p.n_lo, p.sb_n_hi);
    } else {
        la.init(tid, m0, p.m, p.sa_m, p.sa_k);
        lb.init(tid, n0, p.n, p.sb_n, p.sb_k);
    }
    const bool loader = LW > 0 && wave < LW;

    const int kg = KG > 1 ? wave / (WM * WN) : 0, w2 = KG > 1 ? wave % (WM * WN) : wave;
    const int wm = w2 / WN, wn = w2 % WN;
    const int frow = wm * WTM + (lane & 15), fcol = wn * WTN + (lane & 15), kq = lane >> 4;
    // conjugation: the imaginary parts' sign bit flipped with an integer xor (no FP64 multiply)
    typedef typename std::conditional<sizeof(R) == 8, unsigned long long, unsigned>::type U;
    const U sign = (U)1 << (sizeof(R) * 8 - 1);
    const U ma = p.conja ? sign : 0, mb = p.conjb ? sign : 0;
    auto flip = [](R v, U m) { return __builtin_bit_cast(R, __builtin_bit_cast(U, v) ^ m); };

    constexpr bool G3 = CPLX && M3;
    acc_t accR[MT][NT], accI[MT][NT], acc3[G3 ? MT : 1][G3 ? NT : 1];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) {
            accR[i][j] = acc_t{0, 0, 0, 0};
            accI[i][j] = acc_t{0, 0, 0, 0};
            if constexpr (G3) acc3[i][j] = acc_t{0, 0, 0, 0};
        }

    const long nslab = (k_end - k_begin + BKK - 1) / BKK;
    const char *const base = (const char *)lds;
    constexpr bool CAN_SHARE = AK == BK && BM == BN; // same slab image layout for A and B
    const bool share = SH || (CAN_SHARE && p.same_ab && m0 == n0);
    if (nslab > 0) {
        if constexpr (LW == 0) {
            da.issue(rsA, base, wave, k_begin, k_end, p.sa_k, spl, p.k_lo, p.sa_k_hi);
            if (!share)
                db.issue(rsB, base + BM * BKK * ES, wave, k_begin, k_end, p.sb_k, spl, p.k_lo, p.sb_k_hi);
        } else if (loader) {
            la.issue(rsA, base, wave, k_begin, k_end, p.sa_k, 0, LdA::NI, p.dma_nt);
            if (!share) lb.issue(rsB, base + BM * BKK * ES, wave, k_begin, k_end, p.sb_k, 0, LdB::NI, p.dma_nt);
        }
    }
    // EB (loader waves, SP == 0): the barrier of a slab moved before its last k-step, whose
    // fragments are read first; after the barrier the loaders issue slab s + 2 and every wave
    // reads the next slab's first fragments while the last k-step's MFMAs run -- the MFMA pipe
    // has work the moment the barrier opens (the slab turnaround: 17.9k clocks per slab against
    // the 16.4k its MFMAs take, profiles/r05_gemm_slab_probe.txt)
    constexpr bool EB = LW > 0 && SP == 0;
    static_assert(!EB || (KG == 1 && !PF && !M3 && BKK >= 8), "early barrier: plain 4M / real form");
    if constexpr (EB) {
        auto frag = [&](const E *As_, const E *Bs_, int kk, E (&af)[MT], E (&bf)[NT]) {
#pragma unroll
            for (int i = 0; i < MT; ++i) af[i] = As_[OpA::slot(frow + 16 * i, kk + kq)];
#pragma unroll
            for (int j = 0; j < NT; ++j) bf[j] = Bs_[OpB::slot(fcol + 16 * j, kk + kq)];
        };
        auto mma = [&](E (&af)[MT], E (&bf)[NT]) {
            if constexpr (CPLX) {
#pragma unroll
                for (int i = 0; i < MT; ++i) af[i].y = flip(af[i].y, ma);
#pragma unroll
                for (int j = 0; j < NT; ++j) bf[j].y = flip(bf[j].y, mb);
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(af[i].x, bf[j].x, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].x, bf[j].y, accI[i][j]);
                    }
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(-af[i].y, bf[j].y, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].y, bf[j].x, accI[i][j]);
                    }
            } else {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) accR[i][j] = Mfma<R>::mma(af[i], bf[j], accR[i][j]);
            }
        };
        auto issue_slab = [&](long sl, const char *dst) {
            if (!loader || sl >= nslab) return;
            const long kk0 = k_begin + sl * BKK;
            la.issue(rsA, dst, wave, kk0, k_end, p.sa_k, 0, LdA::NI, p.dma_nt);
            if (!share) lb.issue(rsB, dst + BM * BKK * ES, wave, kk0, k_end, p.sb_k, 0, LdB::NI, p.dma_nt);
        };
        E af0[MT], bf0[NT];
        if (nslab > 0) {
            // slab 0 (issued above) landed everywhere; slab 1 into the other buffer
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            issue_slab(1, base + (size_t)SLAB * ES);
            frag(lds, share ? lds : lds + BM * BKK, 0, af0, bf0);
        }
        for (long s = 0; s < nslab; ++s) {
            const int cur = (int)(s & 1);
            const E *As = lds + cur * SLAB;
            const E *Bs = share ? As : As + BM * BKK;
            mma(af0, bf0);
#pragma unroll
            for (int kk = 4; kk < BKK - 4; kk += 4) {
                E af[MT], bf[NT];
                frag(As, Bs, kk, af, bf);
                mma(af, bf);
            }
            E af3[MT], bf3[NT];
            frag(As, Bs, BKK - 4, af3, bf3);
            if (s + 1 < nslab) {
                // every wave's reads of this slab done and slab s + 1 landed: this buffer is free
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                issue_slab(s + 2, base + (size_t)cur * SLAB * ES);
                const E *An = lds + (cur ^ 1) * SLAB;
                frag(An, share ? An : An + BM * BKK, 0, af0, bf0);
            }
            mma(af3, bf3);
        }
    }
    for (long s = 0; s < (EB ? 0 : nslab); ++s) {
#ifdef SBX_SLAB_PROBE
        // (tools only: workgroup 0 stamps, per wave and slab, the clock before the DMA wait and
        // after the barrier: probe[4096 + (wave * nslab + s) * 2 + 0 / 1])
        const unsigned long long sp0 = __builtin_amdgcn_s_memtime();
#endif
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); // this wave's DMA of slab s landed
        __syncthreads(); // ... and every wave's; the other buffer is free again
#ifdef SBX_SLAB_PROBE
        if (p.probe && bid == 0 && lane == 0) {
            const unsigned long long sp1 = __builtin_amdgcn_s_memtime();
            p.probe[4096 + (wave * nslab + s) * 2] = sp0;
            p.probe[4096 + (wave * nslab + s) * 2 + 1] = sp1;
        }
#endif
        const int cur = (int)(s & 1);
        const char *nb = base + (size_t)(cur ^ 1) * SLAB * ES;
        const long kn = k_begin + (s + 1) * BKK;
        if (LW == 0 && s + 1 < nslab) {
            da.issue(rsA, nb, wave, kn, k_end, p.sa_k, spl, p.k_lo, p.sa_k_hi);
            if (!share)
                db.issue(rsB, nb + BM * BKK * ES, wave, kn, k_end, p.sb_k, spl, p.k_lo, p.sb_k_hi);
        }
        // loader waves: the pieces of k-step q of SP (the next slab's DMA spread over this one's
        // first SP k-steps)
        auto load_part = [&](int q) {
            if constexpr (LW > 0 && SP > 0) {
                if (loader && s + 1 < nslab && q < SP) {
                    la.issue(rsA, nb, wave, kn, k_end, p.sa_k, q * LdA::NI / SP,
                             (q + 1) * LdA::NI / SP, p.dma_nt);
                    if (!share)
                        lb.issue(rsB, nb + BM * BKK * ES, wave, kn, k_end, p.sb_k,
                                 q * LdB::NI / SP, (q + 1) * LdB::NI / SP, p.dma_nt);
                }
            }
        };
        const E *As = lds + cur * SLAB;
        const E *Bs = share ? As : As + BM * BKK;
        if constexpr (PF && CPLX && !M3) {
            E af[2][MT], bf[2][NT];
            auto frag = [&](int kk, E *a_, E *b_) {
#pragma unroll
                for (int i = 0; i < MT; ++i) a_[i] = As[OpA::slot(frow + 16 * i, kk + kq)];
#pragma unroll
                for (int j = 0; j < NT; ++j) b_[j] = Bs[OpB::slot(fcol + 16 * j, kk + kq)];
            };
            frag(0, af[0], bf[0]);
#pragma unroll
            for (int kk = 0; kk < BKK; kk += 4) {
                const int c = (kk / 4) & 1;
                if (kk + 4 < BKK) frag(kk + 4, af[c ^ 1], bf[c ^ 1]);
                E *a = af[c], *b = bf[c];
#pragma unroll
                for (int i = 0; i < MT; ++i) a[i].y = flip(a[i].y, ma);
#pragma unroll
                for (int j = 0; j < NT; ++j) b[j].y = flip(b[j].y, mb);
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(a[i].x, b[j].x, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(a[i].x, b[j].y, accI[i][j]);
                    }
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(-a[i].y, b[j].y, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(a[i].y, b[j].x, accI[i][j]);
                    }
            }
            continue;
        }
#pragma unroll
        for (int kk = 4 * kg; kk < BKK; kk += 4 * KG) {
            load_part(kk / 4);
            E af[MT], bf[NT];
#pragma unroll
            for (int i = 0; i < MT; ++i) af[i] = As[OpA::slot(frow + 16 * i, kk + kq)];
#pragma unroll
            for (int j = 0; j < NT; ++j) bf[j] = Bs[OpB::slot(fcol + 16 * j, kk + kq)];
            if constexpr (G3) {
                // accR = P1, accI = P2, acc3 = P3
                R as[MT], bs[NT];
#pragma unroll
                for (int i = 0; i < MT; ++i) {
                    af[i].y = flip(af[i].y, ma);
                    as[i] = af[i].x + af[i].y;
                }
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    bf[j].y = flip(bf[j].y, mb);
                    bs[j] = bf[j].x + bf[j].y;
                }
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(af[i].x, bf[j].x, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].y, bf[j].y, accI[i][j]);
                        acc3[i][j] = Mfma<R>::mma(as[i], bs[j], acc3[i][j]);
                    }
            } else if constexpr (CPLX) {
#pragma unroll
                for (int i = 0; i < MT; ++i) af[i].y = flip(af[i].y, ma);
#pragma unroll
                for (int j = 0; j < NT; ++j) bf[j].y = flip(bf[j].y, mb);
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(af[i].x, bf[j].x, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].x, bf[j].y, accI[i][j]);
                    }
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) {
                        accR[i][j] = Mfma<R>::mma(-af[i].y, bf[j].y, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].y, bf[j].x, accI[i][j]);
                    }
            } else {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j) accR[i][j] = Mfma<R>::mma(af[i], bf[j], accR[i][j]);
            }
        }
    }

    if constexpr (KG > 1) {
        // sum the k-groups' partial tiles into group 0, one group at a time through the (now
        // free) slab buffers, in group order
        static_assert(BM * BN <= LDS_E, "k-group reduction: LDS too small");
        E *red = lds;
#pragma unroll
        for (int g = 1; g < KG; ++g) {
            __syncthreads(); // every wave is done with the slab buffers / the previous round
            if (kg == g) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            E v;
                            if constexpr (CPLX) v = E{accR[i][j][r], accI[i][j][r]};
                            else v = accR[i][j][r];
                            red[(((w2 * MT + i) * NT + j) * 4 + r) * 64 + lane] = v;
                        }
            }
            __syncthreads();
            if (kg == 0) {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < NT; ++j)
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const E v = red[(((w2 * MT + i) * NT + j) * 4 + r) * 64 + lane];
                            if constexpr (CPLX) {
                                accR[i][j][r] += v.x;
                                accI[i][j][r] += v.y;
                            } else {
                                accR[i][j][r] += v;
                            }
                        }
            }
        }
        if (kg != 0) return;
    }
    if (p.probe && bid == 0 && tid == 0) {
        const unsigned long long clk1 = __builtin_amdgcn_s_memtime();
        const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
        if (p.probe_all < 0) {
            // the library's clock meter (tune "gemm.clock"): summed over launches with vector
            // atomics -- shader clock cycles, 100 MHz reference ticks, launches
            atomicAdd(&p.probe[0], clk1 - clk0);
            atomicAdd(&p.probe[1], rt1 - rt0);
            atomicAdd(&p.probe[2], 1ull);
        } else {
            p.probe[0] = clk1 - clk0; // shader clock cycles
            p.probe[1] = rt1 - rt0;   // 100 MHz reference ticks
        }
    }
    if (p.probe && p.probe_all > 0 && tid == 0) {
        p.probe[2 + 3 * bid] = rt0;
        p.probe[3 + 3 * bid] = __builtin_amdgcn_s_memrealtime();
    }
    const int ccol = lane & 15;
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const long gi = m0 + wm * WTM + 16 * i + Mfma<R>::row(lane, r);
                const long gj = n0 + wn * WTN + 16 * j + ccol;
                if (gi >= p.m || gj >= p.n) continue;
                R vr = accR[i][j][r];
                R vi = CPLX ? accI[i][j][r] : R(0);
                if constexpr (G3) {
                    const R p1 = vr, p2 = vi;
                    vr = p1 - p2;
                    vi = acc3[i][j][r] - p1 - p2;
                }
                if (p.splits == 1) {
                    R *cptr = (R *)((E *)p.c + bb * p.sc_b + c_off(p, gi, gj));
                    epilogue_store<R>(cptr, vr, vi, p, CPLX);
                } else {
                    E *w = (E *)p.work + (((long)split * p.batch + bb) * p.n + gj) * p.m + gi;
                    if constexpr (CPLX)
                        *w = E{vr, vi};
                    else
                        *w = vr;
                }
            }
}

// ---------------------------------------------------------------------------------------------
// Wave-private slabs, for a tensor contracted with itself with one output tile per batch entry
// (same_ab, m = n <= BM: the chain's y^H y correlator, TSnsN with m = n = 48).  Every wave of the
// workgroup owns the whole BM x BM tile over its own contiguous part of the workgroup's k-chunk
// and stages that part by LDS-DMA into a RING-deep slab ring of its own (A only: B's fragments are
// read from the same image), so the main loop has no barrier at all -- a wave waits only on its
// own DMA (vmcnt) and its own LDS reads.  Round-4 measurement: a workgroup-wide slab with a
// barrier per slab kept the MFMA pipe 67 % busy (every workgroup of a CU reaching its barrier and
// DMA wait in lockstep).  The waves' partial tiles are summed through LDS in wave order at the end
// (deterministic), then written like the other kernels (split-K partial or C).
// ---------------------------------------------------------------------------------------------
// FUSE: the split-K partials are summed by the last workgroup of each batch entry to finish
// (an agent-scope counter per entry, zeroed before the launch): it adds the partials of all
// splits in split order -- the same order and arithmetic as splitk_reduce_kernel, so the result
// does not depend on which workgroup finishes last -- and writes C; no second kernel
template <typename R, bool CPLX, bool AK, int BM, int BKK, int KG, int RING, bool FUSE = false>
__global__ void __launch_bounds__(KG * 64) gemm_wave_kernel(const GemmKArgs p, unsigned *counters) {
    typedef typename Elem<R, CPLX>::type E;
    typedef typename Mfma<R>::acc_t acc_t;
    constexpr int ES = (int)sizeof(E);
    constexpr int MT = BM / 16;
    static_assert(MT * 16 == BM && RING >= 2 && BKK % 4 == 0, "wave kernel shape");
    typedef DmaOperand<AK, BM, BKK, 64, ES> Op;
    constexpr int SLAB = BM * BKK;
    constexpr int NI = Op::NI; // DMA instructions per slab
    static_assert(NI * (RING - 1) <= 60, "vmcnt range");
    // the rings; at the end, the KG / 2 partial tiles of the first round of the tree sum
    constexpr int RED_E = (KG / 2 > 1 ? KG / 2 : 1) * BM * BM;
    constexpr int LDS_E = KG * RING * SLAB > RED_E ? KG * RING * SLAB : RED_E;
    __shared__ __attribute__((aligned(16))) E lds[LDS_E];

    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    const int split = wg % p.splits;
    const long bb = wg / p.splits;
    const long k_begin = (long)split * p.kchunk;
    const long k_end = min(p.k, k_begin + p.kchunk);
    const E *A = (const E *)p.a + bb * p.sa_b;
    const __amdgpu_buffer_rsrc_t rsA =
        __builtin_amdgcn_make_buffer_rsrc((void *)A, (short)0, (int)p.a_bytes, 0x00020000);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const bool spl = p.split != 0;
    Op da;
    da.init(lane, 0, p.m, p.sa_m, p.sa_k, spl, p.m_lo, p.sa_m_hi);
    // this wave's slabs [s0, s1) of the workgroup's chunk
    const long nsl = (k_end - k_begin + BKK - 1) / BKK;
    const long per = (nsl + KG - 1) / KG;
    const long s0 = min(nsl, (long)wave * per), s1 = min(nsl, s0 + per);
    const char *const mine = (const char *)lds + (size_t)wave * RING * SLAB * ES;
    auto issue = [&](long sl) {
        da.issue(rsA, mine + (size_t)((sl - s0) % RING) * SLAB * ES, 0, k_begin + sl * BKK, k_end,
                 p.sa_k, spl, p.k_lo, p.sa_k_hi);
    };
    typedef typename std::conditional<sizeof(R) == 8, unsigned long long, unsigned>::type U;
    const U sign = (U)1 << (sizeof(R) * 8 - 1);
    const U ma = p.conja ? sign : 0, mb = p.conjb ? sign : 0;
    auto flip = [](R v, U m) { return __builtin_bit_cast(R, __builtin_bit_cast(U, v) ^ m); };
    acc_t accR[MT][MT], accI[MT][MT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) {
            accR[i][j] = acc_t{0, 0, 0, 0};
            accI[i][j] = acc_t{0, 0, 0, 0};
        }
    const int frow = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int r = 0; r < RING - 1; ++r)
        if (s0 + r < s1) issue(s0 + r);
    for (long sl = s0; sl < s1; ++sl) {
        const long sn = sl + RING - 1;
        if (sn < s1) {
            // the slot of slab sn was last read for slab sl - 1: those LDS reads have returned
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            issue(sn);
        }
        // slab sl landed: the DMA of the slabs issued after it may stay in flight
        const long after = min((long)(RING - 1), s1 - 1 - sl);
        if constexpr (RING >= 3) {
            if (after >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NI) : "memory");
            else if (after == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        } else {
            if (after >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI) : "memory");
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const E *As = (const E *)(mine + (size_t)((sl - s0) % RING) * SLAB * ES);
#pragma unroll
        for (int kk = 0; kk < BKK; kk += 4) {
            E af[MT], bf[MT];
#pragma unroll
            for (int i = 0; i < MT; ++i) af[i] = As[Op::slot(frow + 16 * i, kk + kq)];
#pragma unroll
            for (int j = 0; j < MT; ++j) bf[j] = af[j]; // the same image: B's fragment = A's
            if constexpr (CPLX) {
#pragma unroll
                for (int i = 0; i < MT; ++i) af[i].y = flip(af[i].y, ma);
#pragma unroll
                for (int j = 0; j < MT; ++j) bf[j].y = flip(bf[j].y, mb);
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) {
                        accR[i][j] = Mfma<R>::mma(af[i].x, bf[j].x, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].x, bf[j].y, accI[i][j]);
                    }
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) {
                        accR[i][j] = Mfma<R>::mma(-af[i].y, bf[j].y, accR[i][j]);
                        accI[i][j] = Mfma<R>::mma(af[i].y, bf[j].x, accI[i][j]);
                    }
            } else {
#pragma unroll
                for (int i = 0; i < MT; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) accR[i][j] = Mfma<R>::mma(af[i], bf[j], accR[i][j]);
            }
        }
    }
    // the waves' partial tiles summed into wave 0 by a fixed binary tree (wave w + step into wave
    // w at each level), so the order, and the result, do not depend on timing
#pragma unroll
    for (int step = 1; step < KG; step *= 2) {
        __syncthreads();
        E *red = lds + (size_t)(wave / (2 * step)) * BM * BM;
        if (wave % (2 * step) == step) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < MT; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        E v;
                        if constexpr (CPLX) v = E{accR[i][j][r], accI[i][j][r]};
                        else v = accR[i][j][r];
                        red[((i * MT + j) * 4 + r) * 64 + lane] = v;
                    }
        }
        __syncthreads();
        if (wave % (2 * step) == 0) {
#pragma unroll
            for (int i = 0; i < MT; ++i)
#pragma unroll
                for (int j = 0; j < MT; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const E v = red[((i * MT + j) * 4 + r) * 64 + lane];
                        if constexpr (CPLX) {
                            accR[i][j][r] += v.x;
                            accI[i][j][r] += v.y;
                        } else {
                            accR[i][j][r] += v;
                        }
                    }
        }
    }
    const bool fuse = FUSE && p.splits > 1;
    if (wave != 0 && !fuse) return;
    if (wave == 0) {
#pragma unroll
        for (int i = 0; i < MT; ++i)
#pragma unroll
            for (int j = 0; j < MT; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const long gi = 16 * i + Mfma<R>::row(lane, r);
                    const long gj = 16 * j + frow;
                    if (gi >= p.m || gj >= p.n) continue;
                    const R vr = accR[i][j][r];
                    const R vi = CPLX ? accI[i][j][r] : R(0);
                    if (p.splits == 1) {
                        R *cptr = (R *)((E *)p.c + bb * p.sc_b + c_off(p, gi, gj));
                        epilogue_store<R>(cptr, vr, vi, p, CPLX);
                    } else {
                        E *w = (E *)p.work + (((long)split * p.batch + bb) * p.n + gj) * p.m + gi;
                        E v;
                        if constexpr (CPLX) v = E{vr, vi};
                        else v = vr;
                        if constexpr (FUSE) {
                            // write-through (sc1) stores: the partial reaches memory without a
                            // release fence (no L2 write-back)
                            if constexpr (sizeof(E) == 8)
                                __hip_atomic_store((unsigned long long *)w, __builtin_bit_cast(unsigned long long, v),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            else if constexpr (sizeof(E) == 4)
                                __hip_atomic_store((unsigned *)w, __builtin_bit_cast(unsigned, v),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            else {
                                const R re = vr, im = vi;
                                __hip_atomic_store((unsigned long long *)w, __builtin_bit_cast(unsigned long long, re),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                                __hip_atomic_store((unsigned long long *)w + 1, __builtin_bit_cast(unsigned long long, im),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            }
                        } else {
                            *w = v;
                        }
                    }
                }
    }
    if constexpr (FUSE) {
        if (!fuse) return;
        // the partial published (wave 0's stores drained, then one agent-scope add on the batch
        // entry's counter); the workgroup whose add comes last sums the entry's partials of all
        // splits in split order -- the arithmetic of splitk_reduce_kernel, so the result does not
        // depend on which workgroup finishes last -- writes C and resets the counter for the next
        // launch on this stream
        __shared__ int last_s;
        if (wave == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (lane == 0) {
                const unsigned old = __hip_atomic_fetch_add(counters + bb, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                last_s = old == (unsigned)p.splits - 1;
                if (old == (unsigned)p.splits - 1) {
                    // one agent-scope acquire (this CU's L1 dropped) before the workgroup's loads
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                }
            }
        }
        __syncthreads();
        if (!last_s) return;
        const long mn = p.m * p.n, sstride = p.batch * mn;
        const E *wb = (const E *)p.work + bb * mn;
        for (long e = tid; e < mn; e += KG * 64) {
            const long gi = e % p.m, gj = e / p.m;
            R sr = 0, si = 0;
            for (int sp = 0; sp < p.splits; ++sp) {
                const E v = wb[(long)sp * sstride + e];
                if constexpr (CPLX) {
                    sr += v.x;
                    si += v.y;
                } else {
                    sr += v;
                }
            }
            R *cptr = (R *)((E *)p.c + bb * p.sc_b + c_off(p, gi, gj));
            epilogue_store<R>(cptr, sr, si, p, CPLX);
        }
        if (tid == 0) __hip_atomic_store(counters + bb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// ---------------------------------------------------------------------------------------------
// Skinny products: an output dimension of a few rows gets no 16x16 MFMA padding (the
// reference's dot / gemv shortcuts for m = 1 / n = 1, blas.h:686-800; the inner-product and
// update shapes its tests/dist.cpp:160-195 times).
//  * gemm_dot_kernel, m, n <= 4 (inner products, long k): one workgroup per (batch entry,
//    k-chunk); lanes stride over k keeping all m x n sums in registers, which are reduced across
//    the wave (xor shuffles) and the workgroup (LDS) in a fixed order; split-K partials are summed
//    by splitk_reduce_kernel in split order -- deterministic.
//  * gemm_rows_kernel, n <= 16 (updates and matrix-vector products, long m): one lane per (row,
//    batch entry) keeps its row's n outputs; the lanes of a wave read 64 consecutive rows of A.
//    m <= 16 with a long n runs as the transposed problem (C^T = op(B)^T op(A)^T).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ double2 madd(double2 c, double2 a, double2 b) {
    return double2{c.x + a.x * b.x - a.y * b.y, c.y + a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ float2 madd(float2 c, float2 a, float2 b) {
    return float2{c.x + a.x * b.x - a.y * b.y, c.y + a.x * b.y + a.y * b.x};
}
__device__ __forceinline__ double madd(double c, double a, double b) { return c + a * b; }
__device__ __forceinline__ float madd(float c, float a, float b) { return c + a * b; }
template <typename E> __device__ __forceinline__ E xor_sum(E v, int m) {
    if constexpr (std::is_same<E, double2>::value || std::is_same<E, float2>::value)
        return E{v.x + __shfl_xor(v.x, m), v.y + __shfl_xor(v.y, m)};
    else
        return v + __shfl_xor(v, m);
}
template <typename R, bool CPLX> __device__ __forceinline__ void store_out(const GemmKArgs &p, long bb, long gi, long gj, typename Elem<R, CPLX>::type v) {
    if constexpr (CPLX)
        epilogue_store<R>((R *)((typename Elem<R, CPLX>::type *)p.c + bb * p.sc_b + gi * p.sc_m + gj * p.sc_n), v.x, v.y, p, true);
    else
        epilogue_store<R>((R *)p.c + bb * p.sc_b + gi * p.sc_m + gj * p.sc_n, v, R(0), p, false);
}

template <typename R, bool CPLX, int MM, int NN>
__global__ void __launch_bounds__(256) gemm_dot_kernel(const GemmKArgs p) {
    typedef typename Elem<R, CPLX>::type E;
    const int split = (int)(blockIdx.x % (unsigned)p.splits);
    const long bb = blockIdx.x / (unsigned)p.splits;
    const long k0 = (long)split * p.kchunk, k1 = min(p.k, k0 + p.kchunk);
    const E *A = (const E *)p.a + bb * p.sa_b, *B = (const E *)p.b + bb * p.sb_b;
    const int m = (int)p.m, n = (int)p.n;
    E acc[MM][NN];
#pragma unroll
    for (int i = 0; i < MM; ++i)
#pragma unroll
        for (int j = 0; j < NN; ++j) acc[i][j] = zero_elem<E>();
    // four k per thread per pass, all their loads issued before the first product
    constexpr int U = 4;
    for (long k = k0 + threadIdx.x; k < k1; k += 256 * U) {
        E a[U][MM], b[U][NN];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long kk = k + 256L * u;
            const bool in = kk < k1;
#pragma unroll
            for (int i = 0; i < MM; ++i)
                a[u][i] = in && i < m ? conj_if(A[i * p.sa_m + kk * p.sa_k], p.conja) : zero_elem<E>();
#pragma unroll
            for (int j = 0; j < NN; ++j)
                b[u][j] = in && j < n ? conj_if(B[kk * p.sb_k + j * p.sb_n], p.conjb) : zero_elem<E>();
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
            for (int i = 0; i < MM; ++i)
#pragma unroll
                for (int j = 0; j < NN; ++j) acc[i][j] = madd(acc[i][j], a[u][i], b[u][j]);
    }
    __shared__ E red[4][MM * NN];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < MM; ++i)
#pragma unroll
        for (int j = 0; j < NN; ++j) {
            E v = acc[i][j];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v = xor_sum(v, o);
            if (lane == 0) red[wave][i * NN + j] = v;
        }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < m * n) {
        const int i = t % m, j = t / m;
        E v = red[0][i * NN + j];
#pragma unroll
        for (int w = 1; w < 4; ++w) {
            if constexpr (CPLX) {
                v.x += red[w][i * NN + j].x;
                v.y += red[w][i * NN + j].y;
            } else {
                v += red[w][i * NN + j];
            }
        }
        if (p.splits == 1)
            store_out<R, CPLX>(p, bb, i, j, v);
        else
            ((E *)p.work)[(((long)split * p.batch + bb) * p.n + j) * p.m + i] = v;
    }
}

template <typename R, bool CPLX, int NN>
__global__ void __launch_bounds__(256) gemm_rows_kernel(const GemmKArgs p) {
    typedef typename Elem<R, CPLX>::type E;
    const long total = p.m * p.batch;
    const int n = (int)p.n;
    for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256L) {
        const long i = idx % p.m, bb = idx / p.m;
        const E *A = (const E *)p.a + bb * p.sa_b + i * p.sa_m;
        const E *B = (const E *)p.b + bb * p.sb_b;
        E acc[NN];
#pragma unroll
        for (int j = 0; j < NN; ++j) acc[j] = zero_elem<E>();
        for (long k = 0; k < p.k; ++k) {
            const E a = conj_if(A[k * p.sa_k], p.conja);
#pragma unroll
            for (int j = 0; j < NN; ++j)
                if (j < n) acc[j] = madd(acc[j], a, conj_if(B[k * p.sb_k + j * p.sb_n], p.conjb));
        }
#pragma unroll
        for (int j = 0; j < NN; ++j)
            if (j < n) store_out<R, CPLX>(p, bb, i, j, acc[j]);
    }
}

// Small outputs and tall-skinny products straight from global memory into MFMA fragments: one
// wave per (16 x 16 output tile, batch entry, k-split), no LDS.  The reference's dist.cpp
// xgemm_batch_strided sweep (tests/dist.cpp:160-195, the Krylov inner products m = n <= 64 with
// k = the local volume, and the updates m = volume, n = k <= 64) ran through the 64x64 LDS-DMA
// tiles (99 % MFMA padding at m = n = 8: 0.22 TFLOP/s) or one lane per output row walking k
// serially (the updates: 1.2 TFLOP/s at n = k = 8), 10-50x under the HBM roofline of those
// shapes.  Lane (r, q) of a k-step reads A(m0 + r, k + q) and B(k + q, n0 + r) through buffer
// descriptors (an offset past the range reads zero: rows, columns and k past the ends), UK
// k-steps per group, the next group's loads issued before the current group's MFMAs; the
// split-K partials go to the work array and the split-K reduce sums them in split order.
// KP (8-byte elements, k even): lane q of the k-steps u, u + 1 of a group takes the pair k0 + 4u +
// 2q, + 1 (the same permutation of a group's k for A and B), so an operand with unit k stride
// reads each pair with one 16-byte load: 64 contiguous bytes per row and instruction instead of
// 32 (pair_a / pair_b; the other operand reads the pair's two elements)
// NT > 1: the wave computes NT adjacent 16 x 16 tiles of a row of tiles (columns n0 .. n0 + 16 NT),
// so its A fragments are loaded once for NT tiles (the tall-skinny updates n = 32 / 64: A was
// re-read n / 16 times)
template <typename R, bool CPLX, int UK, bool KP = false, int NT = 1>
__global__ void __launch_bounds__(256) gemm_frag_kernel(const GemmKArgs p) {
    typedef typename Elem<R, CPLX>::type E;
    typedef typename Mfma<R>::acc_t acc_t;
    constexpr int ES = (int)sizeof(E);
    const int lane = threadIdx.x & 63;
    const long item = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    const long items = (long)p.tm * p.tn * p.batch * p.splits;
    if (item >= items) return; // whole waves only: MFMA needs all 64 lanes
    const int split = (int)(item % p.splits);
    long rest = item / p.splits;
    const long ti = rest % p.tm;
    rest /= p.tm;
    const long tj = rest % p.tn;
    const long bb = rest / p.tn;
    const long m0 = ti * 16, n0 = tj * 16 * NT;
    const long k_begin = (long)split * p.kchunk, k_end = min(p.k, k_begin + p.kchunk);
    const __amdgpu_buffer_rsrc_t rsA = __builtin_amdgcn_make_buffer_rsrc(
        (void *)((const E *)p.a + bb * p.sa_b), (short)0, (int)p.a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsB = __builtin_amdgcn_make_buffer_rsrc(
        (void *)((const E *)p.b + bb * p.sb_b), (short)0, (int)p.b_bytes, 0x00020000);
    const int r = lane & 15, q = lane >> 4;
    const bool okA = m0 + r < p.m;
    const long baseA = (m0 + r) * p.sa_m;
    bool okB[NT];
    long baseB[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        okB[j] = n0 + 16 * j + r < p.n;
        baseB[j] = (n0 + 16 * j + r) * p.sb_n;
    }
    typedef typename std::conditional<sizeof(R) == 8, unsigned long long, unsigned>::type U;
    const U sign = (U)1 << (sizeof(R) * 8 - 1);
    const U ma = p.conja ? sign : 0, mb = p.conjb ? sign : 0;
    auto flip = [](R v, U m) { return __builtin_bit_cast(R, __builtin_bit_cast(U, v) ^ m); };
    static_assert(!KP || (ES == 8 && UK % 2 == 0), "k pairs: 8-byte elements, even UK");
    auto load = [&](long k0, E (&a)[UK], E (&b)[NT][UK]) {
        if constexpr (KP) {
#pragma unroll
            for (int u = 0; u < UK; u += 2) {
                const long kk = k0 + 4 * u + 2 * q; // (k_end even: kk + 1 is in range with kk)
                const bool kin = kk < k_end;
                auto pair = [&](__amdgpu_buffer_rsrc_t rs, bool ok, bool paired, long base, long sk,
                                E &lo, E &hi) {
                    if (paired) {
                        const auto v = __builtin_amdgcn_raw_buffer_load_b128(
                            rs, ok && kin ? (unsigned)((base + kk) * ES) : 0x80000000u, 0, 0);
                        typedef typename std::conditional<sizeof(R) == 8, double, float2>::type H;
                        struct Two { H lo, hi; };
                        const Two t = __builtin_bit_cast(Two, v);
                        lo = __builtin_bit_cast(E, t.lo);
                        hi = __builtin_bit_cast(E, t.hi);
                    } else {
                        lo = buf_load<E>(rs, ok && kin ? (unsigned)((base + kk * sk) * ES) : 0x80000000u);
                        hi = buf_load<E>(rs, ok && kin ? (unsigned)((base + (kk + 1) * sk) * ES) : 0x80000000u);
                    }
                };
                pair(rsA, okA, p.pair_a != 0, baseA, p.sa_k, a[u], a[u + 1]);
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    pair(rsB, okB[j], p.pair_b != 0, baseB[j], p.sb_k, b[j][u], b[j][u + 1]);
            }
        } else {
#pragma unroll
            for (int u = 0; u < UK; ++u) {
                const long kk = k0 + 4 * u + q;
                const bool kin = kk < k_end;
                a[u] = buf_load<E>(rsA, okA && kin ? (unsigned)((baseA + kk * p.sa_k) * ES) : 0x80000000u);
#pragma unroll
                for (int j = 0; j < NT; ++j)
                    b[j][u] = buf_load<E>(rsB, okB[j] && kin ? (unsigned)((baseB[j] + kk * p.sb_k) * ES) : 0x80000000u);
            }
        }
    };
    acc_t accR[NT], accI[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
        accR[j] = acc_t{0, 0, 0, 0};
        accI[j] = acc_t{0, 0, 0, 0};
    }
    E a[UK], b[NT][UK], an[UK], bn[NT][UK];
    if (k_begin < k_end) load(k_begin, a, b);
    for (long k = k_begin; k < k_end; k += 4 * UK) {
        if (k + 4 * UK < k_end) load(k + 4 * UK, an, bn);
#pragma unroll
        for (int u = 0; u < UK; ++u) {
            if constexpr (CPLX) {
                const R ar = a[u].x, ai = flip(a[u].y, ma);
#pragma unroll
                for (int j = 0; j < NT; ++j) {
                    const R br = b[j][u].x, bi = flip(b[j][u].y, mb);
                    accR[j] = Mfma<R>::mma(ar, br, accR[j]);
                    accI[j] = Mfma<R>::mma(ar, bi, accI[j]);
                    accR[j] = Mfma<R>::mma(-ai, bi, accR[j]);
                    accI[j] = Mfma<R>::mma(ai, br, accI[j]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < NT; ++j) accR[j] = Mfma<R>::mma(a[u], b[j][u], accR[j]);
            }
        }
#pragma unroll
        for (int u = 0; u < UK; ++u) {
            a[u] = an[u];
#pragma unroll
            for (int j = 0; j < NT; ++j) b[j][u] = bn[j][u];
        }
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const long gi = m0 + Mfma<R>::row(lane, i), gj = n0 + 16 * j + r;
            if (gi >= p.m || gj >= p.n) continue;
            const R vr = accR[j][i], vi = CPLX ? accI[j][i] : R(0);
            if (p.splits == 1) {
                epilogue_store<R>((R *)((E *)p.c + bb * p.sc_b + gi * p.sc_m + gj * p.sc_n), vr, vi, p, CPLX);
            } else {
                E *w = (E *)p.work + (((long)split * p.batch + bb) * p.n + gj) * p.m + gi;
                if constexpr (CPLX)
                    *w = E{vr, vi};
                else
                    *w = vr;
            }
        }
    }
}

// C = alpha * sum_s W[s] + beta * C, summed in split order (deterministic)
template <typename R, bool CPLX>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const GemmKArgs p) {
    typedef typename Elem<R, CPLX>::type E;
    const long total = p.batch * p.n * p.m;
    const long slab = total;
    for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
         idx += (long)gridDim.x * blockDim.x) {
        const long gi = idx % p.m;
        const long gj = (idx / p.m) % p.n;
        const long bb = idx / (p.m * p.n);
        const E *w = (const E *)p.work + idx;
        R sr = 0, si = 0;
        for (int s = 0; s < p.splits; ++s) {
            if constexpr (CPLX) {
                E v = w[s * slab];
                sr += v.x;
                si += v.y;
            } else {
                sr += w[s * slab];
            }
        }
        R *cptr = (R *)((E *)p.c + bb * p.sc_b + c_off(p, gi, gj));
        epilogue_store<R>(cptr, sr, si, p, CPLX);
    }
}

// C = beta * C (k == 0)
template <typename R, bool CPLX>
__global__ void __launch_bounds__(256) scale_c_kernel(const GemmKArgs p) {
    typedef typename Elem<R, CPLX>::type E;
    const long total = p.batch * p.n * p.m;
    for (long idx = blockIdx.x * (long)blockDim.x + threadIdx.x; idx < total;
         idx += (long)gridDim.x * blockDim.x) {
        const long gi = idx % p.m;
        const long gj = (idx / p.m) % p.n;
        const long bb = idx / (p.m * p.n);
        R *cptr = (R *)((E *)p.c + bb * p.sc_b + c_off(p, gi, gj));
        GemmKArgs q = p;
        q.alpha_re = 0;
        q.alpha_im = 0;
        epilogue_store<R>(cptr, R(0), R(0), q, CPLX);
    }
}

/// Grid shape, split-K factor, descriptor ranges and the split-K workspace of one launch
/// (`splits` <= 0 picks the split-K factor so that ~target_wgs workgroups are in flight)
template <typename E>
long prepare_launch(GemmKArgs &p, int BM, int BN, int BKK, long splits, long target_wgs,
                    Scratch &work, int device) {
    p.tm = (int)((p.m + BM - 1) / BM);
    p.tn = (int)((p.n + BN - 1) / BN);
    const long tiles = (long)p.tm * p.tn * p.batch;
    if (splits <= 0) {
        splits = 1;
        if (tiles < target_wgs) {
            splits = (target_wgs + tiles - 1) / tiles;
            const long max_splits = std::max(1L, p.k / 256); // keep >= 256-deep chunks
            splits = std::min(splits, max_splits);
        }
    }
    // largest element offset of a split (or plain) group index
    auto ext = [](long n, long lo, long st, long st_hi) {
        return (n / lo - 1) * std::labs(st_hi) + (lo - 1) * std::labs(st);
    };
    const long ea = p.split ? (ext(p.m, p.m_lo, p.sa_m, p.sa_m_hi) +
                               ext(p.k, p.k_lo, p.sa_k, p.sa_k_hi) + 1) * (long)sizeof(E)
                            : ((p.m - 1) * std::labs(p.sa_m) + (p.k - 1) * std::labs(p.sa_k) + 1) *
                                  (long)sizeof(E);
    const long eb = p.split ? (ext(p.k, p.k_lo, p.sb_k, p.sb_k_hi) +
                               ext(p.n, p.n_lo, p.sb_n, p.sb_n_hi) + 1) * (long)sizeof(E)
                            : ((p.k - 1) * std::labs(p.sb_k) + (p.n - 1) * std::labs(p.sb_n) + 1) *
                                  (long)sizeof(E);
    if (ea >= 0x7fffffffL || eb >= 0x7fffffffL || p.sa_m < 0 || p.sa_k < 0 || p.sb_k < 0 ||
        p.sb_n < 0 || p.sa_m_hi < 0 || p.sa_k_hi < 0 || p.sb_k_hi < 0 || p.sb_n_hi < 0)
        throw Error("gemm: operand batch entries of 2 GiB or more are not supported yet");
    p.a_bytes = (unsigned)ea;
    p.b_bytes = (unsigned)eb;
    long kchunk = (p.k + splits - 1) / splits;
    kchunk = (kchunk + BKK - 1) / BKK * BKK;
    splits = std::max(1L, (p.k + kchunk - 1) / kchunk);
    p.splits = (int)splits;
    p.kchunk = kchunk;
    p.work = nullptr;
    if (splits > 1) {
        work = Scratch(sizeof(E) * splits * p.batch * p.m * p.n, device);
        p.work = work.ptr;
    }
    const long nwg = tiles * splits;
    if (nwg > 0x7fffffffL) throw Error("gemm: grid too large");
    return nwg;
}

template <typename R, bool CPLX>
void launch_reduce(const GemmKArgs &p, hipStream_t stream) {
    if (p.splits <= 1) return;
    const long total = p.batch * p.m * p.n;
    const long blocks = std::min((total + 255) / 256, 4096L);
    KernelTimer timer("gemm_splitk_reduce", stream);
    hipLaunchKernelGGL((splitk_reduce_kernel<R, CPLX>), dim3((unsigned)blocks), dim3(256), 0,
                       stream, p);
    SBX_HIP_CHECK(hipGetLastError());
}

/// Launch one tile configuration of the register-staged kernel
template <typename R, bool CPLX, bool AK, bool BK, int BM, int BN, int BKK, int WM, int WN>
void launch_tiled_cfg(const GemmKArgs &p0, int device, hipStream_t stream, long splits = 0,
                      long target_wgs = 1024) {
    GemmKArgs p = p0;
    Scratch work;
    const long nwg = prepare_launch<typename Elem<R, CPLX>::type>(p, BM, BN, BKK, splits,
                                                                   target_wgs, work, device);
    // "gemm_total": one event pair around the GEMM launch and its split-K reduce (the bench's
    // roofline timer: two event records per GEMM instead of four)
    KernelTimer total("gemm_total", stream);
    {
        KernelTimer timer("gemm", stream);
        hipLaunchKernelGGL((gemm_kernel<R, CPLX, AK, BK, BM, BN, BKK, WM, WN>),
                           dim3((unsigned)nwg), dim3(WM * WN * 64), 0, stream, p);
        SBX_HIP_CHECK(hipGetLastError());
    }
    launch_reduce<R, CPLX>(p, stream);
}

/// The clock meter of the LDS-DMA kernel (tune key "gemm.clock" > 0): workgroup 0 of every
/// launch adds its s_memtime (shader clock) and s_memrealtime (100 MHz) spans and a launch count
/// into three counters per device, read back by "gemm.clock_cycles" / "gemm.clock_ticks" /
/// "gemm.clock_launches" -- the clock the GEMMs ran at, so that a slower box can be told apart
/// from a slower kernel (one thread's three atomics per launch)
static unsigned long long *g_clock_meter[64];
static std::mutex g_clock_mu;

unsigned long long *gemm_clock_meter(int device) {
    if (g_gemm_tune.clock <= 0 || device < 0 || device >= 64) return nullptr;
    std::lock_guard<std::mutex> lock(g_clock_mu);
    if (!g_clock_meter[device]) {
        void *ptr = nullptr;
        SBX_HIP_CHECK(hipMalloc(&ptr, 3 * sizeof(unsigned long long)));
        SBX_HIP_CHECK(hipMemset(ptr, 0, 3 * sizeof(unsigned long long)));
        g_clock_meter[device] = (unsigned long long *)ptr;
    }
    return g_clock_meter[device];
}

void clock_read_impl(int device, unsigned long long out[3], bool reset) {
    out[0] = out[1] = out[2] = 0;
    std::lock_guard<std::mutex> lock(g_clock_mu);
    if (device < 0 || device >= 64 || !g_clock_meter[device]) return;
    SBX_HIP_CHECK(hipDeviceSynchronize());
    SBX_HIP_CHECK(hipMemcpy(out, g_clock_meter[device], 3 * sizeof(unsigned long long),
                            hipMemcpyDeviceToHost));
    if (reset) SBX_HIP_CHECK(hipMemset(g_clock_meter[device], 0, 3 * sizeof(unsigned long long)));
}

/// Launch one tile configuration of the LDS-DMA kernel
template <typename R, bool CPLX, bool AK, bool BK, int BM, int BN, int BKK, int WM, int WN,
          bool ALLOW_M3 = true, bool PF = false, int KG = 1, bool SH = false, int LW = 0, int SP = 1>
void launch_dma_cfg(const GemmKArgs &p0, int device, hipStream_t stream, long splits = 0,
                    long target_wgs = 1024) {
    // complex: the 4-multiplication form unless the 3-multiplication form is asked for (config
    // 2: 1.53 -> 1.20 ms, but only a normwise error bound: near-real products lose the imaginary
    // part's relative accuracy, ADVICE r1 / tests/test_gpu_golden.py)
    const bool m3 = CPLX && g_gemm_tune.m3 > 0;
    GemmKArgs p = p0;
    Scratch work;
    if (g_gemm_tune.splits > 0) splits = g_gemm_tune.splits;
    p.dma_nt = g_gemm_tune.dma_nt;
    p.same_ab = g_gemm_tune.share_ab && p.a == p.b && p.m == p.n && p.sa_m == p.sb_n &&
                p.sa_k == p.sb_k && p.sa_b == p.sb_b && p.m_lo == p.n_lo &&
                p.sa_m_hi == p.sb_n_hi && p.sa_k_hi == p.sb_k_hi;
    const long nwg = prepare_launch<typename Elem<R, CPLX>::type>(p, BM, BN, BKK, splits,
                                                                   target_wgs, work, device);
    if (SH && !(p.same_ab && p.tm == 1 && p.tn == 1))
        throw Error("gemm: internal error, shared slab image for a launch with off-diagonal tiles");
    if (unsigned long long *meter = gemm_clock_meter(device)) {
        p.probe = meter;
        p.probe_all = -1;
    }
    KernelTimer total("gemm_total", stream);
    {
        KernelTimer timer("gemm", stream);
        if constexpr (ALLOW_M3) {
            if (m3)
                hipLaunchKernelGGL((gemm_dma_kernel<R, CPLX, AK, BK, BM, BN, BKK, WM, WN, CPLX>),
                                   dim3((unsigned)nwg), dim3(WM * WN * 64), 0, stream, p);
            else
                hipLaunchKernelGGL((gemm_dma_kernel<R, CPLX, AK, BK, BM, BN, BKK, WM, WN>),
                                   dim3((unsigned)nwg), dim3(WM * WN * 64), 0, stream, p);
        } else
            hipLaunchKernelGGL((gemm_dma_kernel<R, CPLX, AK, BK, BM, BN, BKK, WM, WN, false, PF, KG, SH, LW, SP>),
                               dim3((unsigned)nwg), dim3(WM * WN * KG * 64), 0, stream, p);
        SBX_HIP_CHECK(hipGetLastError());
    }
    launch_reduce<R, CPLX>(p, stream);
}

/// The fused split-K sums' per-batch-entry counters of a stream: zero when allocated and left zero
/// by every launch (the last workgroup of an entry resets its counter), so no memset per call;
/// one array per stream, so launches on different streams never share a counter
unsigned *splitk_counters(hipStream_t stream, long n, int device) {
    static std::mutex mu;
    static std::map<hipStream_t, std::pair<unsigned *, long>> arrays;
    std::lock_guard<std::mutex> lock(mu);
    auto &a = arrays[stream];
    if (a.second < n) {
        // (a smaller array of this stream: its launches have completed in stream order before
        // the new one is used; the old one is released after the stream drains)
        if (a.first) {
            SBX_HIP_CHECK(hipStreamSynchronize(stream));
            SBX_HIP_CHECK(hipFree(a.first));
        }
        const long cap = std::max(n, 1024L);
        void *ptr = nullptr;
        SBX_HIP_CHECK(hipMalloc(&ptr, sizeof(unsigned) * cap));
        SBX_HIP_CHECK(hipMemset(ptr, 0, sizeof(unsigned) * cap));
        a = {(unsigned *)ptr, cap};
    }
    (void)device;
    return a.first;
}

/// Launch the wave-private-slab kernel (tensor contracted with itself, one tile per batch entry)
template <typename R, bool CPLX, bool AK, int BM, int BKK, int KG, int RING, bool FUSE = false>
void launch_wave_cfg(const GemmKArgs &p0, int device, hipStream_t stream, long target_wgs) {
    GemmKArgs p = p0;
    Scratch work;
    long splits = g_gemm_tune.splits > 0 ? g_gemm_tune.splits : 0;
    const long nwg = prepare_launch<typename Elem<R, CPLX>::type>(p, BM, BM, BKK * KG, splits,
                                                                   target_wgs, work, device);
    if (p.tm != 1 || p.tn != 1 || p.m != p.n)
        throw Error("gemm: internal error, wave kernel for a launch with several tiles");
    unsigned *counters = FUSE && p.splits > 1 ? splitk_counters(stream, p.batch, device) : nullptr;
    KernelTimer total("gemm_total", stream);
    {
        KernelTimer timer("gemm", stream);
        hipLaunchKernelGGL((gemm_wave_kernel<R, CPLX, AK, BM, BKK, KG, RING, FUSE>),
                           dim3((unsigned)nwg), dim3(KG * 64), 0, stream, p, counters);
        SBX_HIP_CHECK(hipGetLastError());
    }
    if (!FUSE) launch_reduce<R, CPLX>(p, stream);
}

/// The LDS-DMA kernel reads whole 16-B granules: every granule must lie inside the operand
/// (granule-aligned extents along the contiguous dimension, 16-B aligned rows and base)
template <typename E> bool dma_ok(const GemmKArgs &p, bool ak, bool bk) {
    constexpr long EPG = 16 / (long)sizeof(E);
    if (EPG == 1) return true;
    auto aligned = [](const void *ptr) { return ((std::uintptr_t)ptr & 15) == 0; };
    if (!aligned(p.a) || !aligned(p.b)) return false;
    // split groups: the inner extent of the contiguous dimension and every outer stride are
    // granule multiples (a granule never straddles two runs)
    if (p.split) {
        if ((ak ? p.k_lo : p.m_lo) % EPG || (bk ? p.k_lo : p.n_lo) % EPG) return false;
        if (p.sa_m_hi % EPG || p.sa_k_hi % EPG || p.sb_k_hi % EPG || p.sb_n_hi % EPG) return false;
    }
    // K-major operand: k extent and the row/batch strides are granule multiples
    if (ak && (p.k % EPG || p.sa_m % EPG || p.sa_b % EPG)) return false;
    if (bk && (p.k % EPG || p.sb_n % EPG || p.sb_b % EPG)) return false;
    // M-major operand: m (n) extent and the k/batch strides are granule multiples
    if (!ak && (p.m % EPG || p.sa_k % EPG || p.sa_b % EPG)) return false;
    if (!bk && (p.n % EPG || p.sb_k % EPG || p.sb_b % EPG)) return false;
    return true;
}

template <typename R, bool CPLX, bool AK, bool BK>
void launch_tiled(const GemmKArgs &p, int device, hipStream_t stream) {
    // complex<double>: LDS-DMA kernel; 128x128 tiles (8 waves, one workgroup per CU) when the
    // output is large enough, else 64x64 (tools/gemm_tune.hip: 67.5 / 65.5 TFLOP/s on the
    // 16^4 lattice contraction, 86 % / 83 % of the 78.6 TFLOP/s FP64 matrix peak)
    typedef typename Elem<R, CPLX>::type E;
    if (!dma_ok<E>(p, AK, BK)) {
        launch_tiled_cfg<R, CPLX, AK, BK, 64, 64, 16, 2, 2>(p, device, stream);
    } else if constexpr (std::is_same<R, double>::value && CPLX) {
        // (16-deep slabs: same time in the 3-multiplication form, 1.68 -> 1.51 ms in the 4-)
        // split-K to one workgroup per CU (config 2: 4 splits 1.19 ms, 8 / 16 splits 1.20 /
        // 1.23 ms once the clocks have ramped up, tools/gemm_chunks.py); 16 waves of 32x32
        // (125 VGPRs, 4 waves/SIMD) measured 1.19-1.22 ms in the 3M form (8 waves: 1.16-1.18)
        // The 4-multiplication form (default): 16-deep slabs (half the barriers per MFMA; 128 KB
        // of LDS double buffer) and 16 waves of 32x32 (4 waves per SIMD, <= 128 VGPRs): config 2
        // in 1.503-1.510 ms against 1.562-1.570 with 8 waves of 32x64 and 1.523-1.530 with
        // 8-deep slabs (tools/gemm_tune.hip, profiles/r02_gemm_tune.txt).  The 3-multiplication
        // form keeps 8 waves and 8-deep slabs (its third accumulator set needs the VGPRs).
        const bool m3 = g_gemm_tune.m3 > 0;
        if (p.m >= 128 && p.n >= 128) {
            if (m3)
                launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 8, 4, 2>(p, device, stream, 0, 256);
            else if constexpr (AK && BK) {
                // loader waves (gemm.loaders / gemm.dma_spread, K-major operands without split
                // groups): only waves 0..LW-1 issue the slab DMA
                const int lw = p.split ? 0 : g_gemm_tune.loaders, sp = g_gemm_tune.dma_spread;
                if (lw == 4 && sp == 4)
                    launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 16, 4, 4, false, false, 1, false, 4, 4>(p, device, stream, 0, 256);
                else if (lw == 4)
                    launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 16, 4, 4, false, false, 1, false, 4, 1>(p, device, stream, 0, 256);
                else if (lw == 8 && sp == 4)
                    launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 16, 4, 4, false, false, 1, false, 8, 4>(p, device, stream, 0, 256);
                else if (lw == 8 && sp == 0)
                    launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 16, 4, 4, false, false, 1, false, 8, 0>(p, device, stream, 0, 256);
                else if (lw == 8)
                    launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 16, 4, 4, false, false, 1, false, 8, 1>(p, device, stream, 0, 256);
                else if (lw == 16 && sp == 4)
                    launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 16, 4, 4, false, false, 1, false, 16, 4>(p, device, stream, 0, 256);
                else
                    launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 16, 4, 4, false>(p, device, stream, 0, 256);
            } else
                launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 16, 4, 4, false>(p, device, stream, 0, 256);
        } else {
            launch_dma_cfg<R, CPLX, AK, BK, 64, 64, 8, 2, 2>(p, device, stream, 0, 1024);
        }
    } else {
        // small outputs (33..48 rows and columns, e.g. the chain's TSnsN contraction: m = n = 4 x
        // 12): 48x48 tiles of three 16x48 wave tiles, no MFMA rows or columns of padding (64x64
        // tiles use 56 % of each dimension); split-K to ~1536 workgroups (six per CU: one round).
        // The chain's complex<float> contraction (k = 12 288, batch 64): 0.302 -> 0.197 ms
        // (tools/chain_contraction.py, profiles/r02_chain_contraction.txt; 16x48 / 48x16 wave
        // tiles, 16- / 32-deep slabs and 1024 / 2048 workgroups: 0.197-0.218 ms); with one slab
        // image for its two (identical) operands, 512 / 768 / 1024 / 1536 / 2048 / 3072 / 4096
        // workgroups: 0.194 / 0.186 / 0.170 / 0.164 / 0.170 / 0.175 / 0.188 ms (warm,
        // profiles/r02c_chain_splits.txt)
        const int t48 = g_gemm_tune.t48;
        if (t48 > 0 && p.m > 32 && p.m <= 48 && p.n > 32 && p.n <= 48) {
            // (round-2 forms, kept for comparison runs)
            if (t48 == 1) return launch_dma_cfg<R, CPLX, AK, BK, 48, 48, 16, 3, 1>(p, device, stream, 0, 1024);
            if (t48 == 2) return launch_dma_cfg<R, CPLX, AK, BK, 48, 48, 16, 1, 3>(p, device, stream, 0, 1024);
            if (t48 == 3) return launch_dma_cfg<R, CPLX, AK, BK, 48, 48, 32, 3, 1>(p, device, stream, 0, 1024);
            if (t48 == 4) return launch_dma_cfg<R, CPLX, AK, BK, 48, 48, 16, 3, 1>(p, device, stream, 0, 1536);
            // a tensor contracted with itself, one tile per batch entry (the chain's y^H y):
            // wave-private slab rings, A-only images (tools/chain_contraction.py, round 4: 0.167 ->
            // 0.142-0.146 ms warm against the t48 = 4 form, profiles/r04_chain_gemm.txt)
            const bool sh = g_gemm_tune.share_ab && p.a == p.b && p.m == p.n && p.sa_m == p.sb_n &&
                            p.sa_k == p.sb_k && p.sa_b == p.sb_b && p.m_lo == p.n_lo &&
                            p.sa_m_hi == p.sb_n_hi && p.sa_k_hi == p.sb_k_hi;
            if constexpr (!AK && !BK && sizeof(E) >= 8) {
                // (comparison forms: 13 four waves per workgroup, 1024 workgroups; 14 the same with
                // 16-deep slabs; 16 sixteen waves, 256 workgroups)
                if (sh && t48 == 13) return launch_wave_cfg<R, CPLX, AK, 48, 8, 4, 2>(p, device, stream, 1024);
                if (sh && t48 == 14) return launch_wave_cfg<R, CPLX, AK, 48, 16, 4, 2>(p, device, stream, 768);
                if (sh && t48 == 16) return launch_wave_cfg<R, CPLX, AK, 48, 8, 16, 2>(p, device, stream, 256);
                // 17: the default form with the split-K sum fused (write-through partials, the
                // last workgroup of a batch entry sums them)
                if (sh && t48 == 17) return launch_wave_cfg<R, CPLX, AK, 48, 8, 8, 2, true>(p, device, stream, 512);
                // eight waves per workgroup, 512 workgroups: half the split-K partials of the
                // four-wave form to write and sum (their per-wave tiles summed through LDS first):
                // 0.138-0.139 -> 0.136-0.137 ms warm, interleaved (profiles/r04_chain_gemm.txt)
                if (sh && t48 != 6) return launch_wave_cfg<R, CPLX, AK, 48, 8, 8, 2>(p, device, stream, 512);
            }
            // otherwise four k-groups of whole 48x48 tiles per workgroup (one wave per SIMD each),
            // 32-deep workgroup slabs: 0.167 -> 0.147-0.150 ms on the same shape unshared
            return launch_dma_cfg<R, CPLX, AK, BK, 48, 48, 32, 1, 1, false, false, 4>(p, device, stream, 0, 768);
        }
        // 8-byte and 4-byte elements: 32-deep slabs (fewer barriers per MFMA; measured against
        // 16 and 64 on the lattice shape: double 50.5, complex<float> 116, float 107 TFLOP/s)
        if (p.m >= 128 && p.n >= 128)
            launch_dma_cfg<R, CPLX, AK, BK, 128, 128, 32, 4, 2>(p, device, stream, 0, 256);
        else
            launch_dma_cfg<R, CPLX, AK, BK, 64, 64, 32, 2, 2>(p, device, stream, 0, 1024);
    }
}

/// The skinny forms (gemm_dot_kernel / gemm_rows_kernel) when an output dimension is tiny;
/// false when the shape is for the MFMA kernels
template <typename R, bool CPLX> bool launch_skinny(const GemmKArgs &p0, int device, hipStream_t s) {
    if (!g_gemm_tune.skinny || p0.split) return false;
    typedef typename Elem<R, CPLX>::type E;
    GemmKArgs p = p0;
    if (p.m <= 4 && p.n <= 4) {
        // split-K to ~gemm.dot_wgs workgroups (256: one per CU), chunks of >= 1024 k
        const long wgs = std::max(1, g_gemm_tune.dot_wgs);
        long splits = std::max(1L, std::min((wgs + p.batch - 1) / p.batch, (p.k + 1023) / 1024));
        p.kchunk = (p.k + splits - 1) / splits;
        splits = std::max(1L, (p.k + p.kchunk - 1) / p.kchunk);
        p.splits = (int)splits;
        Scratch work;
        if (splits > 1) {
            work = Scratch(sizeof(E) * splits * p.batch * p.m * p.n, device);
            p.work = work.ptr;
        }
        const long nwg = p.batch * splits;
        if (nwg > 0x7fffffffL) return false;
        KernelTimer total("gemm_total", s);
        {
            KernelTimer timer("gemm", s);
            const long mx = std::max(p.m, p.n);
            if (mx == 1)
                hipLaunchKernelGGL((gemm_dot_kernel<R, CPLX, 1, 1>), dim3((unsigned)nwg), dim3(256), 0, s, p);
            else if (mx == 2)
                hipLaunchKernelGGL((gemm_dot_kernel<R, CPLX, 2, 2>), dim3((unsigned)nwg), dim3(256), 0, s, p);
            else
                hipLaunchKernelGGL((gemm_dot_kernel<R, CPLX, 4, 4>), dim3((unsigned)nwg), dim3(256), 0, s, p);
            SBX_HIP_CHECK(hipGetLastError());
        }
        launch_reduce<R, CPLX>(p, s);
        return true;
    }
    // one long output dimension, the other <= 16, and a short k (updates): a lane per output
    // row walks k serially, so a long k (a gemv such as V^H w over a local volume) stays on the
    // split-K MFMA tiles
    const bool rows = p.n <= 16 && p.m >= 2 * p.n && p.k <= 64;
    const bool cols = p.m <= 16 && p.n >= 2 * p.m && p.k <= 64;
    if (!rows && !cols) return false;
    if (!rows) { // C^T = op(B)^T op(A)^T: the long dimension becomes the rows
        std::swap(p.m, p.n);
        std::swap(p.a, p.b);
        std::swap(p.sa_m, p.sb_n);
        std::swap(p.sa_k, p.sb_k);
        std::swap(p.sa_b, p.sb_b);
        std::swap(p.conja, p.conjb);
        std::swap(p.sc_m, p.sc_n);
    }
    const long total = p.m * p.batch;
    const long blocks = std::max(1L, std::min((total + 255) / 256, 65536L));
    KernelTimer total_t("gemm_total", s);
    KernelTimer timer("gemm", s);
    if (p.n == 1)
        hipLaunchKernelGGL((gemm_rows_kernel<R, CPLX, 1>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    else if (p.n <= 2)
        hipLaunchKernelGGL((gemm_rows_kernel<R, CPLX, 2>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    else if (p.n <= 4)
        hipLaunchKernelGGL((gemm_rows_kernel<R, CPLX, 4>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    else if (p.n <= 8)
        hipLaunchKernelGGL((gemm_rows_kernel<R, CPLX, 8>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    else
        hipLaunchKernelGGL((gemm_rows_kernel<R, CPLX, 16>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    SBX_HIP_CHECK(hipGetLastError());
    return true;
}

/// The fragment kernel (gemm_frag_kernel) for small outputs with a long k (m, n <= 32) and
/// tall-skinny products (one output dimension <= 16 -- 48 for complex<float> -- with k <= 64, or
/// <= 16 against a long k);
/// false when the shape is for the tiled kernels
template <typename R, bool CPLX> bool launch_frag(const GemmKArgs &p0, int device, hipStream_t s) {
    // (the opt-in 3-multiplication form runs on the tiled kernels only)
    if (!g_gemm_tune.frag || p0.split || (CPLX && g_gemm_tune.m3 > 0)) return false;
    // (measured, tools/studies/gemm_skinny_bench.py, profiles/r06_gemm_skinny.txt: inner products
    // m = n = 8 / 12 / 16 / 32, k = 49152, batch 32: 794 / 792 / 794 / 802 -> 143 / 173 / 228 /
    // 490 us; updates m = 49152, n = k = 12 / 16: 291 / 453 -> 173 / 208 us; n = k <= 4 stay on
    // the rows kernel, 21-49 us against 122)
    const long sm = g_gemm_tune.frag_small;
    const bool small = p0.m <= sm && p0.n <= sm;
    // the short output dimension against a short k: up to 32 for complex<float> (updates m =
    // 49152, n = k = 24 / 32, batch 32: 416 / 463 -> 327 / 427 us against the tiled kernels; 48
    // and 64 no better), 16 otherwise (complex<double> n = k = 32 / 48 / 64: no gain);
    // profiles/r06_gemm_frag_tall.txt; gemm.frag_tall > 0 overrides
    typedef typename Elem<R, CPLX>::type E;
    // (with the k pairs: complex<float> n = k = 48 805 -> 652 us; 64 855 -> 974, so up to 48;
    // profiles/r06_gemm_frag_nt.txt)
    const long tn = g_gemm_tune.frag_tall > 0 ? g_gemm_tune.frag_tall
                    : (CPLX && sizeof(R) == 4) ? 48 : 16;
    const bool tall = (p0.n <= 16 && p0.n > 4 && p0.m <= 16) ||
                      (p0.n <= tn && p0.n > 4 && p0.k <= 64 && p0.k > 4) ||
                      (p0.m <= tn && p0.m > 4 && p0.k <= 64 && p0.k > 4);
    if (!small && !tall) return false;
    if (g_gemm_tune.skinny && p0.m <= 4 && p0.n <= 4 && g_gemm_tune.frag < 2) return false;
    // k-steps per load group: 2 for a k of 8 or less and for small outputs, else 4 (0 = this
    // rule; profiles/r06_gemm_frag_cfg.txt: inner products m = n = 16 229 -> 204 us, the update
    // n = k = 8 150 -> 113 us with 2; n = k = 16 208 -> 226 us, so 4 there)
    const int auto_uk = p0.k <= 8 || (p0.m <= 32 && p0.n <= 32) ? 2 : 4;
    const int uk = g_gemm_tune.frag_uk == 0 ? auto_uk : g_gemm_tune.frag_uk == 8 ? 8
                 : g_gemm_tune.frag_uk == 2 ? 2 : 4;
    // 16 x 16 tiles per wave along n (gemm.frag_nt 1, 2 or 4; 0 = 2 for small outputs of 17-32
    // columns, else 1: inner products m = n = 32 300 / 488 -> 250 / 451 us for complex<float> /
    // <double>; the updates n = k = 24-64 gain nothing from 2 and lose with 4,
    // profiles/r06_gemm_frag_nt.txt)
    const int nt = g_gemm_tune.frag_nt == 4 ? 4 : g_gemm_tune.frag_nt == 2 ? 2
                 : g_gemm_tune.frag_nt == 0 && small && p0.n > 16 ? 2 : 1;
    GemmKArgs p = p0;
    Scratch work;
    // ~gemm.frag_waves waves: split-K when the tiles alone are fewer
    const long items = prepare_launch<E>(p, 16, 16 * nt, 4 * uk, 0,
                                         std::max(64, g_gemm_tune.frag_waves), work, device);
    const long blocks = (items + 3) / 4;
    if (blocks > 0x7fffffffL) return false;
    // 16-byte k pairs for an operand with 8-byte elements, unit k stride and 16-byte aligned rows
    // (gemm.frag_pair 0 = off)
    auto aligned = [](const void *ptr, long s1, long s2) {
        return ((std::uintptr_t)ptr % 16) == 0 && s1 % 2 == 0 && s2 % 2 == 0;
    };
    constexpr bool E8 = sizeof(E) == 8;
    p.pair_a = E8 && p.sa_k == 1 && aligned(p.a, p.sa_m, p.sa_b);
    p.pair_b = E8 && p.sb_k == 1 && aligned(p.b, p.sb_n, p.sb_b);
    // (measured, complex<float>, tools/studies/gemm_skinny_bench.py GEMM_PAIR, profiles/
    // r06_gemm_frag_pairs.txt: inner products, both operands paired, m = n = 8 / 12 / 16 / 32
    // 121 / 139 / 172 / 428 -> 100 / 122 / 160 / 288 us; updates, B alone paired, n = k = 8 / 12
    // 80 / 136 -> 82 / 142 us, 16 the same, 32 427 -> 385 us: so B alone from n > 16; inner
    // products with an m-contiguous A, B alone paired: within 3 %, profiles/r06_gemm_frag_pairs_nn.txt)
    const bool kp = E8 && g_gemm_tune.frag_pair && p.k % 2 == 0 &&
                    (p.pair_a || (p.pair_b && p.n > 16));
    KernelTimer total("gemm_total", s);
    {
        KernelTimer timer("gemm", s);
        const dim3 grid((unsigned)blocks), wg(256);
        auto go = [&](auto ukc, auto kpc, auto ntc) {
            constexpr int UKv = decltype(ukc)::value, NTv = decltype(ntc)::value;
            constexpr bool KPv = decltype(kpc)::value;
            hipLaunchKernelGGL((gemm_frag_kernel<R, CPLX, UKv, KPv, NTv>), grid, wg, 0, s, p);
        };
        auto by_nt = [&](auto ukc, auto kpc) {
            if (nt == 4)
                go(ukc, kpc, std::integral_constant<int, 4>());
            else if (nt == 2)
                go(ukc, kpc, std::integral_constant<int, 2>());
            else
                go(ukc, kpc, std::integral_constant<int, 1>());
        };
        auto by_uk = [&](auto kpc) {
            if (uk == 8)
                by_nt(std::integral_constant<int, 8>(), kpc);
            else if (uk == 2)
                by_nt(std::integral_constant<int, 2>(), kpc);
            else
                by_nt(std::integral_constant<int, 4>(), kpc);
        };
        if constexpr (E8) {
            if (kp) by_uk(std::true_type());
        }
        if (!kp) by_uk(std::false_type());
        SBX_HIP_CHECK(hipGetLastError());
    }
    launch_reduce<R, CPLX>(p, s);
    return true;
}

template <typename R, bool CPLX> void launch_typed(const GemmKArgs &p, int device, hipStream_t s) {
    if (launch_frag<R, CPLX>(p, device, s)) return;
    if (launch_skinny<R, CPLX>(p, device, s)) return;
    // Pick the stage-load thread map from the unit stride of each operand
    const bool ak = (p.sa_k == 1) || (p.sa_m != 1 && std::labs(p.sa_k) <= std::labs(p.sa_m));
    const bool bk = (p.sb_k == 1) || (p.sb_n != 1 && std::labs(p.sb_k) <= std::labs(p.sb_n));
    if (ak && bk)
        launch_tiled<R, CPLX, true, true>(p, device, s);
    else if (ak && !bk)
        launch_tiled<R, CPLX, true, false>(p, device, s);
    else if (!ak && bk)
        launch_tiled<R, CPLX, false, true>(p, device, s);
    else
        launch_tiled<R, CPLX, false, false>(p, device, s);
}

template <typename R, bool CPLX> void launch_scale(const GemmKArgs &p, hipStream_t s) {
    const long total = p.batch * p.m * p.n;
    if (total == 0) return;
    const long blocks = std::min((total + 255) / 256, 4096L);
    hipLaunchKernelGGL((scale_c_kernel<R, CPLX>), dim3((unsigned)blocks), dim3(256), 0, s, p);
    SBX_HIP_CHECK(hipGetLastError());
}

GemmKArgs make_args(const GemmDesc &d) {
    GemmKArgs p{};
    p.m = d.m;
    p.n = d.n;
    p.k = d.k;
    p.batch = d.batch;
    p.a = d.a;
    p.sa_m = d.sa_m;
    p.sa_k = d.sa_k;
    p.sa_b = d.sa_b;
    p.b = d.b;
    p.sb_k = d.sb_k;
    p.sb_n = d.sb_n;
    p.sb_b = d.sb_b;
    p.c = d.c;
    p.sc_m = d.sc_m;
    p.sc_n = d.sc_n;
    p.sc_b = d.sc_b;
    p.alpha_re = d.alpha.re;
    p.alpha_im = dtype_is_complex(d.t) ? d.alpha.im : 0;
    p.beta_re = d.beta.re;
    p.beta_im = dtype_is_complex(d.t) ? d.beta.im : 0;
    p.conja = d.conja;
    p.conjb = d.conjb;
    p.splits = 1;
    p.kchunk = d.k;
    p.m_lo = d.m_lo > 0 ? d.m_lo : d.m;
    p.n_lo = d.n_lo > 0 ? d.n_lo : d.n;
    p.k_lo = d.k_lo > 0 ? d.k_lo : d.k;
    p.sa_m_hi = d.sa_m_hi;
    p.sa_k_hi = d.sa_k_hi;
    p.sb_k_hi = d.sb_k_hi;
    p.sb_n_hi = d.sb_n_hi;
    p.sc_m_hi = d.sc_m_hi;
    p.sc_n_hi = d.sc_n_hi;
    p.split = (p.m_lo != p.m || p.n_lo != p.n || p.k_lo != p.k) ? 1 : 0;
    if (p.split && (p.m_lo < 1 || p.n_lo < 1 || p.k_lo < 1 || p.m % p.m_lo || p.n % p.n_lo ||
                    p.k % p.k_lo))
        throw Error("gemm: invalid split groups");
    return p;
}

} // namespace

void gemm_clock_read(int device, unsigned long long out[3], bool reset) {
    clock_read_impl(device, out, reset);
}

void launch_gemm(const GemmDesc &d, int device) {
    if (d.m == 0 || d.n == 0 || d.batch == 0) return;
    // operands beyond the 32-bit buffer descriptors (2 GiB per batch entry): cut K (the later
    // pieces accumulate with beta = 1), or M / N when one K index alone is too large
    if (d.k > 0 && (d.alpha.re != 0 || d.alpha.im != 0)) {
        const long es = (long)dtype_size(d.t);
        const long max_bytes = g_gemm_tune.max_bytes > 0 ? g_gemm_tune.max_bytes : (1L << 31) - 1;
        auto ext = [&](long n, long lo, long st, long st_hi) {
            return lo > 0 && lo < n ? (n / lo - 1) * std::labs(st_hi) + (lo - 1) * std::labs(st)
                                    : (n - 1) * std::labs(st);
        };
        const long ea = (ext(d.m, d.m_lo, d.sa_m, d.sa_m_hi) + ext(d.k, d.k_lo, d.sa_k, d.sa_k_hi) + 1) * es;
        const long eb = (ext(d.k, d.k_lo, d.sb_k, d.sb_k_hi) + ext(d.n, d.n_lo, d.sb_n, d.sb_n_hi) + 1) * es;
        if (ea > max_bytes || eb > max_bytes) {
            // cut a group of extent n (inner extent lo, 0 = one run) in two: split groups only
            // between outer indices; returns the first part's extent and the second's offset
            // (in elements, per stride pair)
            struct Cut {
                long n1, lo1, n2, lo2, o_outer;
                bool ok;
            };
            auto cut = [](long n, long lo) {
                Cut c{};
                const bool spl = lo > 0 && lo < n;
                if (spl) {
                    const long outer = n / lo, o1 = outer / 2;
                    c = Cut{o1 * lo, lo, n - o1 * lo, lo, o1, true};
                } else {
                    c = Cut{n / 2, 0, n - n / 2, 0, n / 2, n > 1};
                }
                return c;
            };
            // element offset of the second part for one operand's strides
            auto off = [](long n, long lo, long st, long st_hi, long o) {
                return lo > 0 && lo < n ? o * st_hi : o * st;
            };
            const Cut ck = cut(d.k, d.k_lo);
            if (ck.ok) {
                GemmDesc a = d, b = d;
                a.k = ck.n1;
                a.k_lo = ck.lo1;
                b.k = ck.n2;
                b.k_lo = ck.lo2;
                b.a = (const char *)d.a + es * off(d.k, d.k_lo, d.sa_k, d.sa_k_hi, ck.o_outer);
                b.b = (const char *)d.b + es * off(d.k, d.k_lo, d.sb_k, d.sb_k_hi, ck.o_outer);
                b.beta = Scalar{1, 0};
                launch_gemm(a, device);
                launch_gemm(b, device);
                return;
            }
            const Cut cm = cut(d.m, d.m_lo), cn = cut(d.n, d.n_lo);
            if (cm.ok && (ea > max_bytes || !cn.ok)) {
                GemmDesc a = d, b = d;
                a.m = cm.n1;
                a.m_lo = cm.lo1;
                b.m = cm.n2;
                b.m_lo = cm.lo2;
                b.a = (const char *)d.a + es * off(d.m, d.m_lo, d.sa_m, d.sa_m_hi, cm.o_outer);
                b.c = (char *)d.c + es * off(d.m, d.m_lo, d.sc_m, d.sc_m_hi, cm.o_outer);
                launch_gemm(a, device);
                launch_gemm(b, device);
                return;
            }
            if (cn.ok) {
                GemmDesc a = d, b = d;
                a.n = cn.n1;
                a.n_lo = cn.lo1;
                b.n = cn.n2;
                b.n_lo = cn.lo2;
                b.b = (const char *)d.b + es * off(d.n, d.n_lo, d.sb_n, d.sb_n_hi, cn.o_outer);
                b.c = (char *)d.c + es * off(d.n, d.n_lo, d.sc_n, d.sc_n_hi, cn.o_outer);
                launch_gemm(a, device);
                launch_gemm(b, device);
                return;
            }
            throw Error("gemm: operand batch entries of 2 GiB or more are not supported");
        }
    }
    set_device(device);
    hipStream_t s = get_stream(device);
    GemmKArgs p = make_args(d);
    const bool scale_only = (d.k == 0 || (p.alpha_re == 0 && p.alpha_im == 0));
    switch (d.t) {
    case SBX_CDOUBLE:
        scale_only ? launch_scale<double, true>(p, s) : launch_typed<double, true>(p, device, s);
        break;
    case SBX_DOUBLE:
        scale_only ? launch_scale<double, false>(p, s) : launch_typed<double, false>(p, device, s);
        break;
    case SBX_CFLOAT:
        scale_only ? launch_scale<float, true>(p, s) : launch_typed<float, true>(p, device, s);
        break;
    case SBX_FLOAT:
        scale_only ? launch_scale<float, false>(p, s) : launch_typed<float, false>(p, device, s);
        break;
    default: throw Error("gemm: unsupported type");
    }
}

} // namespace sbx
