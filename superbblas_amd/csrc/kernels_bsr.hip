// Block-sparse (BSR) matrix times dense tensor -- the `bsr_krylov` hot loop.
//
// Reference: BSR<Cpu>::operator() builtin loop (bsr.h:535-650; one small GEMM/GEMV per nonzero
// block, OpenMP over block rows) and BSR<Gpu> -> hipsparseXbsrmm (bsr.h:855-928).
// Here: one thread per output element y(row-block i, image component c, rhs column n).
//  * The thread order follows the output layout so the stores are coalesced: for a row-major
//    output (rhs fastest) consecutive lanes take consecutive rhs columns, the nonzero block
//    values are then wave-uniform (broadcast loads) and the x gathers are contiguous along the
//    rhs; for a column-major output consecutive lanes take consecutive image components/rows
//    and read consecutive 16-byte pieces of the row-ordered nonzero blocks.
//  * Bound: HBM (the nonzero blocks are streamed once; x is re-read through L2/MALL).
//  * ELL operators (every block row has the same number of nonzero blocks -- the lattice
//    stencils) use bsr_ell_kernel: a workgroup streams the nonzero blocks of a chunk of block
//    rows into LDS with coalesced 16-byte loads (the value stream is the dominant HBM traffic),
//    then every thread computes all `bi` outputs of one (block row, rhs column) pair reading the
//    blocks from LDS (broadcast across the rhs lanes) and x from global memory (contiguous along
//    the rhs for row-major x).
#include "elem_ops.h"
#include "sbx_internal.h"

#include <algorithm>
#include <type_traits>

namespace sbx {
BsrTune g_bsr_tune;
namespace {

struct BsrArgs {
    long block_rows;
    int bi, bd;
    const int *ii;
    const int *jj;
    const void *v;
    int block_im_fast;
    const void *x;
    long ldx;
    long x_rows; // domain rows of x
    void *y;
    long ldy;
    long ncols;
    double alpha_re, alpha_im;
    int add;
    int ilv = 1; // bsr_ell9_kernel: an XCD's chunks visited as ilv interleaved parts
    int nt = 0;  // the value stream's LDS-DMA loads non-temporal: g_bsr_tune.nt's kernel bits
    // site tiles (bsr_ell9_tile_kernel; [0] 16-site, [1] 8-site tiles; rows == nullptr: none)
    TileSched tiles[2];
};

template <typename E, int BI_, int BD_, bool YROW, bool XROW>
__global__ void __launch_bounds__(256) bsr_kernel(const BsrArgs p) {
    const int bi = BI_ > 0 ? BI_ : p.bi;
    const int bd = BD_ > 0 ? BD_ : p.bd;
    const long total = p.block_rows * bi * p.ncols;
    const E *__restrict__ v = (const E *)p.v;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256L) {
        long i, col;
        int c;
        if (YROW) {
            col = idx % p.ncols;
            const long t = idx / p.ncols;
            c = (int)(t % bi);
            i = t / bi;
        } else {
            c = (int)(idx % bi);
            const long t = idx / bi;
            i = t % p.block_rows;
            col = t / p.block_rows;
        }
        E acc = Ops<E>::zero();
        const int j0 = p.ii[i], j1 = p.ii[i + 1];
        for (int j = j0; j < j1; ++j) {
            const int d0 = p.jj[j];
            if (d0 < 0) continue;
            const E *vb = v + (long)j * bi * bd;
#pragma unroll
            for (int e = 0; e < (BD_ > 0 ? BD_ : 1); ++e) {
                if (BD_ == 0) break;
                const E a = p.block_im_fast ? vb[c + e * bi] : vb[c * bd + e];
                const E xv = XROW ? x[(long)(d0 + e) * p.ldx + col] : x[(d0 + e) + col * p.ldx];
                acc = Ops<E>::fma(a, xv, acc);
            }
            if (BD_ == 0) {
                for (int e = 0; e < bd; ++e) {
                    const E a = p.block_im_fast ? vb[c + e * bi] : vb[c * bd + e];
                    const E xv =
                        XROW ? x[(long)(d0 + e) * p.ldx + col] : x[(d0 + e) + col * p.ldx];
                    acc = Ops<E>::fma(a, xv, acc);
                }
            }
        }
        const long img = i * bi + c;
        E *yp = YROW ? y + img * p.ldy + col : y + img + col * p.ldy;
        const E out = Ops<E>::scale(acc, p.alpha_re, p.alpha_im);
        *yp = p.add ? Ops<E>::add(*yp, out) : out;
    }
}

constexpr int ELL_LDS_BYTES = 24576; // per workgroup: several workgroups share a CU

template <typename E, int BI, int BD, int G, bool YROW, bool XROW>
__global__ void __launch_bounds__(256) bsr_ell_kernel(const BsrArgs p, int nnz, int rb) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    constexpr int BLK = BI * BD;
    E *vals = (E *)smem;
    int *cols = (int *)(smem + (size_t)rb * nnz * BLK * sizeof(E));
    const E *__restrict__ v = (const E *)p.v;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    // consecutive chunks of block rows on one XCD: neighbouring sites share x rows in its L2
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int chunk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const long row0 = (long)chunk * rb;
    const int nrows = (int)min((long)rb, p.block_rows - row0);
    // 1) stream the chunk's nonzero blocks (contiguous in the ELL value array) and block
    //    columns into LDS, 8 loads in flight per thread
    const long vbase = row0 * nnz * BLK;
    const int nv = nrows * nnz * BLK;
    for (int e0 = threadIdx.x; e0 < nv; e0 += 256 * 8) {
        E t[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) t[q] = v[vbase + min(e0 + 256 * q, nv - 1)];
#pragma unroll
        for (int q = 0; q < 8; ++q)
            if (e0 + 256 * q < nv) vals[e0 + 256 * q] = t[q];
    }
    for (int e = threadIdx.x; e < nrows * nnz; e += 256) cols[e] = p.jj[row0 * nnz + e];
    __syncthreads();
    // 2) every thread computes the BI x G outputs of a (block row, group of G rhs columns); the
    //    x rows of block j+1 are fetched while block j is applied
    const long ngroups = (p.ncols + G - 1) / G;
    const long npairs = (long)nrows * ngroups;
    for (long q = threadIdx.x; q < npairs; q += 256) {
        int r;
        long g;
        if (YROW) {
            r = (int)(q / ngroups);
            g = q % ngroups;
        } else {
            r = (int)(q % nrows);
            g = q / nrows;
        }
        long colv[G];
#pragma unroll
        for (int k = 0; k < G; ++k) colv[k] = min(g * G + k, p.ncols - 1);
        E acc[BI][G];
#pragma unroll
        for (int c = 0; c < BI; ++c)
#pragma unroll
            for (int k = 0; k < G; ++k) acc[c][k] = Ops<E>::zero();
        const int *jr = cols + r * nnz;
        const E *vr = vals + r * nnz * BLK;
        auto fetch = [&](int d0, E (*xv)[G]) {
            const long d = d0 < 0 ? 0 : d0;
#pragma unroll
            for (int e = 0; e < BD; ++e)
#pragma unroll
                for (int k = 0; k < G; ++k)
                    xv[e][k] = XROW ? x[(d + e) * p.ldx + colv[k]] : x[(d + e) + colv[k] * p.ldx];
        };
        E xn[BD][G];
        int dn = jr[0];
        fetch(dn, xn);
        for (int j = 0; j < nnz; ++j) {
            E xc[BD][G];
#pragma unroll
            for (int e = 0; e < BD; ++e)
#pragma unroll
                for (int k = 0; k < G; ++k) xc[e][k] = xn[e][k];
            const int dc = dn;
            if (j + 1 < nnz) {
                dn = jr[j + 1];
                fetch(dn, xn);
            }
            if (dc < 0) continue;
            const E *vb = vr + j * BLK;
#pragma unroll
            for (int e = 0; e < BD; ++e)
#pragma unroll
                for (int c = 0; c < BI; ++c) {
                    const E a = p.block_im_fast ? vb[c + e * BI] : vb[c * BD + e];
#pragma unroll
                    for (int k = 0; k < G; ++k) acc[c][k] = Ops<E>::fma(a, xc[e][k], acc[c][k]);
                }
        }
#pragma unroll
        for (int c = 0; c < BI; ++c) {
            const long img = (row0 + r) * BI + c;
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const long col = g * G + k;
                if (col >= p.ncols) break;
                E *yp = YROW ? y + img * p.ldy + col : y + img + col * p.ldy;
                const E out = Ops<E>::scale(acc[c][k], p.alpha_re, p.alpha_im);
                *yp = p.add ? Ops<E>::add(*yp, out) : out;
            }
        }
    }
}

// Large blocks (12x12 spin x color, the Wilson-like operator): block-row products on the FP64
// (FP32) matrix cores.  A wave owns one block row and a tile of 16 rhs columns and computes the
// 16x16 tile  Y_i = sum_j A_ij X_j  with v_mfma_f64_16x16x4_f64 or v_mfma_f32_16x16x4f32 (tile
// rows >= BI are padding), K running over the BD domain rows of every nonzero block (BD/4 steps
// per block, 4 real MFMAs per complex step).  The generic kernels read the fragments straight
// from global memory: lane l reads A_ij[l&15][k+(l>>4)] and x[d_j+k+(l>>4)][col0+(l&15)]
// (contiguous along the rhs for row-major x); out-of-range rows, columns and skipped blocks
// (-1 columns) are clamped loads replaced by zero, so the loop has no divergent branches.
__device__ __forceinline__ unsigned lds_u32(const void *p) {
    return (unsigned)(size_t)(const __attribute__((address_space(3))) void *)p;
}

/// s_waitcnt vmcnt(n) for an n the unrolled caller knows at compile time (folds to one wait)
__device__ __forceinline__ void wait_vmcnt_n(int n) {
    switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    }
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, unsigned off, unsigned dst, int nt = 0) {
    // inline asm: hipcc does not order its ds_reads against an LDS-DMA it cannot see; the kernel
    // retires the DMA with an explicit vmcnt(0) before its barrier.  nt (a uniform kernel
    // argument, so a scalar branch): the streaming policy for data read once (the values)
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

template <typename R, bool CPLX> struct BsrMfmaElem;
template <> struct BsrMfmaElem<double, true> { typedef double2 type; };
template <> struct BsrMfmaElem<double, false> { typedef double type; };
template <> struct BsrMfmaElem<float, true> { typedef float2 type; };
template <> struct BsrMfmaElem<float, false> { typedef float type; };
// 16x16x4 MFMA per real type and its C/D row map (col = lane & 15)
template <typename R> struct BsrMfma;
template <> struct BsrMfma<double> {
    typedef double acc_t __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc_t mma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int lane, int q) { return (lane >> 4) + 4 * q; }
};
template <> struct BsrMfma<float> {
    typedef float acc_t __attribute__((ext_vector_type(4)));
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int lane, int q) { return 4 * (lane >> 4) + q; }
};

// One block row per wave, the fragments of nonzero block t+1 loaded while block t is applied
// (twice the bytes in flight per wave; 985 -> 880 us on the chain's complex<float> operator).
// Mapping consecutive block rows to one XCD was measured no faster.
template <typename R, bool CPLX, int BI, int BD, bool YROW, bool XROW>
__global__ void __launch_bounds__(256) bsr_mfma_pf_kernel(const BsrArgs p, long ntiles_n) {
    typedef typename BsrMfmaElem<R, CPLX>::type E;
    typedef typename BsrMfma<R>::acc_t acc_t;
    static_assert(BI <= 16 && BD % 4 == 0, "block shape");
    constexpr int KS = BD / 4;
    const E *__restrict__ v = (const E *)p.v;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    const int lane = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wave >= p.block_rows * ntiles_n) return; // whole waves only: MFMA needs all 64 lanes
    const long i = wave / ntiles_n;
    const long col0 = (wave % ntiles_n) * 16;
    const int ar = lane & 15, kq = lane >> 4;
    const bool arow_ok = ar < BI;
    const int arc = arow_ok ? ar : 0;
    const long bcol = col0 + (lane & 15);
    const bool bcol_ok = bcol < p.ncols;
    const long bcc = bcol_ok ? bcol : 0;
    acc_t accR = acc_t{0, 0, 0, 0}, accI = acc_t{0, 0, 0, 0};
    const int jb = p.ii[i], je = p.ii[i + 1];
    E an[KS], bn[KS];
    auto fetch = [&](int j) {
        const int dj = p.jj[j];
        const bool ok = dj >= 0;
        const long d0 = ok ? dj : 0;
        const E *vb = v + (long)j * BI * BD;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int e = ks * 4 + kq;
            const E a = p.block_im_fast ? vb[arc + e * BI] : vb[arc * BD + e];
            const E b = XROW ? x[(d0 + e) * p.ldx + bcc] : x[(d0 + e) + bcc * p.ldx];
            an[ks] = (arow_ok && ok) ? a : E{};
            bn[ks] = bcol_ok ? b : E{};
        }
    };
    if (jb < je) fetch(jb);
    for (int j = jb; j < je; ++j) {
        E af[KS], bf[KS];
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            af[ks] = an[ks];
            bf[ks] = bn[ks];
        }
        if (j + 1 < je) fetch(j + 1);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            if constexpr (CPLX) {
                accR = BsrMfma<R>::mma(af[ks].x, bf[ks].x, accR);
                accI = BsrMfma<R>::mma(af[ks].x, bf[ks].y, accI);
                accR = BsrMfma<R>::mma(-af[ks].y, bf[ks].y, accR);
                accI = BsrMfma<R>::mma(af[ks].y, bf[ks].x, accI);
            } else {
                accR = BsrMfma<R>::mma(af[ks], bf[ks], accR);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = BsrMfma<R>::row(lane, q);
        if (row >= BI || !bcol_ok) continue;
        const long img = i * BI + row;
        E *yp = YROW ? y + img * p.ldy + bcol : y + img + bcol * p.ldy;
        E out;
        if constexpr (CPLX)
            out = Ops<E>::scale(E{accR[q], accI[q]}, p.alpha_re, p.alpha_im);
        else
            out = Ops<E>::scale(accR[q], p.alpha_re, p.alpha_im);
        *yp = p.add ? Ops<E>::add(*yp, out) : out;
    }
}

// ELL form with a compile-time number of nonzero blocks per row (the 9-point stencils): the
// row's block columns are read first (scalar loads), then the fragments of NB blocks at a time
// are loaded one group ahead of the MFMAs, so no load waits on another load and NB blocks' bytes
// are in flight per wave.
template <typename R, bool CPLX, int BI, int BD, bool YROW, bool XROW, int NNZ, int NB>
__global__ void __launch_bounds__(256) bsr_mfma_ell_kernel(const BsrArgs p, long ntiles_n) {
    typedef typename BsrMfmaElem<R, CPLX>::type E;
    typedef typename BsrMfma<R>::acc_t acc_t;
    static_assert(BI <= 16 && BD % 4 == 0 && NNZ % NB == 0, "block shape");
    constexpr int KS = BD / 4, NG = NNZ / NB;
    const E *__restrict__ v = (const E *)p.v;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    const int lane = threadIdx.x & 63;
    const long wave = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (wave >= p.block_rows * ntiles_n) return; // whole waves only: MFMA needs all 64 lanes
    const long i = wave / ntiles_n;
    const long col0 = (wave % ntiles_n) * 16;
    const int ar = lane & 15, kq = lane >> 4;
    const bool arow_ok = ar < BI;
    const int arc = arow_ok ? ar : 0;
    const long bcol = col0 + (lane & 15);
    const bool bcol_ok = bcol < p.ncols;
    const long bcc = bcol_ok ? bcol : 0;
    const long jb = i * NNZ;
    int dj[NNZ];
#pragma unroll
    for (int k = 0; k < NNZ; ++k) dj[k] = p.jj[jb + k];
    E af[2][NB][KS], bf[2][NB][KS];
    auto fetch = [&](int g, E (*a_)[KS], E (*b_)[KS]) {
#pragma unroll
        for (int u = 0; u < NB; ++u) {
            const int k = g * NB + u;
            const bool ok = dj[k] >= 0;
            const long d0 = ok ? dj[k] : 0;
            const E *vb = v + (jb + k) * (BI * BD);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const int e = ks * 4 + kq;
                const E a = p.block_im_fast ? vb[arc + e * BI] : vb[arc * BD + e];
                const E b = XROW ? x[(d0 + e) * p.ldx + bcc] : x[(d0 + e) + bcc * p.ldx];
                a_[u][ks] = (arow_ok && ok) ? a : E{};
                b_[u][ks] = bcol_ok ? b : E{};
            }
        }
    };
    acc_t accR = acc_t{0, 0, 0, 0}, accI = acc_t{0, 0, 0, 0};
    fetch(0, af[0], bf[0]);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        if (g + 1 < NG) fetch(g + 1, af[(g + 1) & 1], bf[(g + 1) & 1]);
#pragma unroll
        for (int u = 0; u < NB; ++u)
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                const E a = af[g & 1][u][ks], b = bf[g & 1][u][ks];
                if constexpr (CPLX) {
                    accR = BsrMfma<R>::mma(a.x, b.x, accR);
                    accI = BsrMfma<R>::mma(a.x, b.y, accI);
                    accR = BsrMfma<R>::mma(-a.y, b.y, accR);
                    accI = BsrMfma<R>::mma(a.y, b.x, accI);
                } else {
                    accR = BsrMfma<R>::mma(a, b, accR);
                }
            }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = BsrMfma<R>::row(lane, q);
        if (row >= BI || !bcol_ok) continue;
        const long img = i * BI + row;
        E *yp = YROW ? y + img * p.ldy + bcol : y + img + bcol * p.ldy;
        E out;
        if constexpr (CPLX)
            out = Ops<E>::scale(E{accR[q], accI[q]}, p.alpha_re, p.alpha_im);
        else
            out = Ops<E>::scale(accR[q], p.alpha_re, p.alpha_im);
        *yp = p.add ? Ops<E>::add(*yp, out) : out;
    }
}

template <typename R, bool CPLX, int BI, int BD, int NNZ, int NB>
void launch_bsr_mfma_ell(const BsrArgs &a, bool yrow, bool xrow, hipStream_t s) {
    const long ntn = (a.ncols + 15) / 16;
    const long waves = a.block_rows * ntn;
    const long blocks = (waves + 3) / 4;
    if (blocks >= (1L << 31)) throw Error("bsr: grid too large");
    g_bsr_tune.last = 10;
    KernelTimer timer("bsr", s);
    if (yrow && xrow)
        hipLaunchKernelGGL((bsr_mfma_ell_kernel<R, CPLX, BI, BD, true, true, NNZ, NB>), dim3(blocks), dim3(256), 0, s, a, ntn);
    else if (yrow && !xrow)
        hipLaunchKernelGGL((bsr_mfma_ell_kernel<R, CPLX, BI, BD, true, false, NNZ, NB>), dim3(blocks), dim3(256), 0, s, a, ntn);
    else if (!yrow && xrow)
        hipLaunchKernelGGL((bsr_mfma_ell_kernel<R, CPLX, BI, BD, false, true, NNZ, NB>), dim3(blocks), dim3(256), 0, s, a, ntn);
    else
        hipLaunchKernelGGL((bsr_mfma_ell_kernel<R, CPLX, BI, BD, false, false, NNZ, NB>), dim3(blocks), dim3(256), 0, s, a, ntn);
    SBX_HIP_CHECK(hipGetLastError());
}

template <typename R, bool CPLX, int BI, int BD>
void launch_bsr_mfma_pf(const BsrArgs &a, bool yrow, bool xrow, hipStream_t s) {
    const long ntn = (a.ncols + 15) / 16;
    const long waves = a.block_rows * ntn;
    const long blocks = (waves + 3) / 4;
    if (blocks >= (1L << 31)) throw Error("bsr: grid too large");
    g_bsr_tune.last = 11;
    KernelTimer timer("bsr", s);
    if (yrow && xrow)
        hipLaunchKernelGGL((bsr_mfma_pf_kernel<R, CPLX, BI, BD, true, true>), dim3(blocks), dim3(256), 0, s, a, ntn);
    else if (yrow && !xrow)
        hipLaunchKernelGGL((bsr_mfma_pf_kernel<R, CPLX, BI, BD, true, false>), dim3(blocks), dim3(256), 0, s, a, ntn);
    else if (!yrow && xrow)
        hipLaunchKernelGGL((bsr_mfma_pf_kernel<R, CPLX, BI, BD, false, true>), dim3(blocks), dim3(256), 0, s, a, ntn);
    else
        hipLaunchKernelGGL((bsr_mfma_pf_kernel<R, CPLX, BI, BD, false, false>), dim3(blocks), dim3(256), 0, s, a, ntn);
    SBX_HIP_CHECK(hipGetLastError());
}

// Contiguous-block form (row-major x with ldx == ncols <= 16, ELL with NNZ blocks per row): the
// nonzero block A_ij and the x block of its domain rows are each one contiguous run of
// BI*BD (BD*ncols) elements, so a wave moves them by LDS-DMA (buffer_load_dwordx4 ... lds, every
// lane a distinct 16 bytes, 1 KB per instruction, no VGPR round trip) into its LDS slot, PD
// blocks ahead in a ring of PD + 1 slots, instead of 12-row fragment gathers, and reads the MFMA
// fragments from the slot.  (The round-2 register-staged form measured the same on
// complex<double> and 6 % slower on the chain's complex<float> operator, profiles/r02_bsr_blk_sweep.txt.)
// PK > 0 (packed slots): the value block and the x block are one run of the slot (x right after
// the values, no 1-KB rounding of each), moved by PK global_load_lds_dwordx4 instructions whose
// lanes address either array (a buffer load takes one array per instruction) -- 2304 instead of
// 4096 bytes per complex<float> slot at 12 rhs, 4608 instead of 6144 for complex<double>, so more
// waves (and more bytes in flight) fit a CU's LDS
template <typename R, bool CPLX, int BI, int BD, bool YROW, int NNZ, int PD, bool M3, int PK = 0>
__global__ void __launch_bounds__(256) bsr_mfma_dma_kernel(const BsrArgs p, unsigned v_bytes, unsigned x_bytes) {
    typedef typename BsrMfmaElem<R, CPLX>::type E;
    typedef typename BsrMfma<R>::acc_t acc_t;
    static_assert(BI <= 16 && BD % 4 == 0, "block shape");
    constexpr int KS = BD / 4, ES = (int)sizeof(E);
    constexpr int ABLK = BI * BD, XBLK = BD * 16;        // elements (x: up to 16 cols)
    constexpr int NA = (ABLK * ES + 1023) / 1024, NX = (XBLK * ES + 1023) / 1024; // DMA instructions
    constexpr int NI = PK > 0 ? PK : NA + NX;            // DMA instructions per block
    extern __shared__ __attribute__((aligned(16))) char smem[];
    E *__restrict__ y = (E *)p.y;
    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const long i = (long)blockIdx.x * 4 + w;
    if (i >= p.block_rows) return;
    const int nc = (int)p.ncols, xblk = BD * nc;
    // bytes per ring slot (packed: values then x, 16-byte aligned)
    const unsigned SLOT = PK > 0 ? (unsigned)(ABLK + xblk) * ES : (unsigned)(NA + NX) * 1024u;
    const long jb = i * NNZ;
    int dj[NNZ];
#pragma unroll
    for (int k = 0; k < NNZ; ++k) dj[k] = p.jj[jb + k];
    // the row's NNZ value blocks (one contiguous run) as the buffer: 32-bit offsets at any size
    (void)v_bytes;
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
        (void *)((const E *)p.v + jb * ABLK), (short)0, NNZ * ABLK * ES, 0x00020000);
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)p.x, (short)0, (int)x_bytes, 0x00020000);
    const unsigned slot0 = lds_u32(smem) + (unsigned)w * (SLOT * (PD + 1));
    auto issue = [&](int k) {
        const unsigned base = slot0 + (unsigned)(k % (PD + 1)) * SLOT;
        if constexpr (PK > 0) {
            const char *vrow = (const char *)((const E *)p.v + (jb + k) * ABLK);
            // a skipped block (column -1) reads x's first block row (not used): always BD * nc
            // valid elements, where the block's own values may end before the slot's x part
            const char *xrow = (const char *)((const E *)p.x + (long)(dj[k] < 0 ? 0 : dj[k]) * nc);
#pragma unroll
            for (int q = 0; q < PK; ++q) {
                const unsigned g = (unsigned)(lane + 64 * q) * 16u;
                if (g < SLOT) {
                    const char *src = g < (unsigned)(ABLK * ES) ? vrow + g : xrow + (g - ABLK * ES);
                    // nt on the instructions that carry values only (x rows are reused)
                    if ((p.nt & 1) && (q + 1) * 1024 <= ABLK * ES)
                        asm volatile("s_mov_b32 m0, %1\n\t"
                                     "s_nop 0\n\t"
                                     "global_load_lds_dwordx4 %0, off nt"
                                     :
                                     : "v"(src), "s"(__builtin_amdgcn_readfirstlane(base + (unsigned)q * 1024u))
                                     : "memory", "m0");
                    else
                        asm volatile("s_mov_b32 m0, %1\n\t"
                                     "s_nop 0\n\t"
                                     "global_load_lds_dwordx4 %0, off"
                                     :
                                     : "v"(src), "s"(__builtin_amdgcn_readfirstlane(base + (unsigned)q * 1024u))
                                     : "memory", "m0");
                }
            }
        } else {
            const unsigned av = (unsigned)(k * ABLK * ES), xv = (unsigned)((long)(dj[k] < 0 ? 0 : dj[k]) * nc) * ES;
#pragma unroll
            for (int q = 0; q < NA; ++q) {
                const unsigned g = (unsigned)(lane + 64 * q) * 16u;
                dma16(rv, g < (unsigned)(ABLK * ES) ? av + g : 0x80000000u, base + (unsigned)q * 1024u, p.nt & 1);
            }
#pragma unroll
            for (int q = 0; q < NX; ++q) {
                const unsigned g = (unsigned)(lane + 64 * q) * 16u;
                dma16(rx, g < (unsigned)(xblk * ES) ? xv + g : 0x80000000u, base + (unsigned)(NA + q) * 1024u);
            }
        }
    };
    const int ar = lane & 15, kq = lane >> 4;
    const bool arow_ok = ar < BI, bcol_ok = ar < nc;
    acc_t accR = acc_t{0, 0, 0, 0}, accI = acc_t{0, 0, 0, 0}, acc3 = acc_t{0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < PD && k < NNZ; ++k) issue(k);
#pragma unroll
    for (int k = 0; k < NNZ; ++k) {
        // the slot of block k + PD was last read in iteration k - 1: its reads have returned
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (k + PD < NNZ) issue(k + PD);
        // block k landed: the NI instructions of each later block issued so far may stay in flight
        wait_vmcnt_n(NI * (NNZ - 1 - k < PD ? NNZ - 1 - k : PD));
        if (dj[k] < 0) continue;
        const E *sa = (const E *)(smem + (slot0 - lds_u32(smem)) + (k % (PD + 1)) * SLOT);
        const E *sx = sa + (PK > 0 ? ABLK : NA * 1024 / ES);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
            const int e = ks * 4 + kq;
            E a = arow_ok ? (p.block_im_fast ? sa[ar + e * BI] : sa[ar * BD + e]) : E{};
            E b = bcol_ok ? sx[e * nc + ar] : E{};
            if constexpr (CPLX && M3) {
                accR = BsrMfma<R>::mma(a.x, b.x, accR);
                accI = BsrMfma<R>::mma(a.y, b.y, accI);
                acc3 = BsrMfma<R>::mma(a.x + a.y, b.x + b.y, acc3);
            } else if constexpr (CPLX) {
                accR = BsrMfma<R>::mma(a.x, b.x, accR);
                accI = BsrMfma<R>::mma(a.x, b.y, accI);
                accR = BsrMfma<R>::mma(-a.y, b.y, accR);
                accI = BsrMfma<R>::mma(a.y, b.x, accI);
            } else {
                accR = BsrMfma<R>::mma(a, b, accR);
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int row = BsrMfma<R>::row(lane, q);
        if (row >= BI || !bcol_ok) continue;
        const long img = i * BI + row;
        E *yp = YROW ? y + img * p.ldy + ar : y + img + ar * p.ldy;
        E out;
        if constexpr (CPLX && M3)
            out = Ops<E>::scale(E{accR[q] - accI[q], acc3[q] - accR[q] - accI[q]}, p.alpha_re,
                                p.alpha_im);
        else if constexpr (CPLX)
            out = Ops<E>::scale(E{accR[q], accI[q]}, p.alpha_re, p.alpha_im);
        else
            out = Ops<E>::scale(accR[q], p.alpha_re, p.alpha_im);
        *yp = p.add ? Ops<E>::add(*yp, out) : out;
    }
}

/// false: not this shape (the register-staged kernel runs)
template <typename R, bool CPLX, int BI, int BD, int NNZ, int PD>
bool launch_bsr_mfma_dma(const BsrArgs &a, bool yrow, hipStream_t s) {
    typedef typename BsrMfmaElem<R, CPLX>::type E;
    constexpr int ES = (int)sizeof(E);
    constexpr int NA = (BI * BD * ES + 1023) / 1024, NX = (BD * 16 * ES + 1023) / 1024;
    const long v_bytes = a.block_rows * NNZ * (long)BI * BD * ES, x_bytes = a.x_rows * a.ldx * (long)ES;
    if (a.x_rows <= 0 || x_bytes >= (1L << 31)) return false;
    const long blocks = (a.block_rows + 3) / 4;
    if (blocks >= (1L << 31)) return false;
    // packed slots (values then x in one run): the DMA instruction count of a block
    const bool m3 = CPLX && g_gemm_tune.m3 > 0;
    const long slot_packed = (long)(BI * BD + BD * a.ncols) * ES;
    // for 8-byte elements only (warm round robin, profiles/r02c_blk_pack.txt: the chain's
    // complex<float> operator 719 -> 693 us; complex<double> 327 -> 336 us)
    const bool want = ES == 8;
    const int pk = want && !m3 ? (int)((slot_packed + 1023) / 1024) : 0;
    // (16-byte aligned pieces: the x blocks of an nc-column row and both arrays)
    const bool packed = pk == (CPLX && ES == 16 ? 5 : 3) && a.ncols >= 1 && a.ncols <= 16 &&
                        (BD * a.ncols * ES) % 16 == 0 && ((size_t)a.x & 15) == 0 &&
                        ((size_t)a.v & 15) == 0;
    const size_t lds = packed ? (size_t)4 * slot_packed * (PD + 1) : (size_t)4 * (NA + NX) * 1024 * (PD + 1);
    // 4 waves x (PD + 1) ring slots; a packed slot's last instruction is masked to the slot
    // (lanes past it are inactive), an unpacked slot is NA + NX whole 64-lane instructions
    if (packed && !m3) {
        // the kernel's issue loop: PKN instructions per slot, lane l of instruction q writes the
        // 16 bytes at q * 1024 + 16 l of the slot when that offset is below the slot size; so a
        // slot's DMA writes min(PKN * 1024, slot rounded up to 16 bytes) bytes and must cover the
        // slot's data, and the ring of 4 waves x (PD + 1) slots, slot_packed bytes apart, must fit
        constexpr long PKN = CPLX && ES == 16 ? 5 : 3;
        const long written = std::min(PKN * 1024, (slot_packed + 15) / 16 * 16);
        if (PKN * 1024 < slot_packed || written > slot_packed)
            throw Error("bsr: internal packed-slot sizing error in bsr_mfma_dma_kernel");
        check_dma_lds("bsr_mfma_dma_kernel", lds, 0, 0, 4L * (PD + 1) * written);
    }
    else
        check_dma_lds("bsr_mfma_dma_kernel", lds, 4L * (PD + 1) * (NA + NX), 64);
    g_bsr_tune.last = packed && !m3 ? 8 : 7;
    KernelTimer timer("bsr", s);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, s, a, (unsigned)v_bytes, (unsigned)x_bytes);
    };
    if (packed && !m3) {
        constexpr int PKN = CPLX && ES == 16 ? 5 : 3;
        if (yrow) go(bsr_mfma_dma_kernel<R, CPLX, BI, BD, true, NNZ, PD, false, PKN>);
        else go(bsr_mfma_dma_kernel<R, CPLX, BI, BD, false, NNZ, PD, false, PKN>);
    } else if (yrow && m3) go(bsr_mfma_dma_kernel<R, CPLX, BI, BD, true, NNZ, PD, true>);
    else if (yrow) go(bsr_mfma_dma_kernel<R, CPLX, BI, BD, true, NNZ, PD, false>);
    else if (m3) go(bsr_mfma_dma_kernel<R, CPLX, BI, BD, false, NNZ, PD, true>);
    else go(bsr_mfma_dma_kernel<R, CPLX, BI, BD, false, NNZ, PD, false>);
    SBX_HIP_CHECK(hipGetLastError());
    return true;
}

template <typename R, bool CPLX, int BI, int BD>
void launch_bsr_mfma(const BsrArgs &a, int nnz, bool yrow, bool xrow, hipStream_t s) {
    // contiguous x blocks (row-major x, ldx == ncols <= 16), 9 blocks per row: the blocks staged
    // by LDS-DMA one ahead (16^4 complex<double> n = 12: 426 us for the round-1 fragment kernel,
    // 348-355 us staged; the chain's complex<float> operator 985 -> 693 us with packed slots;
    // two or three blocks of lookahead were slower, profiles/r02_bsr_blk_sweep.txt; round 6:
    // the value blocks straight into the MFMA fragments with x by LDS-DMA, 757 against 689 us on
    // the chain's operator, and a streaming form with 1-4 workgroups per CU whose waves stream
    // every W-th row through an 8-slot ring, 787-1221 against 695 us -- both removed again,
    // profiles/r06_bsr12_vreg_chain.txt, r06_bsr12_stream_chain.txt, commit ad3532b)
    if (g_bsr_tune.variant == 0 && nnz == 9 && xrow && a.ldx == a.ncols && a.ncols <= 16 &&
        (g_bsr_tune.blk_pd == 2   ? launch_bsr_mfma_dma<R, CPLX, BI, BD, 9, 2>(a, yrow, s)
         : g_bsr_tune.blk_pd == 3 ? launch_bsr_mfma_dma<R, CPLX, BI, BD, 9, 3>(a, yrow, s)
                                  : launch_bsr_mfma_dma<R, CPLX, BI, BD, 9, 1>(a, yrow, s)))
        return;
    // the 9-point stencils otherwise: columns preloaded, fragments one block ahead (a 3- or
    // 9-block lookahead, the XCD-grouped row order and non-temporal value loads were all
    // measured slower, non-temporal stores of y no faster); any other pattern: generic rows
    if (g_bsr_tune.variant != 1 && nnz == 9) return launch_bsr_mfma_ell<R, CPLX, BI, BD, 9, 1>(a, yrow, xrow, s);
    launch_bsr_mfma_pf<R, CPLX, BI, BD>(a, yrow, xrow, s);
}

template <typename E, int BI, int BD, int G>
void launch_ell_g(const BsrArgs &a, int nnz, bool yrow, bool xrow, hipStream_t s, long lds_bytes) {
    const long blk_bytes = (long)nnz * (BI * BD * (long)sizeof(E) + 4);
    const long ngroups = (a.ncols + G - 1) / G;
    int rb = (int)std::max(1L, lds_bytes / std::max(1L, blk_bytes));
    // about one (row, column group) per thread
    if (ngroups <= 256) rb = (int)std::min<long>(rb, std::max(1L, 256 / ngroups));
    const long blocks = (a.block_rows + rb - 1) / rb;
    if (blocks >= (1L << 31)) throw Error("bsr: grid too large");
    const size_t lds = (size_t)rb * blk_bytes;
    KernelTimer timer("bsr", s);
    if (yrow && xrow)
        hipLaunchKernelGGL((bsr_ell_kernel<E, BI, BD, G, true, true>), dim3(blocks), dim3(256), lds, s, a, nnz, rb);
    else if (yrow && !xrow)
        hipLaunchKernelGGL((bsr_ell_kernel<E, BI, BD, G, true, false>), dim3(blocks), dim3(256), lds, s, a, nnz, rb);
    else if (!yrow && xrow)
        hipLaunchKernelGGL((bsr_ell_kernel<E, BI, BD, G, false, true>), dim3(blocks), dim3(256), lds, s, a, nnz, rb);
    else
        hipLaunchKernelGGL((bsr_ell_kernel<E, BI, BD, G, false, false>), dim3(blocks), dim3(256), lds, s, a, nnz, rb);
    SBX_HIP_CHECK(hipGetLastError());
}


// 9-point ELL form of bsr_ell_kernel: each thread reads its block row's 9 block columns straight
// from global memory into registers and issues the x rows of its first PD blocks before the
// workgroup streams the values into LDS, so the x gathers, the column reads and the value stream
// are in flight together (bsr_ell_kernel: value stream, then the columns, then one x block at a
// time); blocks j+PD are fetched while block j is applied.
template <typename E, int BI, int BD, int G, int PD, bool YROW, bool XROW, int NT = 256,
          bool DMAV = false, bool SC = false>
__global__ void __launch_bounds__(NT) bsr_ell9_kernel(const BsrArgs p, int rb) {
    // SC: a thread's G columns are g, g + ngroups, ... (the lanes of one row read consecutive
    // columns in each load) instead of g*G .. g*G + G-1
    // DMAV: the values staged by LDS-DMA (16-byte elements; launcher: 32-bit offsets)
    static_assert(!DMAV || sizeof(E) == 16, "LDS-DMA staging takes 16-byte elements");
    constexpr int NNZ = 9, BLK = BI * BD, NB = PD + 1;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    E *vals = (E *)smem;
    const E *__restrict__ v = (const E *)p.v;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    // the XCD's range of chunks visited as p.ilv interleaved parts (bsr_ell9_split_kernel)
    const int cnt = xcd < r8 ? q8 + 1 : q8, qx = bid >> 3, npart = cnt / p.ilv;
    const int loc = (p.ilv > 1 && qx < npart * p.ilv) ? (qx % p.ilv) * npart + qx / p.ilv : qx;
    const int chunk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const long row0 = (long)chunk * rb;
    const int nrows = (int)min((long)rb, p.block_rows - row0);
    const long ngroups = (p.ncols + G - 1) / G;
    const long npairs = (long)nrows * ngroups; // <= 256 (launcher)
    const long q = threadIdx.x;
    const bool active = q < npairs;
    int r;
    long g;
    if (YROW) {
        r = (int)(q / ngroups);
        g = q % ngroups;
    } else {
        r = (int)(q % nrows);
        g = q / nrows;
    }
    if (!active) {
        r = 0;
        g = 0;
    }
    long colv[G];
#pragma unroll
    for (int k = 0; k < G; ++k) colv[k] = min(SC ? g + k * ngroups : g * G + k, p.ncols - 1);
    int dj[NNZ];
#pragma unroll
    for (int j = 0; j < NNZ; ++j) dj[j] = p.jj[(row0 + r) * NNZ + j];
    E xb[NB][BD][G];
    auto fetch = [&](int d0, E (*xv)[G]) {
        const long d = d0 < 0 ? 0 : d0;
#pragma unroll
        for (int e = 0; e < BD; ++e)
#pragma unroll
            for (int k = 0; k < G; ++k)
                xv[e][k] = XROW ? x[(d + e) * p.ldx + colv[k]] : x[(d + e) + colv[k] * p.ldx];
    };
#pragma unroll
    for (int j = 0; j < PD; ++j) fetch(dj[j], xb[j]);
    const long vbase = row0 * NNZ * BLK;
    const int nv = nrows * NNZ * BLK;
    if constexpr (DMAV) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)p.v, (short)0, (int)(p.block_rows * NNZ * BLK * 16), 0x00020000);
        const unsigned base = lds_u32(vals) + (unsigned)__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * 1024u;
        for (int u = 0; u * NT < nv; ++u) {
            const int e = u * NT + (int)threadIdx.x;
            const unsigned off = e < nv ? (unsigned)((vbase + e) * 16) : 0x80000000u;
            dma16(rs, off, __builtin_amdgcn_readfirstlane(base + (unsigned)(u * NT) * 16u), p.nt & 2);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
        for (int e0 = threadIdx.x; e0 < nv; e0 += NT * 8) {
            E t[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) t[u] = v[vbase + min(e0 + NT * u, nv - 1)];
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (e0 + NT * u < nv) vals[e0 + NT * u] = t[u];
        }
    }
    __syncthreads();
    if (!active) return;
    E acc[BI][G];
#pragma unroll
    for (int c = 0; c < BI; ++c)
#pragma unroll
        for (int k = 0; k < G; ++k) acc[c][k] = Ops<E>::zero();
    const E *vr = vals + r * NNZ * BLK;
#pragma unroll
    for (int j = 0; j < NNZ; ++j) {
        if (j + PD < NNZ) fetch(dj[j + PD], xb[(j + PD) % NB]);
        if (dj[j] < 0) continue;
        const E *vb = vr + j * BLK;
#pragma unroll
        for (int e = 0; e < BD; ++e)
#pragma unroll
            for (int c = 0; c < BI; ++c) {
                const E a = p.block_im_fast ? vb[c + e * BI] : vb[c * BD + e];
#pragma unroll
                for (int k = 0; k < G; ++k)
                    acc[c][k] = Ops<E>::fma(a, xb[j % NB][e][k], acc[c][k]);
            }
    }
#pragma unroll
    for (int c = 0; c < BI; ++c) {
        const long img = (row0 + r) * BI + c;
#pragma unroll
        for (int k = 0; k < G; ++k) {
            const long col = SC ? g + k * ngroups : g * G + k;
            if (col >= p.ncols) break;
            E *yp = YROW ? y + img * p.ldy + col : y + img + col * p.ldy;
            const E out = Ops<E>::scale(acc[c][k], p.alpha_re, p.alpha_im);
            *yp = p.add ? Ops<E>::add(*yp, out) : out;
        }
    }
}

// Site tiles with their halo in LDS (3x3 complex<double> blocks, 9 per row, many rhs columns;
// row-major x and y).  The rows are grouped into tiles of up to TT lattice sites (the host's
// schedule, bsr.cpp: 2x2x2x2 on a 4-d lattice for TT = 16, 2x2x2 for TT = 8) and a tile's distinct
// x rows -- its own sites and their halo, umax at most -- are staged once per slice of NS rhs
// columns into LDS by LDS-DMA (each x row 3 colours x NS columns, NS * 16-byte runs), so the nine
// neighbours of every row are read from LDS instead of nine gathers through the vector-memory
// path (5 staged rows per site instead of 9 fetched ones on the 9-point stencil at TT = 16, 6 at
// TT = 8).  The tile's values (TT x 9 blocks) are staged once and reused by every slice.  Thread
// (site s, colour i, column e) of TT x 3 x NS.
//
// LDS banks (ds_read_b128 serves a wave in four 16-lane groups, MI355X_MICROARCH.md LDS): the x
// piece (slot u, colour d, column e) sits at 16-byte unit u * 3 NS + d NS + e, whose 16-byte bank
// group is (u * 3 NS + d NS + e) mod 16.  NS = 8 (TT = 16): that is 8 ((u + d) mod 2) + e, so two
// sites of one lane group whose neighbour slots have the same parity read the same 8 bank groups:
// 2-way conflicts that depend on the schedule (round 5: 12.6 M conflict cycles per launch at 16^4,
// n = 64).  NS = 16 (TT = 8): the bank group is e alone, and the lane map (s, i, e) puts two sites
// in a lane group only with complementary column sets ({0-3, 12-15} against {4-11}), so no read
// of x conflicts whatever the slots; the colours of a site read the same piece (a broadcast).
struct TileArgs {
    const int *rows;          // [chunk][TT] block rows of the tile (-1: none)
    const int *uniq;          // [chunk][umax] first domain row of each distinct block column (-1: none)
    const unsigned char *loc; // [chunk][TT][9] slot of each nonzero block in uniq (255: skip)
    int umax;
};

__device__ __forceinline__ void dma16_lane(const void *src, unsigned m0, bool nt) {
    if (nt)
        asm volatile("s_mov_b32 m0, %1\n\t"
                     "s_nop 0\n\t"
                     "global_load_lds_dwordx4 %0, off nt"
                     :
                     : "v"(src), "s"(m0)
                     : "memory", "m0");
    else
        asm volatile("s_mov_b32 m0, %1\n\t"
                     "s_nop 0\n\t"
                     "global_load_lds_dwordx4 %0, off"
                     :
                     : "v"(src), "s"(m0)
                     : "memory", "m0");
}

// the x DMA passes of a slice: umax * 3 * NS pieces over TT * 3 * NS lanes (the launcher bounds umax)
template <int TT, int NS> struct TileForm {
    static constexpr int NT = TT * 3 * NS;
    static constexpr int UMAX = TT == 16 ? 128 : 80;
    static constexpr int MAXP = (UMAX * 3 * NS + NT - 1) / NT;
};

// Thread (site s, colour i, rhs column e) of TT x 3 x NS.  A slice's y stores are issued after
// the next slice's DMA, so the wait for that DMA (vmcnt(1)) leaves them in flight.
template <bool BIMF, int TT, int NS>
__global__ void __launch_bounds__(TT * 3 * NS) bsr_ell9_tile_kernel(const BsrArgs p, const TileArgs t, int nchunks) {
    typedef double2 E;
    constexpr int NNZ = 9, VP = TT * NNZ * 9, NT = TileForm<TT, NS>::NT; // value pieces (16 B)
    constexpr int MAXP = TileForm<TT, NS>::MAXP;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    E *vals = (E *)smem;
    E *xs = vals + VP;
    const int tid = threadIdx.x, w = tid >> 6;
    // XCD-contiguous ranges of tiles: neighbouring tiles share halo rows in that XCD's L2
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int chunk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    if (chunk >= nchunks) return;
    const int umax = t.umax, XP = umax * 3 * NS; // x pieces of a slice
    const int *rows = t.rows + (long)chunk * TT;
    const int *uq = t.uniq + (long)chunk * umax;
    const unsigned char *lc = t.loc + (long)chunk * TT * NNZ;
    const unsigned vbase = lds_u32(vals), xbase = lds_u32(xs);
    // the values of the tile's rows (read once: nt)
    const E *v = (const E *)p.v;
    for (int u = 0; u * NT < VP; ++u) {
        const int L = u * NT + tid;
        if (L < VP) {
            const int s = L / 81, r = rows[s];
            dma16_lane(v + (long)(r < 0 ? 0 : r) * 81 + (L - s * 81),
                       __builtin_amdgcn_readfirstlane(vbase + (unsigned)(u * NT + w * 64) * 16u), (p.nt & 2) != 0);
        }
    }
    // this lane's x pieces (pass u: distinct row pu, colour pd, column pe), the same every slice
    // (element offsets into x: 32 bits, the launcher checks x's size)
    unsigned src[MAXP];
    const E *x = (const E *)p.x;
#pragma unroll
    for (int u = 0; u < MAXP; ++u) {
        const int L = u * NT + tid;
        const int pu = L / (3 * NS), rem = L - pu * 3 * NS, pd = rem / NS, pe = rem - pd * NS;
        const int d = (L < XP) ? uq[L < XP ? pu : 0] : -1; // (the index clamped: no load past the list)
        src[u] = (unsigned)(((long)(d < 0 ? 0 : d) + pd) * p.ldx + pe);
    }
    auto stage = [&](int q) {
#pragma unroll
        for (int u = 0; u < MAXP; ++u) {
            const int L = u * NT + tid;
            if (u * NT < XP && L < XP)
                dma16_lane(x + src[u] + q * NS, __builtin_amdgcn_readfirstlane(xbase + (unsigned)(u * NT + w * 64) * 16u), false);
        }
    };
    // this thread's output and its nine slots
    const int e = tid % NS, i = (tid / NS) % 3, s = tid / (3 * NS);
    const int row = rows[s];
    const bool wave_stores = __ballot(row >= 0) != 0;
    int slot[NNZ];
#pragma unroll
    for (int k = 0; k < NNZ; ++k) slot[k] = lc[s * NNZ + k];
    const E *vr = vals + s * NNZ * 9;
    E *y = (E *)p.y;
    const int nslices = (int)(p.ncols / NS);
    stage(0);
    for (int q = 0; q < nslices; ++q) {
        // slice q landed (only the previous slice's y store, issued after it, may be pending; a
        // wave whose rows are all padding stores nothing: it waits for everything)
        if (q == 0 || !wave_stores) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
        __syncthreads();
        E acc = Ops<E>::zero();
#pragma unroll
        for (int k = 0; k < NNZ; ++k) {
            if (slot[k] == 255) continue;
            const E *xr = xs + slot[k] * 3 * NS + e;
            const E *vb = vr + k * 9;
#pragma unroll
            for (int d = 0; d < 3; ++d) acc = Ops<E>::fma(BIMF ? vb[i + d * 3] : vb[i * 3 + d], xr[d * NS], acc);
        }
        __syncthreads(); // every read of the buffer is done
        if (q + 1 < nslices) stage(q + 1);
        if (row >= 0) {
            E *yp = y + ((long)row * 3 + i) * p.ldy + q * NS + e;
            const E out = Ops<E>::scale(acc, p.alpha_re, p.alpha_im);
            *yp = p.add ? Ops<E>::add(*yp, out) : out;
        }
    }
}

/// false: no tile schedule, not this shape, or bsr.tile off.  bsr.tile 1: 16-site tiles, slices
/// of 8 columns (schedule 0); 2: 8-site tiles, slices of 16 columns (schedule 1)
bool launch_ell9_tile(const BsrArgs &a, bool yrow, bool xrow, hipStream_t s) {
    const int form = g_bsr_tune.tile;
    if (form != 1 && form != 2) return false;
    const TileSched &ts = a.tiles[form - 1];
    const int NS = form == 1 ? 8 : 16, TT = form == 1 ? 16 : 8;
    const int umax_cap = form == 1 ? TileForm<16, 8>::UMAX : TileForm<8, 16>::UMAX;
    if (!ts.rows || ts.tt != TT || !yrow || !xrow || a.ncols % NS != 0 || ts.umax < 1 ||
        ts.umax > umax_cap || ts.chunks >= (1L << 31) || a.ldx < a.ncols || a.ldy < a.ncols ||
        a.x_rows <= 0 || a.x_rows * a.ldx >= (1L << 32))
        return false;
    const TileArgs t{ts.rows, ts.uniq, ts.loc, ts.umax};
    const long vp = TT * 9L * 9, xp = ts.umax * 3L * NS;
    const size_t lds = (size_t)(vp + xp) * 16;
    // the DMA passes write lanes L < vp (values) and L < xp (x) only
    check_dma_lds("bsr_ell9_tile_kernel", lds, 1, vp + xp);
    g_bsr_tune.last = form == 1 ? 4 : 13;
    KernelTimer timer("bsr", s);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3((unsigned)ts.chunks), dim3(TT * 3 * NS), lds, s, a, t, (int)ts.chunks);
    };
    if (form == 1) {
        if (a.block_im_fast) go(bsr_ell9_tile_kernel<true, 16, 8>);
        else go(bsr_ell9_tile_kernel<false, 16, 8>);
    } else {
        if (a.block_im_fast) go(bsr_ell9_tile_kernel<true, 8, 16>);
        else go(bsr_ell9_tile_kernel<false, 8, 16>);
    }
    SBX_HIP_CHECK(hipGetLastError());
    return true;
}

template <typename E, int BI, int BD, int G, int PD, int NT = 256, bool DMAV = false, bool SC = false>
void launch_ell9(const BsrArgs &a, bool yrow, bool xrow, hipStream_t s, long lds_bytes) {
    const long blk_bytes = 9L * BI * BD * (long)sizeof(E);
    const long ngroups = (a.ncols + G - 1) / G;
    if (ngroups > NT) throw Error("bsr: internal ELL9 sizing error");
    int rb = (int)std::max(1L, lds_bytes / blk_bytes);
    rb = (int)std::min<long>(rb, std::max(1L, NT / ngroups));
    const long blocks = (a.block_rows + rb - 1) / rb;
    if (blocks >= (1L << 31)) throw Error("bsr: grid too large");
    if constexpr (DMAV)
        if (a.block_rows * blk_bytes >= (1L << 31)) return launch_ell9<E, BI, BD, G, PD, NT, false, SC>(a, yrow, xrow, s, lds_bytes);
    // the DMA form fills whole workgroup-wide rows of 16-byte lanes
    const size_t lds = DMAV ? (size_t)((rb * 9L * BI * BD + NT - 1) / NT * NT) * sizeof(E)
                            : (size_t)rb * blk_bytes;
    // the DMA loop: passes u < ceil(nv / NT) of NT lanes, nv <= rb * 81 (the last chunk fewer)
    if constexpr (DMAV) check_dma_lds("bsr_ell9_kernel", lds, (rb * 9L * BI * BD + NT - 1) / NT, NT);
    g_bsr_tune.last = 3;
    KernelTimer timer("bsr", s);
    if (yrow && xrow)
        hipLaunchKernelGGL((bsr_ell9_kernel<E, BI, BD, G, PD, true, true, NT, DMAV, SC>), dim3(blocks), dim3(NT), lds, s, a, rb);
    else if (yrow && !xrow)
        hipLaunchKernelGGL((bsr_ell9_kernel<E, BI, BD, G, PD, true, false, NT, DMAV, SC>), dim3(blocks), dim3(NT), lds, s, a, rb);
    else if (!yrow && xrow)
        hipLaunchKernelGGL((bsr_ell9_kernel<E, BI, BD, G, PD, false, true, NT, DMAV, SC>), dim3(blocks), dim3(NT), lds, s, a, rb);
    else
        hipLaunchKernelGGL((bsr_ell9_kernel<E, BI, BD, G, PD, false, false, NT, DMAV, SC>), dim3(blocks), dim3(NT), lds, s, a, rb);
    SBX_HIP_CHECK(hipGetLastError());
}

// Few rhs columns (n <= NC <= 4), 3x3 blocks, 9 per row: one thread per (block row, nonzero
// block).  The value stream is read by 9 x more threads than in the row-chunk kernel, without
// an LDS staging pass, and every thread has a single x gather (its block's domain rows) in
// flight beside its 9 values; the 9 partial products of a row are summed through LDS in block
// order.  At n = 1 the row-chunk kernel keeps one thread per row busy through 9 dependent
// gathers (18 of 256 threads of a workgroup active).
template <typename E, int NC, bool YROW, bool XROW, bool DMA>
__global__ void __launch_bounds__(256) bsr_ell9_row_kernel(const BsrArgs p, unsigned v_bytes) {
    constexpr int NNZ = 9, BI = 3, BD = 3, BLK = 9, RW = 28; // 28 rows x 9 blocks = 252 threads
    constexpr int NV = RW * NNZ * BLK, NP = RW * NNZ * BI * NC;
    constexpr int NS = (DMA ? (NV + 255) / 256 * 256 : 0) > NP ? (NV + 255) / 256 * 256 : NP;
    // static LDS: every DMA pass (256 lanes, the last one partly zeros) and the partial products
    static_assert((!DMA || NS >= (NV + 255) / 256 * 256) && NS >= NP, "LDS sizing");
    __shared__ __attribute__((aligned(16))) E sh[NS]; // values (DMA), then the partial products
    const E *__restrict__ v = (const E *)p.v;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const long chunk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int tid = threadIdx.x, rl = tid / NNZ, j = tid - rl * NNZ;
    const long row = chunk * RW + rl;
    const int ncols = (int)p.ncols;
    const bool active = rl < RW && row < p.block_rows;
    const long q = row * NNZ + j;
    int dj = -1;
    E xv[BD][NC];
    if (active) {
        dj = p.jj[q];
        const long d = dj < 0 ? 0 : dj;
#pragma unroll
        for (int e = 0; e < BD; ++e)
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                const long col = c < ncols ? c : 0;
                xv[e][c] = XROW ? x[(d + e) * p.ldx + col] : x[(d + e) + col * p.ldx];
            }
    }
    E a[BLK];
    if constexpr (DMA) {
        // the chunk's values, lane-linear into LDS (a contiguous run of the ELL value array)
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)p.v, (short)0, (int)v_bytes, 0x00020000);
        const unsigned base = lds_u32(sh) + (unsigned)__builtin_amdgcn_readfirstlane(tid >> 6) * 1024u;
        const unsigned v0 = (unsigned)(chunk * NV) * 16u;
#pragma unroll
        for (int u = 0; u < (NV + 255) / 256; ++u) {
            const unsigned e = (unsigned)(u * 256 + tid);
            const unsigned off = e < (unsigned)NV ? v0 + e * 16u : 0x80000000u;
            dma16(rs, off, __builtin_amdgcn_readfirstlane(base + (unsigned)u * 4096u), p.nt & 8);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (active) {
#pragma unroll
            for (int k = 0; k < BLK; ++k) a[k] = sh[(rl * NNZ + j) * BLK + k];
        }
        __syncthreads(); // the buffer now holds the partial products
    } else if (active) {
#pragma unroll
        for (int k = 0; k < BLK; ++k) a[k] = v[q * BLK + k];
    }
    E *part = sh;
    if (active) {
#pragma unroll
        for (int i = 0; i < BI; ++i)
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                E acc = Ops<E>::zero();
#pragma unroll
                for (int e = 0; e < BD; ++e)
                    acc = Ops<E>::fma(p.block_im_fast ? a[i + e * BI] : a[i * BD + e], xv[e][c], acc);
                part[((rl * NNZ + j) * BI + i) * NC + c] = dj < 0 ? Ops<E>::zero() : acc;
            }
    }
    __syncthreads();
    // sums: one thread per (row, i, column)
    for (int o = tid; o < RW * BI * ncols; o += 256) {
        const int r2 = o / (BI * ncols), rem = o - r2 * BI * ncols, i = rem / ncols, c = rem - i * ncols;
        const long rw = chunk * RW + r2;
        if (rw >= p.block_rows) continue;
        E acc = part[((r2 * NNZ) * BI + i) * NC + c];
#pragma unroll
        for (int jj = 1; jj < NNZ; ++jj) acc = Ops<E>::add(acc, part[((r2 * NNZ + jj) * BI + i) * NC + c]);
        const long img = rw * BI + i;
        E *yp = YROW ? y + img * p.ldy + c : y + img + (long)c * p.ldy;
        const E out = Ops<E>::scale(acc, p.alpha_re, p.alpha_im);
        *yp = p.add ? Ops<E>::add(*yp, out) : out;
    }
}

template <typename E, int NC>
void launch_ell9_row(const BsrArgs &a, bool yrow, bool xrow, hipStream_t s) {
    const long blocks = (a.block_rows + 27) / 28;
    if (blocks >= (1L << 31)) throw Error("bsr: grid too large");
    // the LDS-DMA form for 16-byte elements whose value array has 32-bit offsets
    const long v_bytes = a.block_rows * 81L * (long)sizeof(E);
    const bool dma = sizeof(E) == 16 && v_bytes < (1L << 31);
    g_bsr_tune.last = 1;
    KernelTimer timer("bsr", s);
    auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, a, (unsigned)v_bytes);
    };
    if (dma) {
        if (yrow && xrow) go(bsr_ell9_row_kernel<E, NC, true, true, true>);
        else if (yrow && !xrow) go(bsr_ell9_row_kernel<E, NC, true, false, true>);
        else if (!yrow && xrow) go(bsr_ell9_row_kernel<E, NC, false, true, true>);
        else go(bsr_ell9_row_kernel<E, NC, false, false, true>);
    } else {
        if (yrow && xrow) go(bsr_ell9_row_kernel<E, NC, true, true, false>);
        else if (yrow && !xrow) go(bsr_ell9_row_kernel<E, NC, true, false, false>);
        else if (!yrow && xrow) go(bsr_ell9_row_kernel<E, NC, false, true, false>);
        else go(bsr_ell9_row_kernel<E, NC, false, false, false>);
    }
    SBX_HIP_CHECK(hipGetLastError());
}

// Rows split over their nonzero blocks, 3x3 complex<double> blocks, 9 per row, row-major x, from
// 4 rhs columns on: one thread per (block row, group of JB nonzero blocks, rhs lane g), the lane
// computing columns g, g + nct, ... (CW of them; nct = ceil(ncols / CW) lanes per block group).
//  * Every thread issues the x rows of its JB blocks at once (JB x 3 x CW independent 16-byte
//    loads, no chain of dependent gathers), the nct lanes of a block group read whole runs of a
//    domain row (12 columns: 192 B pieces; the row-chunk kernel's lanes read 96 B pieces, which
//    the vector-memory pipeline serves ~1.4x slower from the Infinity Cache,
//    tools/gather_shape.hip), through 32-bit buffer offsets (one multiply per block instead of
//    six 64-bit address computations).
//  * The workgroup's block values (one contiguous run) are staged by LDS-DMA and read from LDS,
//    broadcast across the lanes of a block group.
//  * The 9 / JB partial products of a row are summed through LDS in block order.
__device__ __forceinline__ unsigned fdiv(unsigned n, unsigned m, int s) {
    return (unsigned)(((unsigned long long)__umulhi(n, m) + n) >> s);
}

static void magic(unsigned d, unsigned &m, int &s) {
    s = 0;
    while ((1ull << s) < d) ++s;
    m = (unsigned)((((1ull << 32) * ((1ull << s) - d)) / d) + 1);
}

struct SplitArgs {
    int nct, tpr, rw; // lanes per block group, threads per row, rows per workgroup
    unsigned v_bytes, x_bytes;
    unsigned tpr_m, nct_m; // magic multipliers and shifts of tpr and nct (fdiv)
    int tpr_s, nct_s;
    int ilv; // an XCD's chunks visited as ilv interleaved parts (x rows reused across parts)
    int ovl; // the partial products overwrite the staged values (one more barrier, half the LDS)
};

template <int CW, int JB, bool YROW>
__global__ void __launch_bounds__(512) bsr_ell9_split_kernel(const BsrArgs p, const SplitArgs s) {
    constexpr int NNZ = 9, NG = NNZ / JB;
    static_assert(NNZ % JB == 0, "JB divides 9");
    extern __shared__ __attribute__((aligned(16))) char smem[];
    double2 *vals = (double2 *)smem;
    const int nth = blockDim.x, tid = threadIdx.x;
    const int nwg = gridDim.x, bid = blockIdx.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    // the XCD's contiguous range of chunks, its parts interleaved: with ilv = 2 the two halves
    // (on the 16^4 lattice: the XCD's two x slices) are visited together, so a site's +-x
    // neighbour rows are read while the other half still holds them in this XCD's L2
    const int cnt = xcd < r8 ? q8 + 1 : q8, q = bid >> 3, npart = cnt / s.ilv;
    const int loc = (s.ilv > 1 && q < npart * s.ilv) ? (q % s.ilv) * npart + q / s.ilv : q;
    const long chunk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const long row0 = chunk * s.rw;
    const int nrows = (int)min((long)s.rw, p.block_rows - row0);
    const int nv = nrows * NNZ * 9, nvp = (s.rw * NNZ * 9 + nth - 1) / nth * nth;
    double2 *part = s.ovl ? vals : vals + nvp;
    const int rl = (int)fdiv(tid, s.tpr_m, s.tpr_s), rem = tid - rl * s.tpr;
    const int jg = (int)fdiv(rem, s.nct_m, s.nct_s), g = rem - jg * s.nct;
    const bool active = rl < nrows;
    const int ncs = s.nct * CW; // padded columns of a partial-product row
    // 1) the x rows of the thread's JB blocks
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc((void *)p.x, (short)0, (int)s.x_bytes, 0x00020000);
    const unsigned rowb = (unsigned)p.ldx * 16u;
    int dj[JB];
    double2 xv[JB][3][CW];
#pragma unroll
    for (int b = 0; b < JB; ++b) dj[b] = active ? p.jj[(row0 + rl) * NNZ + jg * JB + b] : -1;
    // the lane's columns, clamped to the last one (the surplus lanes' results are not stored)
    unsigned colb[CW];
#pragma unroll
    for (int k = 0; k < CW; ++k) colb[k] = (unsigned)min(g + k * s.nct, (int)p.ncols - 1) * 16u;
#pragma unroll
    for (int b = 0; b < JB; ++b) {
        // skipped blocks (-1) read zero beyond the buffer range; the block's 3 domain rows by the
        // uniform offset e * rowb
        const unsigned vb = dj[b] < 0 ? 0x80000000u : (unsigned)dj[b] * rowb;
#pragma unroll
        for (int e = 0; e < 3; ++e)
#pragma unroll
            for (int k = 0; k < CW; ++k) {
                const auto t = __builtin_amdgcn_raw_buffer_load_b128(rx, vb + colb[k], (unsigned)e * rowb, 0);
                xv[b][e][k] = __builtin_bit_cast(double2, t);
            }
    }
    // 2) the workgroup's block values, lane-linear into LDS
    {
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc((void *)p.v, (short)0, (int)s.v_bytes, 0x00020000);
        const unsigned base = lds_u32(vals) + (unsigned)__builtin_amdgcn_readfirstlane(tid >> 6) * 1024u;
        const unsigned v0 = (unsigned)(row0 * NNZ * 9) * 16u;
        for (int u = 0; u * nth < nv; ++u) {
            const int e = u * nth + tid;
            const unsigned off = e < nv ? v0 + (unsigned)e * 16u : 0x80000000u;
            dma16(rs, off, __builtin_amdgcn_readfirstlane(base + (unsigned)(u * nth) * 16u), p.nt & 4);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    // 3) the partial products of the thread's blocks
    double2 acc[3][CW];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < CW; ++k) acc[c][k] = double2{0, 0};
    if (active) {
#pragma unroll
        for (int b = 0; b < JB; ++b) {
            if (dj[b] < 0) continue;
            const double2 *vb = vals + (rl * NNZ + jg * JB + b) * 9;
#pragma unroll
            for (int e = 0; e < 3; ++e)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    const double2 a = p.block_im_fast ? vb[c + e * 3] : vb[c * 3 + e];
#pragma unroll
                    for (int k = 0; k < CW; ++k) acc[c][k] = Ops<double2>::fma(a, xv[b][e][k], acc[c][k]);
                }
        }
    }
    auto store = [&](long img, int col, double2 v) {
        double2 *yp = YROW ? (double2 *)p.y + img * p.ldy + col : (double2 *)p.y + img + (long)col * p.ldy;
        const double2 out = Ops<double2>::scale(v, p.alpha_re, p.alpha_im);
        *yp = p.add ? Ops<double2>::add(*yp, out) : out;
    };
    if constexpr (NG == 1) {
        if (!active) return;
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int k = 0; k < CW; ++k) {
                const int col = g + k * s.nct;
                if (col < p.ncols) store((row0 + rl) * 3 + c, col, acc[c][k]);
            }
    } else {
        if (s.ovl) __syncthreads(); // every thread is done reading the values
        if (active) {
#pragma unroll
            for (int c = 0; c < 3; ++c)
#pragma unroll
                for (int k = 0; k < CW; ++k) part[((rl * NG + jg) * 3 + c) * ncs + g + k * s.nct] = acc[c][k];
        }
        __syncthreads();
        // 4) sums in block order: the lanes of block group c < 3 sum image component c
        if (!active || jg >= 3) return;
#pragma unroll
        for (int k = 0; k < CW; ++k) {
            const int col = g + k * s.nct;
            if (col >= p.ncols) break;
            const double2 *pp = part + ((rl * NG) * 3 + jg) * ncs + col;
            double2 sum = pp[0];
#pragma unroll
            for (int q = 1; q < NG; ++q) sum = Ops<double2>::add(sum, pp[q * 3 * ncs]);
            store((row0 + rl) * 3 + jg, col, sum);
        }
    }
}

/// false: not this shape (the caller falls back to the row-chunk kernel)
template <typename E>
bool launch_ell9_split(const BsrArgs &a, bool yrow, bool xrow, hipStream_t st) {
    if constexpr (!std::is_same<E, double2>::value) {
        return false;
    } else {
        if (!xrow || a.ncols < 1) return false;
        const long x_bytes = a.x_rows * a.ldx * 16L;
        const long v_bytes = a.block_rows * 81L * 16L;
        if (v_bytes >= (1L << 31) || a.block_rows * 36L >= (1L << 31)) return false;
        if (a.x_rows <= 0 || x_bytes >= (1L << 31)) return false;
        // defaults from tools/bsr_split_sweep.py (16^4, profiles/r02_bsr_split_sweep.txt)
        int cw = g_bsr_tune.split_cw;
        if (cw <= 0) cw = a.ncols <= 4 ? 1 : 2;
        int jb = g_bsr_tune.split_jb;
        if (jb <= 0) jb = a.ncols <= 24 ? 3 : 9;
        // the forms the defaults use (the sweep's other forms were slower everywhere)
        if ((cw != 1 && cw != 2) || (jb != 3 && jb != 9)) return false;
        const int nct = (int)((a.ncols + cw - 1) / cw), tpr = 9 / jb * nct;
        const int ntmax = 256; // 512-thread workgroups measured slower (profiles/r02c_split_ovl.txt)
        if (tpr > ntmax) return false;
        // rows per workgroup: by the thread budget and at most 40 KB of LDS; the partial products
        // overlay the staged values (one more barrier, four workgroups per CU instead of three)
        const bool ovl = true;
        const long part_row = jb == 9 ? 0L : (long)(9 / jb) * 3 * nct * cw * 16;
        const long row_lds = std::max(81L * 16, part_row);
        const int rw = std::max(1, std::min<int>(ntmax / tpr, (int)(40960 / row_lds)));
        const int nth = (rw * tpr + 63) / 64 * 64;
        const long nvp = (rw * 81L + nth - 1) / nth * nth;
        const long npart = jb == 9 ? 0L : (long)rw * (9 / jb) * 3 * nct * cw;
        const long lds = (ovl ? std::max(nvp, npart) : nvp + npart) * 16L;
        if (lds > 65536) return false;
        // DMA passes u < ceil(nv / nth) of nth lanes (nv <= rw * 81); the partial products
        // overlay them (ovl) or follow them
        check_dma_lds("bsr_ell9_split_kernel", (size_t)lds, (rw * 81L + nth - 1) / nth, nth,
                      ovl ? 0 : npart * 16);
        check_dma_lds("bsr_ell9_split_kernel partials", (size_t)lds, 0, 0,
                      (ovl ? 0 : nvp * 16) + npart * 16);
        SplitArgs sa{nct, tpr, rw, (unsigned)v_bytes, (unsigned)x_bytes, 0, 0, 0, 0,
                     std::max(1, g_bsr_tune.split_ilv), ovl ? 1 : 0};
        magic((unsigned)tpr, sa.tpr_m, sa.tpr_s);
        magic((unsigned)nct, sa.nct_m, sa.nct_s);
        const long nchunks = (a.block_rows + rw - 1) / rw;
        if (nchunks >= (1L << 31)) return false;
        g_bsr_tune.last = 2;
        KernelTimer timer("bsr", st);
        auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(nchunks), dim3(nth), (size_t)lds, st, a, sa); };
#define SBX_SPLIT(CW_, JB_)                                                                        \
    if (cw == CW_ && jb == JB_) {                                                                  \
        if (yrow) go(bsr_ell9_split_kernel<CW_, JB_, true>);                                       \
        else go(bsr_ell9_split_kernel<CW_, JB_, false>);                                           \
    }
        SBX_SPLIT(1, 3) SBX_SPLIT(1, 9) SBX_SPLIT(2, 3) SBX_SPLIT(2, 9)
#undef SBX_SPLIT
        SBX_HIP_CHECK(hipGetLastError());
        return true;
    }
}

template <typename E, int BI, int BD>
void launch_ell(const BsrArgs &a, int nnz, bool yrow, bool xrow, hipStream_t s) {
    // two rhs columns per thread (measured against 1 and 4, and 48 KB of LDS per workgroup:
    // 16^4 3x3 n = 12: 46 us vs 51 / 61; n = 64: 191 us vs 218 / 234; one column per thread
    // over all 256 threads with the x rows of all 9 blocks in flight: 56-60 us; non-temporal
    // loads of the value stream: 50 us)
    // the 9-point stencils: ell9 with 12 KB of values per workgroup from 8 rhs columns on, else
    // 24 KB (16^4 3x3: n = 1 30.6 -> 26.5 us, n = 4 33.3 -> 28.1, n = 12 47.3 -> 42.9, n = 64
    // 190 -> 181-188; at n = 12 6 / 8 / 16 / 24 KB: 72 / 52 / 48 / 45 us; one or four columns
    // per thread, or the x rows of two blocks ahead: 46-82 us).  The x gathers are the bound:
    // without them the value stream and y run at 5.5 TB/s (22 us at n = 12).
    if constexpr (BI == 3 && BD == 3) {
        if (nnz == 9 && g_bsr_tune.variant != 1 && a.ncols <= g_bsr_tune.row_max_cols) {
            if (a.ncols == 1) return launch_ell9_row<E, 1>(a, yrow, xrow, s);
            if (a.ncols == 2) return launch_ell9_row<E, 2>(a, yrow, xrow, s);
            if (a.ncols <= 4) return launch_ell9_row<E, 4>(a, yrow, xrow, s);
        }
        if (nnz == 9 && g_bsr_tune.variant != 1 && a.ncols > g_bsr_tune.row_max_cols &&
            a.ncols <= g_bsr_tune.split_max_cols && launch_ell9_split<E>(a, yrow, xrow, s))
            return;
    }
    if constexpr (std::is_same<E, double2>::value && BI == 3 && BD == 3) {
        if (nnz == 9 && g_bsr_tune.variant != 1 && g_bsr_tune.tile && a.ncols >= g_bsr_tune.tile_min_cols &&
            launch_ell9_tile(a, yrow, xrow, s))
            return;
    }
    // (the row-chunk kernel takes at most 2 x 256 rhs columns per workgroup row)
    if (nnz == 9 && g_bsr_tune.variant != 1 && a.ncols <= 512) {
        const long lds = a.ncols >= 8 ? 12288 : 24576;
        // 16-byte elements: values by LDS-DMA, a row's lanes on consecutive columns (n = 12:
        // 42 -> 39 us, n = 24: 67 -> 61, n = 64: 182 -> 172; profiles/r02_bsr_sweep.txt; 64- and
        // 128-thread workgroups, two blocks of x lookahead, non-temporal value loads or y stores
        // were slower)
        if constexpr (sizeof(E) == 16) return launch_ell9<E, BI, BD, 2, 1, 256, true, true>(a, yrow, xrow, s, lds);
        else return launch_ell9<E, BI, BD, 2, 1>(a, yrow, xrow, s, lds);
    }
    launch_ell_g<E, BI, BD, 2>(a, nnz, yrow, xrow, s, ELL_LDS_BYTES);
}

template <typename E, int BI, int BD>
void launch_layouts(const BsrArgs &a, bool yrow, bool xrow, long blocks, hipStream_t s) {
    KernelTimer timer("bsr", s);
    if (yrow && xrow)
        hipLaunchKernelGGL((bsr_kernel<E, BI, BD, true, true>), dim3(blocks), dim3(256), 0, s, a);
    else if (yrow && !xrow)
        hipLaunchKernelGGL((bsr_kernel<E, BI, BD, true, false>), dim3(blocks), dim3(256), 0, s, a);
    else if (!yrow && xrow)
        hipLaunchKernelGGL((bsr_kernel<E, BI, BD, false, true>), dim3(blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((bsr_kernel<E, BI, BD, false, false>), dim3(blocks), dim3(256), 0, s,
                           a);
    SBX_HIP_CHECK(hipGetLastError());
}

template <typename E>
void launch_typed(const BsrArgs &a, int nnz_per_row, bool yrow, bool xrow, hipStream_t s) {
    const long total = a.block_rows * a.bi * a.ncols;
    const long blocks = std::min((total + 255) / 256, 65536L);
    const bool ell = nnz_per_row > 0 &&
                     (long)nnz_per_row * (a.bi * a.bd * (long)sizeof(E) + 4) <= ELL_LDS_BYTES;
    if (ell && a.bi == 3 && a.bd == 3)
        launch_ell<E, 3, 3>(a, nnz_per_row, yrow, xrow, s);
    else if (a.bi == 3 && a.bd == 3)
        launch_layouts<E, 3, 3>(a, yrow, xrow, blocks, s);
    else if (a.bi == 12 && a.bd == 12) {
        // one block row per wave: interleaving 2 or 4 rows per wave measured 6 % / 25 % slower
        // (more VGPRs, fewer waves to hide the HBM latency of the value stream)
        if constexpr (std::is_same<E, double2>::value)
            launch_bsr_mfma<double, true, 12, 12>(a, nnz_per_row, yrow, xrow, s);
        else if constexpr (std::is_same<E, double>::value)
            launch_bsr_mfma<double, false, 12, 12>(a, nnz_per_row, yrow, xrow, s);
        else if constexpr (std::is_same<E, float2>::value)
            launch_bsr_mfma<float, true, 12, 12>(a, nnz_per_row, yrow, xrow, s);
        else
            launch_bsr_mfma<float, false, 12, 12>(a, nnz_per_row, yrow, xrow, s);
    }
    else
        launch_layouts<E, 0, 0>(a, yrow, xrow, blocks, s);
}

template <typename E> __device__ __forceinline__ E conj_of(E v) { return v; }
template <> __device__ __forceinline__ double2 conj_of<double2>(double2 v) { return double2{v.x, -v.y}; }
template <> __device__ __forceinline__ float2 conj_of<float2>(float2 v) { return float2{v.x, -v.y}; }

template <typename E>
__global__ void __launch_bounds__(256) gather_blocks_kernel(const E *__restrict__ src,
                                                            const int *__restrict__ perm,
                                                            long nblocks, long be, int conj,
                                                            E *__restrict__ dst) {
    const long total = nblocks * be;
    for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256L) {
        const long q = idx / be, e = idx - q * be;
        const E v = src[(long)perm[q] * be + e];
        dst[idx] = conj ? conj_of<E>(v) : v;
    }
}

template <typename E>
void gather_typed(const void *src, const int *perm, long nblocks, long be, bool cj, void *dst,
                  hipStream_t s) {
    const long blocks = std::min((nblocks * be + 255) / 256, 65536L);
    hipLaunchKernelGGL(gather_blocks_kernel<E>, dim3((unsigned)blocks), dim3(256), 0, s,
                       (const E *)src, perm, nblocks, be, cj ? 1 : 0, (E *)dst);
    SBX_HIP_CHECK(hipGetLastError());
}

} // namespace

void launch_gather_blocks(int t, const void *src, const int *perm, long nblocks, long block_elems,
                          bool conj_values, void *dst, int device) {
    if (nblocks == 0 || block_elems == 0) return;
    set_device(device);
    hipStream_t s = get_stream(device);
    switch (t) {
    case SBX_CDOUBLE: return gather_typed<double2>(src, perm, nblocks, block_elems, conj_values, dst, s);
    case SBX_CFLOAT: return gather_typed<float2>(src, perm, nblocks, block_elems, conj_values, dst, s);
    case SBX_DOUBLE: return gather_typed<double>(src, perm, nblocks, block_elems, false, dst, s);
    case SBX_FLOAT: return gather_typed<float>(src, perm, nblocks, block_elems, false, dst, s);
    default: throw Error("bsr: unsupported type");
    }
}

void launch_bsr(const BsrDesc &d, int device) {
    if (d.block_rows == 0 || d.ncols == 0) return;
    g_bsr_tune.last = 0;
    set_device(device);
    hipStream_t s = get_stream(device);
    BsrArgs a{};
    a.block_rows = d.block_rows;
    a.bi = d.bi;
    a.bd = d.bd;
    a.ii = d.ii;
    a.jj = d.jj;
    a.v = d.v;
    a.block_im_fast = d.block_im_fast ? 1 : 0;
    a.x = d.x;
    a.ldx = d.ldx;
    a.x_rows = d.x_rows;
    a.y = d.y;
    a.ldy = d.ldy;
    a.ncols = d.ncols;
    a.alpha_re = d.alpha.re;
    a.alpha_im = d.alpha.im;
    a.add = d.add ? 1 : 0;
    a.ilv = 2; // an XCD's row chunks visited as two interleaved halves (bsr_ell9_kernel)
    a.nt = g_bsr_tune.nt;
    a.tiles[0] = d.tiles[0];
    a.tiles[1] = d.tiles[1];
    switch (d.t) {
    case SBX_CDOUBLE: return launch_typed<double2>(a, d.num_nnz_per_row, d.y_row_major, d.x_row_major, s);
    case SBX_CFLOAT: return launch_typed<float2>(a, d.num_nnz_per_row, d.y_row_major, d.x_row_major, s);
    case SBX_DOUBLE: return launch_typed<double>(a, d.num_nnz_per_row, d.y_row_major, d.x_row_major, s);
    case SBX_FLOAT: return launch_typed<float>(a, d.num_nnz_per_row, d.y_row_major, d.x_row_major, s);
    default: throw Error("bsr: unsupported type");
    }
}

} // namespace sbx
