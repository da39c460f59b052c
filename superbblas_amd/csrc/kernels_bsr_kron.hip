// Kronecker BSR operator times dense tensor (the Wilson-type stencil: a color block per
// direction times a spin matrix shared by all sites of that direction).
//
// Reference: create_kron_bsr (bsr.h:2476-2490), get_kron_indices (bsr.h:1485-1537), the builtin
// CPU operator (bsr.h:587-648) and BSR<Gpu>::contract_kron_cols + hipsparseXbsrmm
// (bsr.h:933-998, 1001-1029):
//   y(I, i, n, a) = alpha * sum_mu sum_b K_mu(a, b) sum_d U_{I,mu}(i, d) x(J(I,mu), d, n, b)
// with mu the position of the nonzero within its block row (every row has the same count).
// Layout (row major, SlowToFast): x (site, d, n, b), y (site, i, n, a): one thread per
// (block row, rhs column) owns the bi*ki outputs of that pair, reads bd*kd contiguous x values
// per neighbour (consecutive lanes -> consecutive rhs columns -> contiguous 16*kd-byte pieces),
// and the spin matrix K_mu is wave-uniform (scalar loads; zero entries -- half of a Wilson
// projector -- are skipped with a scalar branch).
#include "elem_ops.h"
#include "sbx_internal.h"

#include <algorithm>
#include <type_traits>

namespace sbx {
namespace {

struct KronArgs {
    long block_rows;
    int nnz; ///< nonzero blocks per block row
    int bi, bd, ki, kd;
    const int *jj; ///< domain site of nonzero r*nnz + mu
    const void *v;
    const void *kron;
    int block_im_fast;
    const void *x;
    void *y;
    long ncols;
    double alpha_re, alpha_im;
    int add;
    int ylds; ///< the XL kernels: y written through the wave's LDS ring in whole 64-B spin pieces
    long x_rows; ///< domain rows of x (sites * bd): the extent x's LDS-DMA buffer offsets address
    const int *perm; ///< the spin-first kernel: block row of each row slot (nullptr: the identity)
    const void *ktab; ///< ... the spin matrices' rows as two terms (bsr.cpp build_kron_terms)
    const void *xtab; ///< ... as diagonal + XOR partner (nullptr: not of that form)
};

template <typename E, int BI, int BD, int KI, int KD>
__global__ void __launch_bounds__(256) bsr_kron_kernel(const KronArgs p) {
    const E *__restrict__ v = (const E *)p.v;
    const E *__restrict__ kron = (const E *)p.kron;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    const long total = p.block_rows * p.ncols;
    const long xsite = (long)BD * p.ncols * KD, xrow = p.ncols * KD;
    for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256L) {
        const long c = idx % p.ncols, r = idx / p.ncols;
        E acc[BI][KI];
#pragma unroll
        for (int i = 0; i < BI; ++i)
#pragma unroll
            for (int a = 0; a < KI; ++a) acc[i][a] = Ops<E>::zero();
        for (int mu = 0; mu < p.nnz; ++mu) {
            const long j = r * p.nnz + mu;
            const E *xs = x + p.jj[j] * xsite + c * KD;
            E xv[BD][KD];
#pragma unroll
            for (int d = 0; d < BD; ++d)
#pragma unroll
                for (int b = 0; b < KD; ++b) xv[d][b] = xs[d * xrow + b];
            // spin first: xk(d, a) = sum_b K_mu(a, b) x(d, b)
            const E *K = kron + (long)mu * KI * KD;
            E xk[BD][KI];
#pragma unroll
            for (int d = 0; d < BD; ++d)
#pragma unroll
                for (int a = 0; a < KI; ++a) xk[d][a] = Ops<E>::zero();
#pragma unroll
            for (int a = 0; a < KI; ++a)
#pragma unroll
                for (int b = 0; b < KD; ++b) {
                    const E k = p.block_im_fast ? K[a + b * KI] : K[a * KD + b];
                    if (!Ops<E>::nonzero(k)) continue;
#pragma unroll
                    for (int d = 0; d < BD; ++d) xk[d][a] = Ops<E>::fma(k, xv[d][b], xk[d][a]);
                }
            // color: acc(i, a) += sum_d U(i, d) xk(d, a)
            const E *U = v + j * BI * BD;
#pragma unroll
            for (int i = 0; i < BI; ++i)
#pragma unroll
                for (int d = 0; d < BD; ++d) {
                    const E u = p.block_im_fast ? U[i + d * BI] : U[i * BD + d];
#pragma unroll
                    for (int a = 0; a < KI; ++a) acc[i][a] = Ops<E>::fma(u, xk[d][a], acc[i][a]);
                }
        }
        E *ys = y + (r * BI * p.ncols + c) * KI;
#pragma unroll
        for (int i = 0; i < BI; ++i)
#pragma unroll
            for (int a = 0; a < KI; ++a) {
                E o = Ops<E>::scale(acc[i][a], p.alpha_re, p.alpha_im);
                if (p.add) o = Ops<E>::add(o, ys[i * p.ncols * KI + a]);
                ys[i * p.ncols * KI + a] = o;
            }
    }
}

/// s_waitcnt vmcnt(n) for an n the unrolled caller knows at compile time (folds to one wait)
__device__ __forceinline__ void wait_vmcnt(int n) {
    switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    }
}

/// Wave-uniform element load through the constant address space (scalar loads into SGPRs)
template <typename R> using ConstPtr = const __attribute__((address_space(4))) R *;
template <typename E> struct Uniform {
    static __device__ __forceinline__ E load(const E *p, long i) {
        return ((ConstPtr<E>)p)[i];
    }
};
template <> struct Uniform<double2> {
    static __device__ __forceinline__ double2 load(const double2 *p, long i) {
        const ConstPtr<double> q = (ConstPtr<double>)p;
        return double2{q[2 * i], q[2 * i + 1]};
    }
};
template <> struct Uniform<float2> {
    static __device__ __forceinline__ float2 load(const float2 *p, long i) {
        const ConstPtr<float> q = (ConstPtr<float>)p;
        return float2{q[2 * i], q[2 * i + 1]};
    }
};

/// Many rhs columns: a workgroup owns `S` consecutive block rows x up to 256 columns; the color
/// blocks of its rows (S * NNZ * BI * BD values, contiguous in memory) and their domain sites are
/// staged in LDS with coalesced loads (instead of every lane of a row fetching the same 9 blocks
/// through L1), the spin matrices are read through the constant address space so that they live
/// in SGPRs (wave-uniform operands of the FMAs), and the x values of the next nonzero are loaded
/// while the current one is being applied (the loop over the NNZ nonzeros is unrolled).
template <typename E, int BI, int BD, int KI, int KD, int NNZ>
__global__ void __launch_bounds__(256) bsr_kron_lds_kernel(const KronArgs p, int S, int cpg) {
    extern __shared__ char smem[];
    constexpr int BLK = BI * BD * NNZ;
    E *Us = (E *)smem;
    int *Js = (int *)(Us + (long)S * BLK);
    const E *__restrict__ v = (const E *)p.v;
    const E *kron = (const E *)p.kron;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    // consecutive chunks of block rows on one XCD: neighbouring sites share x lines in its L2
    const int nwg = gridDim.x * gridDim.y, bid = blockIdx.x + blockIdx.y * gridDim.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int gx = wg % gridDim.x, gy = wg / gridDim.x;
    const long r0 = (long)gx * S;
    const int nrows = (int)std::min<long>(S, p.block_rows - r0);
    {
        const E *src = v + r0 * BLK;
        for (int e = threadIdx.x; e < nrows * BLK; e += 256) Us[e] = src[e];
        const int *jsrc = p.jj + r0 * NNZ;
        for (int e = threadIdx.x; e < nrows * NNZ; e += 256) Js[e] = jsrc[e];
    }
    __syncthreads();
    const int sl = threadIdx.x / cpg;
    const long c = (long)gy * cpg + threadIdx.x % cpg;
    if (sl >= nrows || c >= p.ncols) return;
    const long r = r0 + sl;
    const long xsite = (long)BD * p.ncols * KD, xrow = p.ncols * KD;
    const E *xc = x + c * KD;
    E acc[BI][KI];
#pragma unroll
    for (int i = 0; i < BI; ++i)
#pragma unroll
        for (int a = 0; a < KI; ++a) acc[i][a] = Ops<E>::zero();
    const E *Ur = Us + sl * BLK;
    const int *Jr = Js + sl * NNZ;
    E xa[BD][KD];
    {
        const E *xs = xc + Jr[0] * xsite;
#pragma unroll
        for (int d = 0; d < BD; ++d)
#pragma unroll
            for (int b = 0; b < KD; ++b) xa[d][b] = xs[d * xrow + b];
    }
#pragma unroll 1
    for (int mu = 0; mu < NNZ; ++mu) {
        E xb[BD][KD];
        if (mu + 1 < NNZ) {
            const E *xs = xc + Jr[mu + 1] * xsite;
#pragma unroll
            for (int d = 0; d < BD; ++d)
#pragma unroll
                for (int b = 0; b < KD; ++b) xb[d][b] = xs[d * xrow + b];
        }
        const E *K = kron + mu * KI * KD;
        const E *U = Ur + mu * BI * BD;
#pragma unroll
        for (int d = 0; d < BD; ++d) {
            // spin: xk(a) = sum_b K_mu(a, b) x(d, b)
            E xk[KI];
#pragma unroll
            for (int a = 0; a < KI; ++a) {
                xk[a] = Ops<E>::zero();
#pragma unroll
                for (int b = 0; b < KD; ++b)
                    xk[a] = Ops<E>::fma(
                        Uniform<E>::load(K, p.block_im_fast ? a + b * KI : a * KD + b), xa[d][b],
                        xk[a]);
            }
            // color: acc(i, a) += U(i, d) xk(a)
#pragma unroll
            for (int i = 0; i < BI; ++i) {
                const E u = p.block_im_fast ? U[i + d * BI] : U[i * BD + d];
#pragma unroll
                for (int a = 0; a < KI; ++a) acc[i][a] = Ops<E>::fma(u, xk[a], acc[i][a]);
            }
        }
        if (mu + 1 < NNZ) {
#pragma unroll
            for (int d = 0; d < BD; ++d)
#pragma unroll
                for (int b = 0; b < KD; ++b) xa[d][b] = xb[d][b];
        }
    }
    E *ys = y + (r * BI * p.ncols + c) * KI;
#pragma unroll
    for (int i = 0; i < BI; ++i)
#pragma unroll
        for (int a = 0; a < KI; ++a) {
            E o = Ops<E>::scale(acc[i][a], p.alpha_re, p.alpha_im);
            if (p.add) o = Ops<E>::add(o, ys[i * p.ncols * KI + a]);
            ys[i * p.ncols * KI + a] = o;
        }
}

/// Any block / Kronecker sizes: one thread per output element (block row, i, column, a)
template <typename E>
__global__ void __launch_bounds__(256) bsr_kron_generic_kernel(const KronArgs p) {
    const E *__restrict__ v = (const E *)p.v;
    const E *__restrict__ kron = (const E *)p.kron;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    const long total = p.block_rows * p.bi * p.ncols * p.ki;
    for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256L) {
        const int a = (int)(idx % p.ki);
        long t = idx / p.ki;
        const long c = t % p.ncols;
        t /= p.ncols;
        const int i = (int)(t % p.bi);
        const long r = t / p.bi;
        E acc = Ops<E>::zero();
        for (int mu = 0; mu < p.nnz; ++mu) {
            const long j = r * p.nnz + mu;
            const E *xs = x + (long)p.jj[j] * p.bd * p.ncols * p.kd + c * p.kd;
            const E *K = kron + (long)mu * p.ki * p.kd;
            const E *U = v + j * p.bi * p.bd;
            for (int b = 0; b < p.kd; ++b) {
                const E k = p.block_im_fast ? K[a + b * p.ki] : K[a * p.kd + b];
                if (!Ops<E>::nonzero(k)) continue;
                E s = Ops<E>::zero();
                for (int d = 0; d < p.bd; ++d) {
                    const E u = p.block_im_fast ? U[i + d * p.bi] : U[i * p.bd + d];
                    s = Ops<E>::fma(u, xs[d * p.ncols * p.kd + b], s);
                }
                acc = Ops<E>::fma(k, s, acc);
            }
        }
        E o = Ops<E>::scale(acc, p.alpha_re, p.alpha_im);
        if (p.add) o = Ops<E>::add(o, y[idx]);
        y[idx] = o;
    }
}

// complex<double>, 3x3 color blocks, 4x4 spin matrices, from 8 rhs columns: one wave per (block
// row, group of 16 rhs columns), lane l = 16 b + q owning spin b of column q of the group.
//  * color on the VALU: T_mu(i, b, q) = sum_d U_mu(i, d) x(J_mu, d, q, b) -- the row's color
//    blocks and block columns are wave-uniform (scalar loads, SGPR operands), the x loads of a
//    neighbour are lane-linear 16-byte pieces (1 KB per wave instruction at 16 columns);
//  * spin on the matrix cores: acc(a, i, q) += sum_b K_mu(a, b) T_mu(i, b, q) is a 4x4x4 product
//    per group of 4 columns, i.e. v_mfma_f64_4x4x4_4b_f64 with A = K_mu (lane 16 b + 4 g + a, the
//    same in all 4 blocks), B = T (lane 16 b + q) and C = acc (lane 16 a + q) -- the lane maps
//    measured by tools/mfma_small.hip -- 4 real products per complex one (the BLAS rounding);
//  * the next neighbour's x is loaded while the current one is applied; 4 rows per workgroup,
//    an XCD's rows visited as two interleaved halves (its ilv form of the 3x3 kernels).
// The previous kernel (one thread per (row, column) owning all 12 outputs) ran at 256 VGPRs:
// 2 waves per SIMD.
// XL > 0: x staged by LDS-DMA in whole 64-B spin pieces, XL neighbours ahead (see
// bsr_kron_mfma_packed_kernel)
template <int NNZ, bool kpf = false, int XL = 0>
__global__ void __launch_bounds__(256) bsr_kron_mfma_kernel(const KronArgs p, int ngroups) {
    typedef double2 E;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-contiguous chunks of 4 block rows, the XCD's range visited as two interleaved halves
    const long nchunk = (p.block_rows + 3) / 4;
    const int bid = blockIdx.x, nwg = gridDim.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int cnt = xcd < r8 ? q8 + 1 : q8, qx = bid >> 3, npart = cnt / 2;
    const int loc = (npart > 0 && qx < npart * 2) ? (qx % 2) * npart + qx / 2 : qx;
    const long wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const long task = wgi * 4 + w; // (row chunk, column group) tasks: row-major over groups
    const long r = task / ngroups;
    const int cg = (int)(task - r * ngroups);
    // the color blocks of the workgroup's rows (rows of a task group are consecutive: one
    // contiguous run) into LDS by one DMA pass, read back as broadcasts
    // (rounded up to whole DMA passes of 256 lanes: the lanes past the run write zeros)
    __shared__ __attribute__((aligned(16))) E us[(4 * NNZ * 9 + 255) / 256 * 256];
    // a workgroup's 4 tasks span at most 4 rows: nu <= 4 * NNZ * 9, every pass of 256 lanes fits
    static_assert(sizeof(us) / sizeof(E) >= (4 * NNZ * 9 + 255) / 256 * 256, "LDS sizing");
    // XL: the spin matrices in LDS -- no vector-memory load in the main loop, where the
    // compiler's own vmcnt waits (blind to the DMAs) would drain the x ring
    __shared__ __attribute__((aligned(16))) E ks[XL ? NNZ * 16 : 1];
    if constexpr (XL > 0)
        for (int e = (int)threadIdx.x; e < NNZ * 16; e += 256) ks[e] = ((const E *)p.kron)[e];
    {
        const long rlo = (wgi * 4) / ngroups, rhi = min((wgi * 4 + 3) / ngroups, p.block_rows - 1);
        const int nu = (int)(rhi - rlo + 1) * NNZ * 9;
        // (launcher: the value array is below 2 GiB)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)p.v, (short)0, (int)(p.block_rows * NNZ * 9 * 16), 0x00020000);
        const unsigned base = (unsigned)(size_t)(const __attribute__((address_space(3))) void *)us +
                              (unsigned)w * 1024u;
        for (int u = 0; u * 256 < nu; ++u) {
            const int e = u * 256 + (int)threadIdx.x;
            const unsigned off = e < nu ? (unsigned)(rlo * NNZ * 9 + e) * 16u : 0x80000000u;
            asm volatile("s_mov_b32 m0, %1\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %0, %2, 0 offen lds"
                         :
                         : "v"(off), "s"(__builtin_amdgcn_readfirstlane(base + (unsigned)(u * 256) * 16u)),
                           "s"(rs)
                         : "memory", "m0");
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        (void)nchunk;
    }
    if (r >= p.block_rows) return;
    const E *urow_s = us + (r - (wgi * 4) / ngroups) * NNZ * 9;
    const int b = lane >> 4, q = lane & 15;
    const long n = p.ncols;
    const long col = (long)cg * 16 + q;
    const bool ok = col < n;
    const long colc = ok ? col : n - 1;
    // spin matrices as the A operand: lane 16 k + 4 g + a holds K_mu(a, k)
    const int ka = lane & 3, kk = lane >> 4;
    const E *kron = (const E *)p.kron;
    const int kidx = p.block_im_fast ? ka + kk * 4 : ka * 4 + kk;
    // block columns and color blocks of the row: wave-uniform
    const ConstPtr<int> jrow = (ConstPtr<int>)(p.jj + r * NNZ);
    const long xsite = 3 * n * 4; // elements per domain site: (d, n, b)
    auto load_x = [&](int J, E *xv) {
        const E *xs = x + (long)J * xsite + colc * 4 + b;
#pragma unroll
        for (int d = 0; d < 3; ++d) xv[d] = xs[d * n * 4];
    };
    double accR[3] = {0, 0, 0}, accI[3] = {0, 0, 0};
    E xa[3], xb[3];
    // XL: a ring of XL + 1 neighbours x 3 KB per wave; the DMA lane's piece: column lane / 4 of
    // the group, its spins rotated as xpos below
    constexpr int NS = XL + 1;
    __shared__ __attribute__((aligned(16))) E xr[XL ? 4 * NS * 3 * 64 : 1];
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, 0x7fffffff, 0x00020000);
    const int qd = lane >> 2, bd = ((lane & 3) - (qd >> 1) - (qd >> 3)) & 3;
    const long cold = min((long)cg * 16 + qd, n - 1);
    const unsigned xoff_d = (unsigned)(cold * 4 + bd) * 16u;
    const unsigned ring = (unsigned)(size_t)(const __attribute__((address_space(3))) void *)xr + (unsigned)w * (NS * 3072u);
    auto issue_x = [&](int mu) {
        const unsigned base = ring + (unsigned)(mu % NS) * 3072u;
        const unsigned o = (unsigned)((long)jrow[mu] * xsite) * 16u + xoff_d;
#pragma unroll
        for (int d = 0; d < 3; ++d)
            asm volatile("s_mov_b32 m0, %1\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %0, %2, 0 offen lds"
                         :
                         : "v"(o + (unsigned)(d * n * 4) * 16u),
                           "s"(__builtin_amdgcn_readfirstlane(base + (unsigned)d * 1024u)), "s"(rx)
                         : "memory", "m0");
    };
    const int xpos = 4 * q + ((b + (q >> 1) + (q >> 3)) & 3);
    if constexpr (XL > 0) {
#pragma unroll
        for (int mu = 0; mu < XL && mu < NNZ; ++mu) issue_x(mu);
    } else {
        load_x(jrow[0], xa);
    }
    // the spin matrix of neighbour mu + 1 is loaded with its x rows; the compiler barrier keeps
    // the unrolled loop from hoisting all 9 spin-matrix loads to the top (36 more VGPRs: fewer
    // waves per SIMD)
    E Kc = XL > 0 ? E{} : kron[kidx];
#pragma unroll
    for (int mu = 0; mu < NNZ; ++mu) {
        if constexpr (kpf) asm volatile("" ::: "memory");
        E Kn = Kc;
        if constexpr (XL > 0) {
            // the ring slot of neighbour mu + XL was read in iteration mu - 1: those reads are done
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (mu + XL < NNZ) issue_x(mu + XL);
            // neighbour mu landed: its successors' DMAs (and the next spin load) may stay in flight
            wait_vmcnt(3 * (NNZ - 1 - mu < XL ? NNZ - 1 - mu : XL));
            const E *xs = xr + w * (NS * 192) + (mu % NS) * 192;
#pragma unroll
            for (int d = 0; d < 3; ++d) xa[d] = xs[d * 64 + xpos];
        } else if (mu + 1 < NNZ) {
            load_x(jrow[mu + 1], xb);
            if constexpr (kpf) Kn = kron[(mu + 1) * 16 + kidx];
        }
        const E K = XL > 0 ? ks[mu * 16 + kidx] : kpf ? Kc : kron[mu * 16 + kidx];
        Kc = Kn;
        // color: T(i) = sum_d U(i, d) x(d)
        E t[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            t[i] = Ops<E>::zero();
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const long ui = mu * 9 + (p.block_im_fast ? i + d * 3 : i * 3 + d);
                t[i] = Ops<E>::fma(urow_s[ui], xa[d], t[i]);
            }
        }
        // spin: acc(a) += K(a, b) T(b) on the matrix cores, 4 real products per complex one
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            accR[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(K.x, t[i].x, accR[i], 0, 0, 0);
            accR[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(-K.y, t[i].y, accR[i], 0, 0, 0);
            accI[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(K.x, t[i].y, accI[i], 0, 0, 0);
            accI[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(K.y, t[i].x, accI[i], 0, 0, 0);
        }
        if (XL == 0 && mu + 1 < NNZ) {
#pragma unroll
            for (int d = 0; d < 3; ++d) xa[d] = xb[d];
        }
    }
    if constexpr (XL > 0) {
        if (p.ylds) {
            // C lane 16 a + q -> ring position xpos (a in place of b); lane l stores column l / 4
            E *ys = xr + w * (NS * 192);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                ys[i * 64 + xpos] = Ops<E>::scale(E{accR[i], accI[i]}, p.alpha_re, p.alpha_im);
            asm volatile("" ::: "memory");
            const long cs = (long)cg * 16 + qd;
            if (cs >= n) return;
            const int ad = bd;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                E *yp = y + ((r * 3 + i) * n + cs) * 4 + ad;
                E o = ys[i * 64 + lane];
                if (p.add) o = Ops<E>::add(o, *yp);
                *yp = o;
            }
            return;
        }
    }
    if (!ok) return;
    // C lane 16 a + q: spin a of column q
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        E *yp = y + ((r * 3 + i) * n + col) * 4 + b;
        E o = Ops<E>::scale(E{accR[i], accI[i]}, p.alpha_re, p.alpha_im);
        if (p.add) o = Ops<E>::add(o, *yp);
        *yp = o;
    }
}

// The same kernel for rhs counts below 16 that divide 16 W (W <= 4 waves): a wave's 16 column
// slots are (row, column) pairs of the workgroup's RW = 16 W / n consecutive block rows, so no lane
// idles (at n = 12 one wave per row left 4 of 16 slots empty: 25 % of the VALU and MFMA work).
// The row's block columns and color blocks become per-lane (LDS reads of the staged color blocks,
// block columns loaded per lane); the spin matrices stay the MFMA's A operand.
// XL: the neighbours' x pieces staged by LDS-DMA instead of VGPR loads.  The MFMA's B operand
// wants lane 16 b + q = spin b of slot q, but spin is the fastest index of x in memory, so a
// 16-lane quarter of such a load touches 16 pieces 64 B apart (8 cache lines; 32 TA/TCP accesses
// per 1-KB instruction against 8 for a linear one, and TA/TD busy 85-92 %).  The DMA instead
// moves each slot's 4 spins as one 64-B piece (lane l: slot l / 4), writes them lane-linear into
// the wave's ring (XL neighbours ahead, 3 KB per neighbour: deeper prefetch costs LDS, not
// VGPRs), and the B lanes read them back with the spins rotated (position 4 q + (b + q / 2 +
// q / 8) mod 4: the 16-B granules of any 8 or 16 lanes reading together fall on distinct banks).
template <int NNZ, bool kpf = false, int XL = 0>
__global__ void __launch_bounds__(256) bsr_kron_mfma_packed_kernel(const KronArgs p, int rw, int xring) {
    constexpr int NS = XL + 1;
    typedef double2 E;
    const E *__restrict__ x = (const E *)p.x;
    E *__restrict__ y = (E *)p.y;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = blockIdx.x, nwg = gridDim.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int cnt = xcd < r8 ? q8 + 1 : q8, qx = bid >> 3, npart = cnt / 2;
    const int loc = (npart > 0 && qx < npart * 2) ? (qx % 2) * npart + qx / 2 : qx;
    const long wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    const long r0 = wgi * rw;
    const int nrows = (int)min((long)rw, p.block_rows - r0);
    const long n = p.ncols;
    const int b = lane >> 4, q = lane & 15;
    const int slot = w * 16 + q, rl = slot / (int)n;
    const long col = slot - (long)rl * n;
    const bool live = rl < nrows;
    const int rlc = live ? rl : nrows - 1;
    const long r = r0 + rlc;
    // the color blocks of the workgroup's rows (one contiguous run) into LDS by one DMA pass
    // (dynamic LDS: rw rows of NNZ 3x3 blocks)
    extern __shared__ __attribute__((aligned(16))) char smem_k[];
    E *us = (E *)smem_k;
    {
        const int nu = nrows * NNZ * 9;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void *)p.v, (short)0, (int)(p.block_rows * NNZ * 9 * 16), 0x00020000);
        const unsigned base = (unsigned)(size_t)(const __attribute__((address_space(3))) void *)smem_k +
                              (unsigned)w * 1024u;
        const int nth = (int)blockDim.x;
        for (int u = 0; u * nth < nu; ++u) {
            const int e = u * nth + (int)threadIdx.x;
            const unsigned off = e < nu ? (unsigned)(r0 * NNZ * 9 + e) * 16u : 0x80000000u;
            asm volatile("s_mov_b32 m0, %1\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %0, %2, 0 offen lds"
                         :
                         : "v"(off), "s"(__builtin_amdgcn_readfirstlane(base + (unsigned)(u * nth) * 16u)),
                           "s"(rs)
                         : "memory", "m0");
        }
    }
    // the lane's row: block columns (per lane), then the first neighbour's x
    int jrow[NNZ];
#pragma unroll
    for (int mu = 0; mu < NNZ; ++mu) jrow[mu] = p.jj[r * NNZ + mu];
    const int ka = lane & 3, kk = lane >> 4;
    const E *kron = (const E *)p.kron;
    const int kidx = p.block_im_fast ? ka + kk * 4 : ka * 4 + kk;
    const long xsite = 3 * n * 4;
    auto load_x = [&](int J, E *xv) {
        const E *xs = x + (long)J * xsite + col * 4 + b;
#pragma unroll
        for (int d = 0; d < 3; ++d) xv[d] = xs[d * n * 4];
    };
    E xa[3], xb[3];
    // XL: the DMA lane's piece (slot lane / 4, spin rotated back) and its slot's block columns
    int jd[XL > 0 ? NNZ : 1];
    unsigned xoff_d = 0, xring_w = 0;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc((void *)x, (short)0, 0x7fffffff, 0x00020000);
    if constexpr (XL > 0) {
        const int qd = lane >> 2, bd = ((lane & 3) - (qd >> 1) - (qd >> 3)) & 3;
        const int sd = w * 16 + qd, rld = sd / (int)n;
        const long cold = sd - (long)rld * n;
        const long rd = r0 + (rld < nrows ? rld : nrows - 1);
#pragma unroll
        for (int mu = 0; mu < NNZ; ++mu) jd[mu] = p.jj[rd * NNZ + mu];
        xoff_d = (unsigned)(cold * 4 + bd) * 16u;
        xring_w = (unsigned)xring + (unsigned)w * (NS * 3072u);
    }
    const unsigned lds0 = (unsigned)(size_t)(const __attribute__((address_space(3))) void *)smem_k;
    // XL: the spin matrices in LDS after the rings -- no vector-memory load in the main loop,
    // where the compiler's own vmcnt waits (blind to the DMAs) would drain the x ring
    E *ks = (E *)(smem_k + xring + (int)(blockDim.x >> 6) * NS * 3072);
    if constexpr (XL > 0) {
        for (int e = (int)threadIdx.x; e < NNZ * 16; e += (int)blockDim.x) ks[e] = kron[e];
        // the DMA lanes' block columns: consumed here, so that no load of them is pending
        // (and waited for by the compiler) inside the loop
#pragma unroll
        for (int mu = 0; mu < NNZ; ++mu) asm volatile("" : "+v"(jd[mu]));
    }
    auto issue_x = [&](int mu) {
        const unsigned base = lds0 + xring_w + (unsigned)(mu % NS) * 3072u;
        const unsigned o = (unsigned)((long)jd[mu] * xsite) * 16u + xoff_d;
#pragma unroll
        for (int d = 0; d < 3; ++d)
            asm volatile("s_mov_b32 m0, %1\n\t"
                         "s_nop 0\n\t"
                         "buffer_load_dwordx4 %0, %2, 0 offen lds"
                         :
                         : "v"(o + (unsigned)(d * n * 4) * 16u),
                           "s"(__builtin_amdgcn_readfirstlane(base + (unsigned)d * 1024u)), "s"(rx)
                         : "memory", "m0");
    };
    // the B lane's position in a ring slot
    const int xpos = 4 * q + ((b + (q >> 1) + (q >> 3)) & 3);
    if constexpr (XL > 0) {
#pragma unroll
        for (int mu = 0; mu < XL && mu < NNZ; ++mu) issue_x(mu);
    } else {
        load_x(jrow[0], xa);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const E *urow_s = us + rlc * NNZ * 9;
    double accR[3] = {0, 0, 0}, accI[3] = {0, 0, 0};
    // the spin matrix of neighbour mu + 1 is loaded with its x rows; the compiler barrier keeps
    // the unrolled loop from hoisting all 9 spin-matrix loads to the top (36 more VGPRs: fewer
    // waves per SIMD)
    E Kc = XL > 0 ? E{} : kron[kidx];
#pragma unroll
    for (int mu = 0; mu < NNZ; ++mu) {
        if constexpr (kpf) asm volatile("" ::: "memory");
        E Kn = Kc;
        if constexpr (XL > 0) {
            // the ring slot of neighbour mu + XL was read in iteration mu - 1: those reads are done
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (mu + XL < NNZ) issue_x(mu + XL);
            // neighbour mu landed: its successors' DMAs (and the next spin load) may stay in flight
            wait_vmcnt(3 * (NNZ - 1 - mu < XL ? NNZ - 1 - mu : XL));
            const E *xs = (const E *)(smem_k + xring_w + (mu % NS) * 3072);
#pragma unroll
            for (int d = 0; d < 3; ++d) xa[d] = xs[d * 64 + xpos];
        } else if (mu + 1 < NNZ) {
            load_x(jrow[mu + 1], xb);
            if constexpr (kpf) Kn = kron[(mu + 1) * 16 + kidx];
        }
        const E K = XL > 0 ? ks[mu * 16 + kidx] : kpf ? Kc : kron[mu * 16 + kidx];
        Kc = Kn;
        E t[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            t[i] = Ops<E>::zero();
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                const long ui = mu * 9 + (p.block_im_fast ? i + d * 3 : i * 3 + d);
                t[i] = Ops<E>::fma(urow_s[ui], xa[d], t[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            accR[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(K.x, t[i].x, accR[i], 0, 0, 0);
            accR[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(-K.y, t[i].y, accR[i], 0, 0, 0);
            accI[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(K.x, t[i].y, accI[i], 0, 0, 0);
            accI[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(K.y, t[i].x, accI[i], 0, 0, 0);
        }
        if (XL == 0 && mu + 1 < NNZ) {
#pragma unroll
            for (int d = 0; d < 3; ++d) xa[d] = xb[d];
        }
    }
    if constexpr (XL > 0) {
        if (p.ylds) {
            // C lane 16 a + q -> ring position xpos (the B read's map, a in place of b); then
            // lane l stores the piece of slot l / 4: each slot's 4 spins one 64-B run
            E *ys = (E *)(smem_k + xring_w);
#pragma unroll
            for (int i = 0; i < 3; ++i)
                ys[i * 64 + xpos] = Ops<E>::scale(E{accR[i], accI[i]}, p.alpha_re, p.alpha_im);
            asm volatile("" ::: "memory");
            const int qd = lane >> 2, ad = ((lane & 3) - (qd >> 1) - (qd >> 3)) & 3;
            const int sd = w * 16 + qd, rld = sd / (int)n;
            if (rld >= nrows) return;
            const long cold = sd - (long)rld * n;
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                E *yp = y + (((r0 + rld) * 3 + i) * n + cold) * 4 + ad;
                E o = ys[i * 64 + lane];
                if (p.add) o = Ops<E>::add(o, *yp);
                *yp = o;
            }
            return;
        }
    }
    if (!live) return;
    // C lane 16 a + q: spin a of slot q
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        E *yp = y + ((r * 3 + i) * n + col) * 4 + b;
        E o = Ops<E>::scale(E{accR[i], accI[i]}, p.alpha_re, p.alpha_im);
        if (p.add) o = Ops<E>::add(o, *yp);
        *yp = o;
    }
}


// complex<double>, 3x3 color blocks, 4x4 spin matrices with at most two nonzeros per row (the
// Wilson projectors 1 -+ gamma_mu, the identity, gamma matrices), from 8 rhs columns, spin first
// -- the reference's order (contract_kron_cols applies K_mu to x, then bsrmm the color blocks,
// bsr.h:933-998).  A lane owns one (block row, rhs column) pair and its 12 outputs, so no lane
// idles at any column count (pair p = row slot p / n, column p % n); per step (mu, d):
//   h(a) = c0 x(J_mu, d, col, b0) + c1 x(J_mu, d, col, b1)   (row a of K_mu as two terms: the
//                                                           host's table, build_kron_terms)
//   acc(i, a) += U_mu(i, d) h(a)
// i.e. 32 + 48 FMAs a step, no branches; the MFMA form spends 48 FMA-equivalents of 4x4x4 MFMA
// on the spin product of a dense K_mu and leaves a quarter of its lanes idle at 12 columns.
// Per wave and step one LDS-DMA group, one step ahead: x of the 64 pairs (4 KB: 16 pairs' 4
// spins a 1-KB piece, lane-linear over the pairs' 64-B spin runs, spin b of pair q at position
// b ^ (q / 4 % 4): a read of one spin by 16 lanes hits distinct banks in each of
// ds_read_b128's lane groups), U_mu(., d) of the wave's rows (<= 9 rows of 3 values, lanes <
// 32), and at d = 0 the wave rows' block columns of the next neighbour (one dword per row).
// Rows optionally visited in the host's XCD order (perm: each XCD's share of the row slots one
// compact lattice box).
constexpr int KS_WAVE_LDS = 2 * 4096 + 2 * 512 + 2 * 256;

/// DMA of 16 (or 4: dword) bytes per lane into LDS at m0 = base (+ 16 or 4 per lane)
__device__ __forceinline__ void dma16(unsigned off, unsigned base, __amdgpu_buffer_rsrc_t r) {
    asm volatile("s_mov_b32 m0, %1\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dwordx4 %0, %2, 0 offen lds"
                 :
                 : "v"(off), "s"(__builtin_amdgcn_readfirstlane(base)), "s"(r)
                 : "memory", "m0");
}
__device__ __forceinline__ void dma4(unsigned off, unsigned base, __amdgpu_buffer_rsrc_t r) {
    asm volatile("s_mov_b32 m0, %1\n\t"
                 "s_nop 0\n\t"
                 "buffer_load_dword %0, %2, 0 offen lds"
                 :
                 : "v"(off), "s"(__builtin_amdgcn_readfirstlane(base)), "s"(r)
                 : "memory", "m0");
}

__global__ void __launch_bounds__(256) bsr_kron_spin_kernel(const KronArgs p) {
    typedef double2 E;
    extern __shared__ __attribute__((aligned(16))) char smem_s[];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // XCD-contiguous workgroup order: the hardware deals workgroups round robin over the 8 XCDs
    const int bid = blockIdx.x, nwg = gridDim.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    // (launcher: pairs, x, values and block columns below 2^31 elements / bytes)
    const int n = (int)p.ncols, nnz = p.nnz;
    const int total = (int)(p.block_rows * n);
    const int pw0 = (wgi * 4 + w) * 64; // the wave's first pair
    if (pw0 >= total) return;
    const int slot_lo = pw0 / n;
    const int rows_w = min(pw0 + 63, total - 1) / n - slot_lo + 1; // <= 9 (n >= 8)
    const int *perm = p.perm;
    auto row_of = [&](int slot) -> int { return perm ? perm[slot] : slot; };
    // the lane's pair
    const int pp = min(pw0 + lane, total - 1);
    const bool live = pw0 + lane < total;
    const int slot = pp / n, col = pp - slot * n;
    const int wr = slot - slot_lo;
    // LDS per wave: x slots [2][4096], U slots [2][512], J slots [2][256]
    char *wl = smem_s + w * KS_WAVE_LDS;
    const unsigned wl_a = (unsigned)(size_t)(const __attribute__((address_space(3))) void *)wl;
    const E *xs = (const E *)wl;
    const E *us = (const E *)(wl + 8192);
    const int *js = (const int *)(wl + 9216);
    // x DMA: instruction k, lane l -> pair q = 16 k + l / 4, spin (l % 4) ^ (q / 4 % 4); its
    // (column * 4 + spin) in elements (-1: past the last pair) and wave row
    const int xd = 4 * n; // elements between the colors of a site
    int xcolb[4], xwr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int q = 16 * k + (lane >> 2);
        const int pq = pw0 + q, pc = min(pq, total - 1);
        const int b = (lane & 3) ^ ((q >> 2) & 3);
        const int sq = pc / n;
        xwr[k] = sq - slot_lo;
        xcolb[k] = pq < total ? (pc - sq * n) * 4 + b : -1;
    }
    // U DMA: lane l < 3 rows_w -> value i = l % 3 of wave row l / 3; J DMA: lane l < rows_w -> row l
    const bool u_ok = lane < 3 * rows_w;
    const int ui = lane % 3;
    const int ubase = (u_ok ? row_of(slot_lo + lane / 3) : 0) * nnz * 9 + (p.block_im_fast ? ui : 3 * ui);
    const int ustep = p.block_im_fast ? 3 : 1;
    const bool j_ok = lane < rows_w;
    const int jbase = (j_ok ? row_of(slot_lo + lane) : 0) * nnz;
    const int orow = row_of(slot); // the output row
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        (void *)p.x, (short)0, (int)(p.x_rows * 4 * n * 16), 0x00020000);
    const __amdgpu_buffer_rsrc_t ru = __builtin_amdgcn_make_buffer_rsrc(
        (void *)p.v, (short)0, (int)(p.block_rows * nnz * 9 * 16), 0x00020000);
    const __amdgpu_buffer_rsrc_t rj = __builtin_amdgcn_make_buffer_rsrc(
        (void *)p.jj, (short)0, (int)(p.block_rows * nnz * 4), 0x00020000);
    // block columns of the x pieces for the current neighbour: mu = 0 from global memory, then
    // from the J slots
    int jx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) jx[k] = p.jj[row_of(slot_lo + xwr[k]) * nnz];
    // (offsets past the buffers for the pieces without data: the DMA writes zeros; selects, not
    // branches)
    unsigned xbad = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) xbad |= (xcolb[k] < 0 ? 1u : 0u) << k;
    const unsigned ubad = u_ok ? 0u : 0x80000000u, jbad = j_ok ? 0u : 0x80000000u;
    auto issue = [&](int mu, int d, int par) {
        const unsigned xb = wl_a + (unsigned)par * 4096u;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const unsigned off = (unsigned)((jx[k] * 3 + d) * xd + xcolb[k]) * 16u;
            dma16((xbad >> k & 1) ? 0x80000000u : off, xb + (unsigned)k * 1024u, rx);
        }
        if (lane < 32) dma16((unsigned)(ubase + mu * 9 + d * ustep) * 16u | ubad, wl_a + 8192u + (unsigned)par * 512u, ru);
        if (d == 0 && mu + 1 < nnz)
            dma4((unsigned)(jbase + mu + 1) * 4u | jbad, wl_a + 9216u + (unsigned)((mu + 1) & 1) * 256u, rj);
    };
    double ar[3][4], ai[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int a = 0; a < 4; ++a) ar[i][a] = 0, ai[i][a] = 0;
    // spin b of the lane's pair sits at piece 4 lane + (b ^ (lane / 4 % 4)) of an x slot: byte
    // address xa0 ^ 16 b
    const unsigned xa0 = (unsigned)(64 * lane + 16 * ((lane >> 2) & 3));
    const double *ctab = (const double *)p.ktab;          // [nnz][4 rows][2 terms] complex
    const int *btab = (const int *)(ctab + 16L * nnz);    // [nnz][4 rows][2 terms] spin index
    issue(0, 0, 0);
#pragma unroll 1
    for (int mu = 0; mu < nnz; ++mu) {
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const int t = mu * 3 + d, par = t & 1;
            const bool more = t + 1 < 3 * nnz;
            // the slot about to be refilled was read in step t - 1
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if (more) {
                if (d == 2) {
                    // the next neighbour's block columns (landed with step t - 2's group)
#pragma unroll
                    for (int k = 0; k < 4; ++k) jx[k] = js[((mu + 1) & 1) * 64 + xwr[k]];
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    issue(mu + 1, 0, par ^ 1);
                } else {
                    issue(mu, d + 1, par ^ 1);
                }
            }
            // step t's group landed; step t + 1's (5 instructions, 6 with a J piece) may stay in flight
            if (!more) wait_vmcnt(0);
            else if (d == 2 && mu + 2 < nnz) wait_vmcnt(6); // (mu + 1, 0) carries the J piece
            else wait_vmcnt(5);
            const char *xp = (const char *)(xs + par * 256);
            const E *up = us + par * 32 + wr * 3;
            E uv[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) uv[i] = up[i];
#pragma unroll
            for (int a = 0; a < 4; ++a) {
                // (the compiler barrier keeps the scalar loads of the 12 rows of a neighbour from
                // being hoisted together: 96 SGPRs, spilled)
                asm volatile("" ::: "memory");
                // h(a) = c0 x(b0) + c1 x(b1): the row's (at most) two nonzero spin entries
                const int b0 = Uniform<int>::load(btab, mu * 8 + 2 * a);
                const int b1 = Uniform<int>::load(btab, mu * 8 + 2 * a + 1);
                const E x0 = *(const E *)(xp + (xa0 ^ (unsigned)(16 * b0)));
                const E x1 = *(const E *)(xp + (xa0 ^ (unsigned)(16 * b1)));
                const double c0r = Uniform<double>::load(ctab, mu * 16 + 4 * a);
                const double c0i = Uniform<double>::load(ctab, mu * 16 + 4 * a + 1);
                const double c1r = Uniform<double>::load(ctab, mu * 16 + 4 * a + 2);
                const double c1i = Uniform<double>::load(ctab, mu * 16 + 4 * a + 3);
                double hr = c0r * x0.x, hi = c0r * x0.y;
                hr = __builtin_fma(-c0i, x0.y, hr);
                hi = __builtin_fma(c0i, x0.x, hi);
                hr = __builtin_fma(c1r, x1.x, hr);
                hi = __builtin_fma(c1r, x1.y, hi);
                hr = __builtin_fma(-c1i, x1.y, hr);
                hi = __builtin_fma(c1i, x1.x, hi);
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    ar[i][a] = __builtin_fma(uv[i].x, hr, ar[i][a]);
                    ar[i][a] = __builtin_fma(-uv[i].y, hi, ar[i][a]);
                    ai[i][a] = __builtin_fma(uv[i].x, hi, ai[i][a]);
                    ai[i][a] = __builtin_fma(uv[i].y, hr, ai[i][a]);
                }
            }
            // the step's products finish before the next step's waits and DMAs (otherwise the
            // compiler overlaps the steps and holds two steps' x values: 167 VGPRs)
#pragma unroll
            for (int i = 0; i < 3; ++i)
                asm volatile("" : "+v"(ar[i][0]), "+v"(ar[i][1]), "+v"(ar[i][2]), "+v"(ar[i][3]),
                             "+v"(ai[i][0]), "+v"(ai[i][1]), "+v"(ai[i][2]), "+v"(ai[i][3]));
        }
    }
    if (!live) return;
    E *yp = (E *)p.y + ((long)orow * 3 * n + col) * 4;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            E o = Ops<E>::scale(E{ar[i][a], ai[i][a]}, p.alpha_re, p.alpha_im);
            if (p.add) o = Ops<E>::add(o, yp[(long)i * n * 4 + a]);
            yp[(long)i * n * 4 + a] = o;
        }
}


// The same spin-first product with the spin rows in "diagonal + XOR partner" form (every row a of
// K_mu nonzero at most at spins a and a ^ s_mu: the Wilson projectors 1 -+ gamma_mu and the gamma
// matrices in the chiral, Dirac-Pauli and DeGrand-Rossi bases), so that a lane keeps its pair's
// 4 spins in registers and the partner is a compile-time register (one instantiation of the
// step per s, chosen per neighbour by a scalar switch):
//   h(a) = c0(a) x(a) + c1(a) x(a ^ s)                  (the host's table, build_kron_terms)
//   acc(i, a) += U_mu(i, d) h(a)
// and everything comes by plain vector loads one step ahead (a pair's x: 64 contiguous bytes per
// lane and color; U_mu(., d) of its row; J_mu one neighbour ahead) -- no LDS and no LDS-DMA,
// whose issue cost (about 60 cycles a piece, MI355X_MICROARCH.md) set the first form's time.
/// h(a) = c0(a) x(a) + c1(a) x(a ^ S), the coefficients from the table by scalar loads
template <int S>
__device__ __forceinline__ void kron_xor_h(const double2 (&x)[4], const double *c, double (&hr)[4], double (&hi)[4]) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const double c0r = Uniform<double>::load(c, 4 * a), c0i = Uniform<double>::load(c, 4 * a + 1);
        const double2 x0 = x[a], x1 = x[a ^ S];
        hr[a] = c0r * x0.x;
        hi[a] = c0r * x0.y;
        hr[a] = __builtin_fma(-c0i, x0.y, hr[a]);
        hi[a] = __builtin_fma(c0i, x0.x, hi[a]);
        if (S != 0) {
            const double c1r = Uniform<double>::load(c, 4 * a + 2), c1i = Uniform<double>::load(c, 4 * a + 3);
            hr[a] = __builtin_fma(c1r, x1.x, hr[a]);
            hi[a] = __builtin_fma(c1r, x1.y, hi[a]);
            hr[a] = __builtin_fma(-c1i, x1.y, hr[a]);
            hi[a] = __builtin_fma(c1i, x1.x, hi[a]);
        }
    }
}

__global__ void __launch_bounds__(256) bsr_kron_xor_kernel(const KronArgs p) {
    typedef double2 E;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int bid = blockIdx.x, nwg = gridDim.x;
    const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
    const int wgi = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    // (launcher: pairs, x and values below 2^31 elements)
    const int n = (int)p.ncols, nnz = p.nnz;
    const int total = (int)(p.block_rows * n);
    const int pw0 = (wgi * 4 + w) * 64;
    if (pw0 >= total) return;
    const int pp = min(pw0 + lane, total - 1);
    const bool live = pw0 + lane < total;
    const int slot = pp / n, col = pp - slot * n;
    const int row = p.perm ? p.perm[slot] : slot;
    const E *x = (const E *)p.x, *v = (const E *)p.v;
    const int *jrow = p.jj + (long)row * nnz;
    const E *urow = v + (long)row * nnz * 9;
    const int xd = 4 * n; // elements between the colors of a site
    const int ust = p.block_im_fast ? 3 : 1, uis = p.block_im_fast ? 1 : 3;
    // the table: [nnz] { c[4 rows][c0 re, c0 im, c1 re, c1 im] } then [nnz] s
    const double *ctab = (const double *)p.ktab;
    const int *stab = (const int *)(ctab + 16L * nnz);
    double ar[3][4], ai[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int a = 0; a < 4; ++a) ar[i][a] = 0, ai[i][a] = 0;
    E xv[4], uv[3], xn[4], un[3];
    auto load = [&](int J, int mu, int d, E (&xo)[4], E (&uo)[3]) {
        const E *xp = x + (long)(J * 3 + d) * xd + col * 4;
#pragma unroll
        for (int b = 0; b < 4; ++b) xo[b] = xp[b];
        const E *up = urow + mu * 9 + d * ust;
#pragma unroll
        for (int i = 0; i < 3; ++i) uo[i] = up[i * uis];
    };
    int J = jrow[0];
    load(J, 0, 0, xv, uv);
#pragma unroll 1
    for (int mu = 0; mu < nnz; ++mu) {
        const int Jn = mu + 1 < nnz ? jrow[mu + 1] : J;
        const int sm = Uniform<int>::load(stab, mu);
        const double *c = ctab + mu * 16;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            // the next step's operands (the last step reloads its own: harmless)
            if (d < 2) load(J, mu, d + 1, xn, un);
            else load(Jn, mu + 1 < nnz ? mu + 1 : mu, 0, xn, un);
            // spin: one instantiation per partner (only h crosses the branches)
            double hr[4], hi[4];
            switch (sm) {
            case 0: kron_xor_h<0>(xv, c, hr, hi); break;
            case 1: kron_xor_h<1>(xv, c, hr, hi); break;
            case 2: kron_xor_h<2>(xv, c, hr, hi); break;
            default: kron_xor_h<3>(xv, c, hr, hi); break;
            }
            // color
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    ar[i][a] = __builtin_fma(uv[i].x, hr[a], ar[i][a]);
                    ar[i][a] = __builtin_fma(-uv[i].y, hi[a], ar[i][a]);
                    ai[i][a] = __builtin_fma(uv[i].x, hi[a], ai[i][a]);
                    ai[i][a] = __builtin_fma(uv[i].y, hr[a], ai[i][a]);
                }
            // the step's products finish before the next step's loads are issued
#pragma unroll
            for (int i = 0; i < 3; ++i)
                asm volatile("" : "+v"(ar[i][0]), "+v"(ar[i][1]), "+v"(ar[i][2]), "+v"(ar[i][3]),
                             "+v"(ai[i][0]), "+v"(ai[i][1]), "+v"(ai[i][2]), "+v"(ai[i][3])::"memory");
#pragma unroll
            for (int b = 0; b < 4; ++b) xv[b] = xn[b];
#pragma unroll
            for (int i = 0; i < 3; ++i) uv[i] = un[i];
        }
        J = Jn;
    }
    if (!live) return;
    E *yp = (E *)p.y + ((long)row * 3 * n + col) * 4;
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            E o = Ops<E>::scale(E{ar[i][a], ai[i][a]}, p.alpha_re, p.alpha_im);
            if (p.add) o = Ops<E>::add(o, yp[(long)i * n * 4 + a]);
            yp[(long)i * n * 4 + a] = o;
        }
}

constexpr long KRON_LDS_BYTES = 64 * 1024;

template <typename E> void launch_kron_typed(const KronArgs &a, hipStream_t s) {
    KernelTimer timer("bsr", s);
    const long row_bytes = (long)a.nnz * (a.bi * a.bd * sizeof(E) + sizeof(int));
    if constexpr (std::is_same<E, double2>::value) {
        if (g_bsr_tune.kron_spin == 2 && a.xtab && a.bi == 3 && a.bd == 3 && a.ki == 4 && a.kd == 4 &&
            a.nnz >= 1 && a.ncols >= g_bsr_tune.kron_spin_min_cols && a.x_rows * 4 * a.ncols < (1L << 31) &&
            a.block_rows * a.ncols + 1024 < (1L << 31)) {
            const long waves = (a.block_rows * a.ncols + 63) / 64, blocks = (waves + 3) / 4;
            if (blocks < (1L << 31)) {
                g_bsr_tune.last = 12;
                KronArgs b = a;
                b.ktab = a.xtab;
                hipLaunchKernelGGL(bsr_kron_xor_kernel, dim3((unsigned)blocks), dim3(256), 0, s, b);
                SBX_HIP_CHECK(hipGetLastError());
                return;
            }
        }
        if (g_bsr_tune.kron_spin == 1 && a.ktab && a.bi == 3 && a.bd == 3 && a.ki == 4 && a.kd == 4 && a.nnz >= 1 &&
            a.nnz <= 64 && a.ncols >= std::max(8L, g_bsr_tune.kron_spin_min_cols) &&
            a.block_rows * a.nnz * 9 * 16 < (1L << 31) && a.x_rows * 4 * a.ncols * 16 < (1L << 31) &&
            a.block_rows * a.ncols + 1024 < (1L << 31)) {
            const long waves = (a.block_rows * a.ncols + 63) / 64, blocks = (waves + 3) / 4;
            if (blocks < (1L << 31)) {
                g_bsr_tune.last = 9;
                const size_t lds = 4 * (size_t)KS_WAVE_LDS;
                hipLaunchKernelGGL(bsr_kron_spin_kernel, dim3((unsigned)blocks), dim3(256), lds, s, a);
                SBX_HIP_CHECK(hipGetLastError());
                return;
            }
        }
        if (g_bsr_tune.kron_mfma && a.bi == 3 && a.bd == 3 && a.ki == 4 && a.kd == 4 && a.nnz == 9 &&
            a.ncols >= g_bsr_tune.kron_mfma_min_cols && a.block_rows * 81L * 16 < (1L << 31)) {
            // packed slots: W waves of 16 (row, column) slots hold RW = 16 W / n whole rows
            int wpk = 0;
            for (int wv = 4; wv >= 1 && g_bsr_tune.kron_pack; --wv)
                if (a.ncols < 16 && (16 * wv) % a.ncols == 0 && 16 * wv / a.ncols <= 32) {
                    wpk = wv;
                    break;
                }
            if (wpk > 0) {
                const int rw = (int)(16 * wpk / a.ncols);
                const long blocks = (a.block_rows + rw - 1) / rw;
                if (blocks < (1L << 31)) {
                    g_bsr_tune.last = 6;
                    // LDS: rw rows of 81 color values, rounded up to whole DMA passes of the
                    // workgroup (the lanes past the run write zeros)
                    const int nth = 64 * wpk;
                    const size_t lds_cb = (size_t)((rw * 81 + nth - 1) / nth * nth) * 16;
                    // the DMA loop: passes u < ceil(nrows * 81 / nth), nrows <= rw
                    check_dma_lds("bsr_kron_mfma_packed_kernel", lds_cb, (rw * 81L + nth - 1) / nth, nth);
                    // x by LDS-DMA: a ring of 2 x 3 KB per wave after the color blocks (lds_cb is
                    // a multiple of 16); 32-bit buffer offsets
                    const int xl = std::max(a.block_rows * 12L, a.x_rows * 4L) * a.ncols * 16 < (1L << 31)
                                       ? std::max(0, std::min(3, g_bsr_tune.kron_xlds)) : 0;
                    // (+ the 9 spin matrices)
                    const size_t lds_bytes = lds_cb + (xl > 0 ? (size_t)wpk * (xl + 1) * 3072 + 9 * 16 * 16 : 0);
                    if (xl) check_dma_lds("bsr_kron_mfma_packed_kernel x ring", lds_bytes, 0, 0, (long)lds_cb + wpk * (xl + 1) * 3072L + 9 * 16 * 16);
                    // spin matrices one neighbour ahead: n = 8 / 12 104 / 166 -> 102 / 163 us
                    // (the one-row-per-wave kernel: 214 -> 221 us at n = 16, so not there;
                    // profiles/r02c_kron_kpf.txt)
                    auto go = [&](auto kern) {
                        hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(64 * wpk), lds_bytes, s, a, rw, (int)lds_cb);
                    };
                    if (xl == 1) go(bsr_kron_mfma_packed_kernel<9, true, 1>);
                    else if (xl == 2) go(bsr_kron_mfma_packed_kernel<9, true, 2>);
                    else if (xl == 3) go(bsr_kron_mfma_packed_kernel<9, true, 3>);
                    else
                        hipLaunchKernelGGL((bsr_kron_mfma_packed_kernel<9, true>), dim3((unsigned)blocks),
                                           dim3(64 * wpk), lds_bytes, s, a, rw, (int)lds_cb);
                    SBX_HIP_CHECK(hipGetLastError());
                    return;
                }
            }
            const long ngroups = (a.ncols + 15) / 16;
            const long tasks = a.block_rows * ngroups, blocks = (tasks + 3) / 4;
            if (blocks < (1L << 31)) {
                g_bsr_tune.last = 5;
                // x by LDS-DMA (32-bit buffer offsets)
                const int xl = std::max(a.block_rows * 12L, a.x_rows * 4L) * a.ncols * 16 < (1L << 31)
                                   ? std::max(0, std::min(3, g_bsr_tune.kron_xlds)) : 0;
                auto go = [&](auto kern) {
                    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, s, a, (int)ngroups);
                };
                if (xl == 1) go(bsr_kron_mfma_kernel<9, false, 1>);
                else if (xl == 2) go(bsr_kron_mfma_kernel<9, false, 2>);
                else if (xl == 3) go(bsr_kron_mfma_kernel<9, false, 3>);
                else
                    hipLaunchKernelGGL((bsr_kron_mfma_kernel<9, false>), dim3((unsigned)blocks), dim3(256), 0,
                                       s, a, (int)ngroups);
                SBX_HIP_CHECK(hipGetLastError());
                return;
            }
        }
    }
    if (a.bi == 3 && a.bd == 3 && a.ki == 4 && a.kd == 4 && a.nnz == 9 && a.ncols >= 4 &&
        row_bytes * (256 / std::min<long>(a.ncols, 256)) <= KRON_LDS_BYTES) {
        const int cpg = (int)std::min<long>(a.ncols, 256);
        const int S = 256 / cpg;
        const dim3 grid((unsigned)((a.block_rows + S - 1) / S), (unsigned)((a.ncols + cpg - 1) / cpg));
        hipLaunchKernelGGL((bsr_kron_lds_kernel<E, 3, 3, 4, 4, 9>), grid, dim3(256),
                           (size_t)(row_bytes * S), s, a, S, cpg);
    } else if (a.bi == 3 && a.bd == 3 && a.ki == 4 && a.kd == 4) {
        const long total = a.block_rows * a.ncols;
        const long blocks = std::min((total + 255) / 256, 65536L);
        hipLaunchKernelGGL((bsr_kron_kernel<E, 3, 3, 4, 4>), dim3(blocks), dim3(256), 0, s, a);
    } else {
        const long total = a.block_rows * a.bi * a.ncols * a.ki;
        const long blocks = std::min((total + 255) / 256, 65536L);
        hipLaunchKernelGGL((bsr_kron_generic_kernel<E>), dim3(blocks), dim3(256), 0, s, a);
    }
    SBX_HIP_CHECK(hipGetLastError());
}

} // namespace

void launch_bsr_kron(const BsrDesc &d, int device) {
    if (d.block_rows == 0 || d.ncols == 0) return;
    if (d.num_nnz_per_row <= 0 || !d.kron || !d.x_row_major || !d.y_row_major)
        throw Error("kron bsr: internal error (layout or pattern)");
    set_device(device);
    g_bsr_tune.last = 0;
    hipStream_t s = get_stream(device);
    KronArgs a{};
    a.block_rows = d.block_rows;
    a.nnz = d.num_nnz_per_row;
    a.bi = d.bi;
    a.bd = d.bd;
    a.ki = d.ki;
    a.kd = d.kd;
    a.jj = d.jj;
    a.v = d.v;
    a.kron = d.kron;
    a.block_im_fast = d.block_im_fast ? 1 : 0;
    a.x = d.x;
    a.y = d.y;
    a.ncols = d.ncols;
    a.alpha_re = d.alpha.re;
    a.alpha_im = d.alpha.im;
    a.add = d.add ? 1 : 0;
    a.ylds = g_bsr_tune.kron_ylds ? 1 : 0;
    // domain sites can exceed block_rows (halo sites): the x staging's 32-bit buffer offsets are
    // bounded by x's extent, not y's
    a.x_rows = d.x_rows > 0 ? d.x_rows : d.block_rows * d.bd;
    a.perm = g_bsr_tune.kron_order ? d.kron_perm : nullptr;
    a.ktab = d.kron_terms;
    a.xtab = d.kron_xor;
    switch (d.t) {
    case SBX_CDOUBLE: return launch_kron_typed<double2>(a, s);
    case SBX_CFLOAT: return launch_kron_typed<float2>(a, s);
    case SBX_DOUBLE: return launch_kron_typed<double>(a, s);
    case SBX_FLOAT: return launch_kron_typed<float>(a, s);
    default: throw Error("kron bsr: unsupported type");
    }
}

} // namespace sbx
