// Dense batched solvers on small column-major matrices: Cholesky (upper), LU with partial
// pivoting + solve, triangular solve -- the local steps of superbblas's dense.h
// (local_cholesky dense.h:56-123 -> potrf('U'), local_gesm 253-330 -> getrf + getrs('N'),
// local_inversion 335-440 -> getrf + getri, local_trsm 136-200 -> trsm(side, 'U', 'N', 'N')),
// where the reference calls rocsolver / rocblas batched routines.
//
// One 256-thread workgroup per matrix.  The matrix is staged in LDS when it fits
// (n*n*sizeof(E) <= 64 KB: n <= 64 for complex<double>) and updated in place in global memory
// otherwise; every step is a right-looking rank-1 update spread over the threads of the
// workgroup.  Pivoting follows LAPACK's i?amax (largest |re| + |im|, first index on ties), so
// pivot sequences match the reference's.  Right-hand sides are solved one column (or row) per
// thread against the factor in LDS (wave-uniform reads).  A non-positive pivot (Cholesky) or a
// zero pivot (LU) stops the factorization of that matrix and is reported as the LAPACK info.
#include "elem_ops.h"
#include "sbx_internal.h"

#include <type_traits>

#include <algorithm>

namespace sbx {
// 2: the small-matrix wave kernels for the factorizations and the triangular solves (round 5:
// 12 rhs per site trsm 467 -> 266 us; the multi-rank dense cases run with every setting,
// tests/dist_worker.py case_dense)
int g_dense_wave = 2;
namespace {

constexpr int DTH = 256;
constexpr long DENSE_LDS_BYTES = 64 * 1024;

template <typename E> struct DOps;
template <> struct DOps<double> {
    static __device__ __forceinline__ double re(double v) { return v; }
    static __device__ __forceinline__ double abs1(double v) { return fabs(v); }
    static __device__ __forceinline__ double conj(double v) { return v; }
    static __device__ __forceinline__ double mul(double a, double b) { return a * b; }
    static __device__ __forceinline__ double sub(double a, double b) { return a - b; }
    static __device__ __forceinline__ double div(double a, double b) { return a / b; }
    static __device__ __forceinline__ double divr(double a, double b) { return a / b; }
    static __device__ __forceinline__ double inv(double b) { return 1.0 / b; }
    static __device__ __forceinline__ double real(double r) { return r; }
    static __device__ __forceinline__ double one() { return 1; }
};
template <> struct DOps<float> {
    static __device__ __forceinline__ double re(float v) { return v; }
    static __device__ __forceinline__ double abs1(float v) { return fabsf(v); }
    static __device__ __forceinline__ float conj(float v) { return v; }
    static __device__ __forceinline__ float mul(float a, float b) { return a * b; }
    static __device__ __forceinline__ float sub(float a, float b) { return a - b; }
    static __device__ __forceinline__ float div(float a, float b) { return a / b; }
    static __device__ __forceinline__ float divr(float a, double b) { return a / (float)b; }
    static __device__ __forceinline__ float inv(float b) { return 1.f / b; }
    static __device__ __forceinline__ float real(double r) { return (float)r; }
    static __device__ __forceinline__ float one() { return 1; }
};
template <typename E, typename R> struct CplxOps {
    static __device__ __forceinline__ double re(E v) { return v.x; }
    static __device__ __forceinline__ double abs1(E v) { return fabs((double)v.x) + fabs((double)v.y); }
    static __device__ __forceinline__ E conj(E v) { return E{v.x, -v.y}; }
    static __device__ __forceinline__ E mul(E a, E b) {
        return E{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x};
    }
    static __device__ __forceinline__ E sub(E a, E b) { return E{a.x - b.x, a.y - b.y}; }
    static __device__ __forceinline__ E div(E a, E b) {
        // Smith's algorithm (robust against overflow, as LAPACK's zladiv family)
        if (fabs((double)b.y) <= fabs((double)b.x)) {
            const R r = b.y / b.x, d = b.x + b.y * r;
            return E{(a.x + a.y * r) / d, (a.y - a.x * r) / d};
        }
        const R r = b.x / b.y, d = b.y + b.x * r;
        return E{(a.x * r + a.y) / d, (a.y * r - a.x) / d};
    }
    /// 1 / b by Smith's algorithm: two real divisions, then a product per use instead of a
    /// complex division per element (LAPACK's getf2 scales the column by the reciprocal pivot)
    /// (branch-free: lanes of different matrices take either form without diverging)
    static __device__ __forceinline__ E inv(E b) {
        const bool xf = fabs((double)b.y) <= fabs((double)b.x);
        const R u = xf ? b.x : b.y, w = xf ? b.y : b.x;
        const R r = w / u, q = (R)1 / (u + w * r);
        return xf ? E{q, -r * q} : E{r * q, -q};
    }
    static __device__ __forceinline__ E divr(E a, double b) { return E{(R)(a.x / b), (R)(a.y / b)}; }
    static __device__ __forceinline__ E real(double r) { return E{(R)r, 0}; }
    static __device__ __forceinline__ E one() { return E{1, 0}; }
};
template <> struct DOps<double2> : CplxOps<double2, double> {};
template <> struct DOps<float2> : CplxOps<float2, float> {};

template <typename E> __device__ __forceinline__ E scale_by(E v, double ar, double ai);
template <> __device__ __forceinline__ double scale_by<double>(double v, double ar, double) { return ar * v; }
template <> __device__ __forceinline__ float scale_by<float>(float v, double ar, double) { return (float)ar * v; }
template <> __device__ __forceinline__ double2 scale_by<double2>(double2 v, double ar, double ai) {
    return double2{ar * v.x - ai * v.y, ar * v.y + ai * v.x};
}
template <> __device__ __forceinline__ float2 scale_by<float2>(float2 v, double ar, double ai) {
    return float2{(float)ar * v.x - (float)ai * v.y, (float)ar * v.y + (float)ai * v.x};
}

/// The matrix of this workgroup: staged in LDS when it fits, else the global copy
template <typename E>
__device__ __forceinline__ E *stage_in(E *g, long nn, bool lds, E *smem) {
    if (!lds) return g;
    for (long e = threadIdx.x; e < nn; e += DTH) smem[e] = g[e];
    __syncthreads();
    return smem;
}
template <typename E> __device__ __forceinline__ void stage_out(E *g, const E *m, long nn, bool lds) {
    __syncthreads();
    if (!lds) return;
    for (long e = threadIdx.x; e < nn; e += DTH) g[e] = m[e];
}

/// Where a factorization reports its LAPACK info: the per-matrix array in device memory and a
/// host-mapped flag that any failed matrix sets, so that a batch without failures costs the host
/// one stream synchronisation and a read of host memory (no memset, search kernel or copy back)
struct InfoOut {
    int *v;   // per matrix (device)
    int *any; // host-mapped, coherent
    __device__ __forceinline__ void put(long i, int bad) const {
        v[i] = bad;
        if (bad) *any = 1;
    }
};

// Cholesky, upper: A = U^H U, U over the upper triangle, the strict lower part untouched
template <typename E>
__global__ void __launch_bounds__(DTH) potrf_kernel(E *a, long n, int lds, InfoOut info) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    typedef DOps<E> O;
    E *g = a + (long)blockIdx.x * n * n;
    E *M = stage_in(g, n * n, lds != 0, (E *)smem_raw);
    int bad = 0;
    for (long j = 0; j < n; ++j) {
        __syncthreads();
        double d = O::re(M[j + j * n]);
        if (!(d > 0)) {
            bad = (int)j + 1;
            break;
        }
        d = sqrt(d);
        __syncthreads();
        if (threadIdx.x == 0) M[j + j * n] = O::real(d);
        for (long c = j + 1 + threadIdx.x; c < n; c += DTH) M[j + c * n] = O::divr(M[j + c * n], d);
        __syncthreads();
        const long w = n - j - 1;
        for (long e = threadIdx.x; e < w * w; e += DTH) {
            const long r = j + 1 + e % w, c = j + 1 + e / w;
            if (r <= c) M[r + c * n] = O::sub(M[r + c * n], O::mul(O::conj(M[j + r * n]), M[j + c * n]));
        }
    }
    stage_out(g, M, n * n, lds != 0);
    if (threadIdx.x == 0) info.put(blockIdx.x, bad);
}

// LU with partial pivoting (getrf), then B <- alpha A^-1 B for the n x m column-major panel of
// this matrix (getrs 'N'); identity != 0 makes B the identity first (the inverse, getri)
template <typename E>
__global__ void __launch_bounds__(DTH) gesv_kernel(E *a, long n, E *b, long m, int identity,
                                                   double alpha_re, double alpha_im, int lds,
                                                   int *ipiv_g, InfoOut info) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    __shared__ double best_v[DTH];
    __shared__ int best_i[DTH];
    typedef DOps<E> O;
    E *g = a + (long)blockIdx.x * n * n;
    E *M = stage_in(g, n * n, lds != 0, (E *)smem_raw);
    int *piv = ipiv_g + (long)blockIdx.x * n;
    int bad = 0;
    for (long j = 0; j < n; ++j) {
        // pivot: the largest |re| + |im| in column j at or below the diagonal, first on ties
        double bv = -1;
        int bi = (int)j;
        for (long r = j + threadIdx.x; r < n; r += DTH) {
            const double v = O::abs1(M[r + j * n]);
            if (v > bv) {
                bv = v;
                bi = (int)r;
            }
        }
        best_v[threadIdx.x] = bv;
        best_i[threadIdx.x] = bi;
        __syncthreads();
        for (int s = DTH / 2; s > 0; s >>= 1) {
            if ((int)threadIdx.x < s) {
                const double ov = best_v[threadIdx.x + s];
                const int oi = best_i[threadIdx.x + s];
                if (ov > best_v[threadIdx.x] || (ov == best_v[threadIdx.x] && oi < best_i[threadIdx.x])) {
                    best_v[threadIdx.x] = ov;
                    best_i[threadIdx.x] = oi;
                }
            }
            __syncthreads();
        }
        const long p = best_i[0];
        const double pv = best_v[0];
        if (threadIdx.x == 0) piv[j] = (int)p;
        __syncthreads();
        if (!(pv > 0)) {
            bad = (int)j + 1;
            break;
        }
        if (p != j)
            for (long c = threadIdx.x; c < n; c += DTH) {
                const E t = M[j + c * n];
                M[j + c * n] = M[p + c * n];
                M[p + c * n] = t;
            }
        __syncthreads();
        const E d = M[j + j * n];
        for (long r = j + 1 + threadIdx.x; r < n; r += DTH) M[r + j * n] = O::div(M[r + j * n], d);
        __syncthreads();
        const long w = n - j - 1;
        for (long e = threadIdx.x; e < w * w; e += DTH) {
            const long r = j + 1 + e % w, c = j + 1 + e / w;
            M[r + c * n] = O::sub(M[r + c * n], O::mul(M[r + j * n], M[j + c * n]));
        }
        __syncthreads();
    }
    if (!bad && b) {
        // one right-hand side per thread: P, L (unit), U
        E *B = b + (long)blockIdx.x * n * m;
        for (long col = threadIdx.x; col < m; col += DTH) {
            E *x = B + col * n;
            if (identity)
                for (long r = 0; r < n; ++r) x[r] = r == col ? O::one() : O::real(0);
            for (long j = 0; j < n; ++j) {
                const long p = piv[j];
                if (p != j) {
                    const E t = x[j];
                    x[j] = x[p];
                    x[p] = t;
                }
            }
            for (long r = 0; r < n; ++r) {
                E v = x[r];
                for (long q = 0; q < r; ++q) v = O::sub(v, O::mul(M[r + q * n], x[q]));
                x[r] = v;
            }
            for (long r = n - 1; r >= 0; --r) {
                E v = x[r];
                for (long q = r + 1; q < n; ++q) v = O::sub(v, O::mul(M[r + q * n], x[q]));
                x[r] = O::div(v, M[r + r * n]);
            }
            if (alpha_re != 1 || alpha_im != 0)
                for (long r = 0; r < n; ++r) x[r] = scale_by<E>(x[r], alpha_re, alpha_im);
        }
    }
    stage_out(g, M, n * n, lds != 0);
    if (threadIdx.x == 0) info.put(blockIdx.x, bad);
}

// Upper triangular solve: left  X (n x m, ld n) <- alpha U^-1 X;  right X (m x n, ld m) <- alpha X U^-1
template <typename E>
__global__ void __launch_bounds__(DTH) trsm_kernel(const E *a, long n, E *x, long m, int left,
                                                   double alpha_re, double alpha_im, int lds) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    typedef DOps<E> O;
    const E *U = a + (long)blockIdx.x * n * n;
    if (lds) {
        E *s = (E *)smem_raw;
        for (long e = threadIdx.x; e < n * n; e += DTH) s[e] = U[e];
        __syncthreads();
        U = s;
    }
    E *X = x + (long)blockIdx.x * n * m;
    for (long t = threadIdx.x; t < m; t += DTH) {
        if (left) {
            E *col = X + t * n;
            for (long r = n - 1; r >= 0; --r) {
                E v = scale_by<E>(col[r], alpha_re, alpha_im);
                for (long q = r + 1; q < n; ++q) v = O::sub(v, O::mul(U[r + q * n], col[q]));
                col[r] = O::div(v, U[r + r * n]);
            }
        } else {
            for (long c = 0; c < n; ++c) {
                E v = scale_by<E>(X[t + c * m], alpha_re, alpha_im);
                for (long q = 0; q < c; ++q) v = O::sub(v, O::mul(X[t + q * m], U[q + c * n]));
                X[t + c * m] = O::div(v, U[c + c * n]);
            }
        }
    }
}

// Small matrices (n <= 16: the 12x12 spin-color blocks of a lattice, 3x3 color blocks): 64 / n
// matrices per wave, four waves per workgroup, no barrier.  A lane holds one column of one
// matrix in registers; a step's pivot, multipliers and row are shuffled from the matrix's lanes,
// so the factorisation is wave-synchronous.  The arithmetic is the block kernels' operation for
// operation (same pivots, same multiply / subtract order), so results agree with them bit for bit
// up to the compiler's contraction choices.  The solve keeps one right-hand side per lane, the
// factors in the wave's LDS slice (broadcast reads).
constexpr int WNMAX = 16;

template <typename E> __device__ __forceinline__ E wshfl(E v, int l);
template <> __device__ __forceinline__ double wshfl<double>(double v, int l) { return __shfl(v, l); }
template <> __device__ __forceinline__ float wshfl<float>(float v, int l) { return __shfl(v, l); }
template <> __device__ __forceinline__ double2 wshfl<double2>(double2 v, int l) {
    return double2{__shfl(v.x, l), __shfl(v.y, l)};
}
template <> __device__ __forceinline__ float2 wshfl<float2>(float2 v, int l) {
    return float2{__shfl(v.x, l), __shfl(v.y, l)};
}

/// A column of up to N elements in registers; complex elements as separate real and imaginary
/// arrays (arrays of the vector types are not promoted to registers: they went to scratch)
template <typename E, int N> struct Col {
    E v[N];
    __device__ __forceinline__ E get(int r) const { return v[r]; }
    __device__ __forceinline__ void set(int r, E e) { v[r] = e; }
};
template <typename E, typename R, int N> struct CCol {
    R re[N], im[N];
    __device__ __forceinline__ E get(int r) const { return E{re[r], im[r]}; }
    __device__ __forceinline__ void set(int r, E e) {
        re[r] = e.x;
        im[r] = e.y;
    }
};
template <int N> struct Col<double2, N> : CCol<double2, double, N> {};
template <int N> struct Col<float2, N> : CCol<float2, float, N> {};

// A wave holds G = 64 / n matrices: lane l = n s + c is column c of slot s (lanes past G n
// idle); slots past the batch hold the identity and write nothing.
template <typename E, int WNM, bool FULL = false>
__global__ void __launch_bounds__(256) potrf_wave_kernel(E *a, int n_, long k, InfoOut info, int rm) {
    const int n = FULL ? WNM : n_; // (FULL: a compile-time size, no conditional steps; the
                                   // solve kernels spill in that form, so only potrf / inversion)
    typedef DOps<E> O;
    const int lane = threadIdx.x & 63, G = 64 / n;
    const int s = lane / n, c = lane - s * n, s0 = s * n;
    const long mi = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * G + s;
    const bool valid = s < G && mi < k;
    E *g = a + (valid ? mi : 0) * n * n;
    Col<E, WNM> v;
#pragma unroll
    for (int r = 0; r < WNM; ++r)
        v.set(r, r < n ? (valid ? g[rm ? c + (long)r * n : r + (long)c * n] : (r == c ? O::one() : O::real(0)))
                       : O::real(0));
    int bad = 0;
    // (no early exits: constant trip counts, so the loops unroll fully and the columns stay in
    // registers; with breaks the 12- and 16-row complex forms went to scratch)
#pragma unroll
    for (int j = 0; j < WNM; ++j) {
        if (j >= n) continue;
        double d = wshfl<double>(O::re(v.get(j)), s0 + j);
        const bool ok = !bad && d > 0;
        if (!bad && !(d > 0)) bad = j + 1;
        d = sqrt(ok ? d : 1.0);
        if (ok && c == j) v.set(j, O::real(d));
        if (ok && c > j) v.set(j, O::divr(v.get(j), d));
        const E vj = v.get(j);
        // row j of U: element r from the slot's lane r
#pragma unroll
        for (int r = j + 1; r < WNM; ++r) {
            const E rj = wshfl<E>(vj, s0 + r);
            if (ok && r <= c && r < n) v.set(r, O::sub(v.get(r), O::mul(O::conj(rj), vj)));
        }
    }
    if (valid)
#pragma unroll
        for (int r = 0; r < WNM; ++r)
            if (r < n) g[rm ? c + (long)r * n : r + (long)c * n] = v.get(r);
    if (valid && c == 0) info.put(mi, bad);
}

template <typename E, int WNM>
__global__ void __launch_bounds__(256) gesv_wave_kernel(E *a, int n, long k, const E *bx, E *b, long m, int identity,
                                                        double alpha_re, double alpha_im,
                                                        InfoOut info, int rm, int keep_lu, int xsi, int xst,
                                                        int ysi, int yst) {
    typedef DOps<E> O;
    __shared__ E lu_s[4][64 * WNM];
    __shared__ E dinv_s[4][64];
    __shared__ int piv_s[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, G = 64 / n;
    const int s = lane / n, c = lane - s * n, s0 = s * n;
    const long mi = ((long)blockIdx.x * 4 + w) * G + s;
    const bool valid = s < G && mi < k;
    E *g = a + (valid ? mi : 0) * n * n;
    Col<E, WNM> v;
#pragma unroll
    for (int r = 0; r < WNM; ++r)
        v.set(r, r < n ? (valid ? g[rm ? c + (long)r * n : r + (long)c * n] : (r == c ? O::one() : O::real(0)))
                       : O::real(0));
    int bad = 0;
#pragma unroll
    for (int j = 0; j < WNM; ++j) {
        if (j >= n) continue;
        // pivot: the largest |re| + |im| in column j at or below the diagonal, first on ties
        double bv = -1;
        int bi = j;
#pragma unroll
        for (int r = j; r < WNM; ++r)
            if (r < n) {
                const double t = O::abs1(v.get(r));
                if (t > bv) {
                    bv = t;
                    bi = r;
                }
            }
        const int p = __shfl(bi, s0 + j);
        const double pv = __shfl(bv, s0 + j);
        if (!bad && c == 0 && s < G) piv_s[w][s0 + j] = p;
        const bool ok = !bad && pv > 0;
        if (!bad && !(pv > 0)) bad = j + 1;
        if (ok && p != j) {
            E vp = v.get(j);
#pragma unroll
            for (int r = j + 1; r < WNM; ++r)
                if (r == p) vp = v.get(r);
#pragma unroll
            for (int r = j + 1; r < WNM; ++r)
                if (r == p) v.set(r, v.get(j));
            v.set(j, vp);
        }
        // the multipliers: the column times the reciprocal pivot (kept for the solve's U^-1)
        const E dinv = O::inv(wshfl<E>(v.get(j), s0 + j));
        if (c == j && s < G) dinv_s[w][s0 + j] = dinv;
        if (ok && c == j)
#pragma unroll
            for (int r = j + 1; r < WNM; ++r)
                if (r < n) v.set(r, O::mul(v.get(r), dinv));
        const E vj = v.get(j);
#pragma unroll
        for (int r = j + 1; r < WNM; ++r) {
            if (r >= n) continue;
            const E l = wshfl<E>(v.get(r), s0 + j);
            if (ok && c > j) v.set(r, O::sub(v.get(r), O::mul(l, vj)));
        }
    }
    // the factors in LDS row-major (the lanes' writes consecutive), one element of padding per
    // matrix where it fits: the matrices of a wave read their factors' element (r, q) together,
    // and n^2 elements apart they would all fall on the same LDS banks
    const int ldm = G * (n * n + 1) <= 64 * WNM ? n * n + 1 : n * n;
    if (s < G)
#pragma unroll
        for (int r = 0; r < WNM; ++r)
            if (r < n) {
                if (valid && keep_lu) g[rm ? c + (long)r * n : r + (long)c * n] = v.get(r);
                lu_s[w][s * ldm + r * n + c] = v.get(r);
            }
    if (valid && !bad && b) {
        // (the wave's LDS writes above are ordered before its reads below)
        const E *M = lu_s[w] + s * ldm;
        const E *Dinv = dinv_s[w] + s0;
        const int *piv = piv_s[w] + s0;
        // right-hand side column col: element r at r * xsi + col * xst of the matrix's n x m
        // block of bx, the solution written at r * ysi + col * yst of b's (bx may be b)
        const E *BX = bx + mi * n * m;
        E *B = b + mi * n * m;
        for (long col = c; col < m; col += n) {
            const E *xg = BX + col * xst;
            E *yg = B + col * yst;
            Col<E, WNM> x;
#pragma unroll
            for (int r = 0; r < WNM; ++r)
                x.set(r, r < n ? (identity ? (r == col ? O::one() : O::real(0)) : xg[r * xsi]) : O::real(0));
#pragma unroll
            for (int j = 0; j < WNM; ++j) {
                if (j >= n) continue;
                const int p = piv[j];
                if (p != j) {
                    E xp = x.get(j);
#pragma unroll
                    for (int r = j + 1; r < WNM; ++r)
                        if (r == p) xp = x.get(r);
#pragma unroll
                    for (int r = j + 1; r < WNM; ++r)
                        if (r == p) x.set(r, x.get(j));
                    x.set(j, xp);
                }
            }
#pragma unroll
            for (int r = 0; r < WNM; ++r) {
                if (r >= n) continue;
                E t = x.get(r);
#pragma unroll
                for (int q = 0; q < r; ++q) t = O::sub(t, O::mul(M[r * n + q], x.get(q)));
                x.set(r, t);
            }
#pragma unroll
            for (int r = WNM - 1; r >= 0; --r) {
                if (r >= n) continue;
                E t = x.get(r);
#pragma unroll
                for (int q = r + 1; q < WNM; ++q)
                    if (q < n) t = O::sub(t, O::mul(M[r * n + q], x.get(q)));
                x.set(r, O::mul(t, Dinv[r]));
            }
            if (alpha_re != 1 || alpha_im != 0)
#pragma unroll
                for (int r = 0; r < WNM; ++r) x.set(r, scale_by<E>(x.get(r), alpha_re, alpha_im));
#pragma unroll
            for (int r = 0; r < WNM; ++r)
                if (r < n) yg[r * ysi] = x.get(r);
        }
    }
    if (valid && c == 0) info.put(mi, bad);
}

/// lane L's value of each 16-lane row (DPP row_newbcast: a VALU move, no LDS)
template <int L> __device__ __forceinline__ int rbc_i(int v) {
    return __builtin_amdgcn_mov_dpp(v, 0x150 + L, 0xf, 0xf, true);
}
template <int L> __device__ __forceinline__ float rbc(float v) {
    return __builtin_bit_cast(float, rbc_i<L>(__builtin_bit_cast(int, v)));
}
template <int L> __device__ __forceinline__ double rbc(double v) {
    const long long b = __builtin_bit_cast(long long, v);
    const int lo = rbc_i<L>((int)b), hi = rbc_i<L>((int)(b >> 32));
    return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
template <int L> __device__ __forceinline__ double2 rbc(double2 v) { return double2{rbc<L>(v.x), rbc<L>(v.y)}; }
template <int L> __device__ __forceinline__ float2 rbc(float2 v) { return float2{rbc<L>(v.x), rbc<L>(v.y)}; }

// In-place inversion of small matrices (n <= 16, B = A^-1, B may be A): Gauss-Jordan with
// LAPACK's partial pivoting (largest |re| + |im| at or below the diagonal, first on ties; rows
// swapped), one 16-lane row of the wave per matrix, lane c holding column c in registers.  A
// step's pivot column reaches the other lanes by DPP row broadcasts (no LDS, no barrier); the
// pivot column is replaced by the inverse's column as it is eliminated, and the row swaps are
// undone on the columns at the end (one shuffle per element).  getrf + getri in one pass over
// registers: n^3 complex multiply-adds per matrix, the matrix read and written once.
/// One Gauss-Jordan elimination update of a complex<double> element on every lane:
///   (re, im) = (x, y) s - (x, y)[lane L of the 16-lane row] * (ar, ai)
/// the broadcast folded into the FP64 FMAs as their DPP row_newbcast operand (the separate 32-bit
/// broadcast moves cost 4 VALU instructions per element, the selects of lane L's column 4 more);
/// the two multiplies come first, so the DPP reads of x and y are 2 instructions after any write
template <int L>
__device__ __forceinline__ void gj_update(double x, double y, double s, double ar, double ai, double &re, double &im) {
    const double nar = -ar, nai = -ai;
    asm volatile("v_mul_f64 %0, %2, %4\n\t"
                 "v_mul_f64 %1, %3, %4\n\t"
                 "v_fmac_f64_dpp %0, %2, %5 row_newbcast:%8 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %0, %3, %6 row_newbcast:%8 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %1, %2, %7 row_newbcast:%8 row_mask:0xf bank_mask:0xf\n\t"
                 "v_fmac_f64_dpp %1, %3, %5 row_newbcast:%8 row_mask:0xf bank_mask:0xf"
                 : "=&v"(re), "=&v"(im)
                 : "v"(x), "v"(y), "v"(s), "v"(nar), "v"(ai), "v"(nai), "i"(L));
}
/// the real form: re = x s - x[lane L] * ar
template <int L> __device__ __forceinline__ void gj_update(double x, double s, double ar, double &re) {
    const double nar = -ar;
    asm volatile("v_mul_f64 %0, %1, %2\n\t"
                 "s_nop 0\n\t"
                 "v_fmac_f64_dpp %0, %1, %3 row_newbcast:%4 row_mask:0xf bank_mask:0xf"
                 : "=&v"(re)
                 : "v"(x), "v"(s), "v"(nar), "i"(L));
}

template <typename E, int WNM, int J>
__device__ __forceinline__ void gj_step(Col<E, WNM> &v, int n, int c, int &bad, int (&pj)[WNM]) {
    typedef DOps<E> O;
    if constexpr (J < WNM) {
        if (J < n) {
            double bv = -1;
            int bi = J;
#pragma unroll
            for (int r = J; r < WNM; ++r)
                if (r < n) {
                    const double t = O::abs1(v.get(r));
                    if (t > bv) {
                        bv = t;
                        bi = r;
                    }
                }
            const int p = rbc_i<J>(bi);
            const double pv = rbc<J>(bv);
            const bool ok = !bad && pv > 0;
            if (!bad && !(pv > 0)) bad = J + 1;
            pj[J] = ok ? p : J;
            if (ok && p != J) {
                E vp = v.get(J);
#pragma unroll
                for (int r = J + 1; r < WNM; ++r)
                    if (r == p) vp = v.get(r);
#pragma unroll
                for (int r = J + 1; r < WNM; ++r)
                    if (r == p) v.set(r, v.get(J));
                v.set(J, vp);
            }
            const E dinv = O::inv(rbc<J>(v.get(J)));
            // the pivot row scaled; the pivot column (lane J) as the identity's column.  (A
            // singular matrix -- !ok -- goes on with infinities: its lanes are its own and its
            // result is not written.)
            const E aj = O::mul(c == J ? O::one() : v.get(J), dinv);
            if constexpr (std::is_same<E, double2>::value || std::is_same<E, double>::value) {
                // v(r) <- v(r) s - v(r)[lane J] aj with s = 0 on lane J (its column becomes the
                // inverse's) and 1 elsewhere: a multiply and DPP-broadcast FMAs, no selects
                const double sc = c == J ? 0.0 : 1.0;
#pragma unroll
                for (int r = 0; r < WNM; ++r) {
                    if (r >= n || r == J) continue;
                    const E vr = v.get(r);
                    if constexpr (std::is_same<E, double2>::value) {
                        double re, im;
                        gj_update<J>(vr.x, vr.y, sc, aj.x, aj.y, re, im);
                        v.set(r, double2{re, im});
                    } else {
                        double re;
                        gj_update<J>(vr, sc, aj, re);
                        v.set(r, re);
                    }
                }
            } else {
#pragma unroll
                for (int r = 0; r < WNM; ++r) {
                    if (r >= n || r == J) continue;
                    const E mr = rbc<J>(v.get(r));
                    v.set(r, O::sub(c == J ? O::real(0) : v.get(r), O::mul(mr, aj)));
                }
            }
            v.set(J, aj);
        }
        gj_step<E, WNM, J + 1>(v, n, c, bad, pj);
    }
}

// FULL: n == WNM (4, 8, 12, 16): the size a compile-time constant, so no step is conditional
// (the conditional steps' register merges cost a 64-bit move per element and step)
template <typename E, int WNM, bool FULL = false>
__global__ void __launch_bounds__(256) inv_wave_kernel(const E *a, int n_, long k, E *b, InfoOut info, int rm) {
    typedef DOps<E> O;
    const int n = FULL ? WNM : n_;
    const int lane = threadIdx.x & 63, s = lane >> 4, c = lane & 15;
    const long mi = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4 + s;
    const bool live = mi < k, valid = live && c < n;
    const E *g = a + (live ? mi : 0) * n * n;
    // lanes past n and matrices past the batch: identity columns (well-defined pivots)
    Col<E, WNM> v;
#pragma unroll
    for (int r = 0; r < WNM; ++r)
        v.set(r, (r < n && valid) ? g[rm ? c + (long)r * n : r + (long)c * n] : (r == c ? O::one() : O::real(0)));
    int bad = 0, pj[WNM];
    gj_step<E, WNM, 0>(v, n, c, bad, pj);
    // undo the row swaps on the columns (last swap first): column c of A^-1 is column src
    int src = c;
#pragma unroll
    for (int l = 0; l < WNM; ++l)
        if (l < n) src = src == l ? pj[l] : (src == pj[l] ? l : src);
    const int from = (lane & 48) + src;
    E *o = b + (live ? mi : 0) * n * n;
#pragma unroll
    for (int r = 0; r < WNM; ++r) {
        if (r >= n) continue;
        const E e = wshfl<E>(v.get(r), from);
        if (valid && !bad) o[rm ? c + (long)r * n : r + (long)c * n] = e;
    }
    if (live && c == 0) info.put(mi, bad);
}

// Triangular solves with small factors (n <= 16): a lane per right-hand side (left: a column of
// X; right: a row), 64 / m matrices per wave when m <= 64, the factor's elements read by every
// lane of its matrix (one address per matrix: broadcast loads); the block kernel's operation
// order.
template <typename E, int WNM>
__global__ void __launch_bounds__(256) trsm_wave_kernel(const E *a, int n, long k, E *x, long m, int left,
                                                        double alpha_re, double alpha_im) {
    typedef DOps<E> O;
    const int lane = threadIdx.x & 63;
    const int per = m <= 64 ? (int)(64 / m) : 1;
    const int s = m <= 64 ? lane / (int)m : 0;
    const long mi = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * per + s;
    if (s >= per || mi >= k) return;
    const E *U = a + mi * n * n;
    E *X = x + mi * n * m;
    // the reciprocals of U's diagonal: when the matrix has at least n lanes, lane q of the matrix
    // computes 1 / U(q, q) and the others read it (one reciprocal per lane instead of n
    // divisions).  The shuffles happen here, before the loop over right-hand sides, while every
    // lane of the matrix is still active: with m > 64 the last pass leaves lanes l >= m % 64
    // idle, and a cross-lane read from an idle lane is undefined.
    const int mp = m <= 64 ? (int)m : 64, base = m <= 64 ? s * (int)m : 0, tl = lane - base;
    const bool shared = mp >= n;
    const E rinv = O::inv(U[(tl < n ? tl : 0) * (n + 1)]);
    E dv[WNM];
#pragma unroll
    for (int r = 0; r < WNM; ++r)
        dv[r] = r < n ? (shared ? wshfl<E>(rinv, base + r) : O::inv(U[r + r * n])) : O::real(0);
    auto dinv = [&](int r) { return dv[r]; };
    for (long t = m <= 64 ? lane - (long)s * m : lane; t < m; t += (m <= 64 ? m : 64)) {
        Col<E, WNM> v;
        const long base = left ? t * n : t, st = left ? 1 : m;
#pragma unroll
        for (int r = 0; r < WNM; ++r) v.set(r, r < n ? X[base + r * st] : O::real(0));
        if (left) {
#pragma unroll
            for (int r = WNM - 1; r >= 0; --r) {
                if (r >= n) continue;
                E w = scale_by<E>(v.get(r), alpha_re, alpha_im);
#pragma unroll
                for (int q = r + 1; q < WNM; ++q)
                    if (q < n) w = O::sub(w, O::mul(U[r + q * n], v.get(q)));
                v.set(r, O::mul(w, dinv(r)));
            }
        } else {
#pragma unroll
            for (int c = 0; c < WNM; ++c) {
                if (c >= n) continue;
                E w = scale_by<E>(v.get(c), alpha_re, alpha_im);
#pragma unroll
                for (int q = 0; q < c; ++q) w = O::sub(w, O::mul(v.get(q), U[q + c * n]));
                v.set(c, O::mul(w, dinv(c)));
            }
        }
#pragma unroll
        for (int r = 0; r < WNM; ++r)
            if (r < n) X[base + r * st] = v.get(r);
    }
}

// Triangular solves straight between the caller's tensors (n <= 16, m <= 64 right-hand sides
// per matrix): a wave's 64 / m matrices have their right-hand sides x and their solutions y as
// contiguous blocks of n x m elements; the wave moves its x blocks into LDS with coalesced
// 16-byte loads, each lane reads its vector there (component i, right-hand side t at
// i * xsi + t * xst of its block: either orientation), solves it exactly as trsm_wave_kernel does,
// writes the result back into the slice in y's orientation and the wave stores the blocks with
// coalesced stores.  The factor is read row- or column-major (rm).
template <typename E, int WNM>
__global__ void __launch_bounds__(256) trsm_io_kernel(const E *a, int n, long k, int rm, const E *x, int xsi,
                                                      int xst, E *y, int ysi, int yst, int m, int left,
                                                      double alpha_re, double alpha_im) {
    typedef DOps<E> O;
    __shared__ E io_s[4][64 * WNM];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int per = 64 / m, s = lane / m, t = lane - s * m;
    const long mi0 = ((long)blockIdx.x * 4 + w) * per; // the wave's first matrix
    const int nm = n * m;
    const int nblk = (int)min((long)per, k - mi0 > 0 ? k - mi0 : 0L); // the wave's matrices
    E *sl = io_s[w];
    // a run of cnt elements from global memory into the slice: every load issued before the
    // first LDS write (cnt <= 64 WNM: per m <= 64); a loop of load -> write pairs waits out one
    // memory latency per pass
    auto stage = [&](const E *src, int cnt) {
        Col<E, WNM> t_; // (complex: separate real / imaginary arrays, kept in registers)
#pragma unroll
        for (int i = 0; i < WNM; ++i)
            t_.set(i, lane + 64 * i < cnt ? src[lane + 64 * i] : O::real(0));
#pragma unroll
        for (int i = 0; i < WNM; ++i)
            if (lane + 64 * i < cnt) sl[lane + 64 * i] = t_.get(i);
    };
    // the wave's x blocks (one contiguous run of nblk * n * m elements)
    stage(x + mi0 * nm, nblk * nm);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    const bool live = s < nblk;
    const long mi = live ? mi0 + s : 0;
    Col<E, WNM> v;
    const E *xb = sl + s * nm;
#pragma unroll
    for (int r = 0; r < WNM; ++r) v.set(r, (r < n && live) ? xb[r * xsi + t * xst] : O::real(0));
    // the factors of the wave's matrices into the slice too when they fit it (m >= n): every
    // product then reads its factor element from LDS (a broadcast within the matrix's lanes)
    const int nn = n * n;
    const bool ulds = per * nn <= 64 * WNM;
    // (one element of padding per factor where it fits: the wave's matrices read their factors'
    // element (r, q) together, and nn elements apart they would fall on the same LDS banks)
    const int ldu = per * (nn + 1) <= 64 * WNM ? nn + 1 : nn;
    if (ulds) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); // every lane has read its x
        __builtin_amdgcn_wave_barrier();
        if (ldu == nn) {
            stage(a + mi0 * nn, nblk * nn);
        } else {
            const E *src = a + mi0 * nn;
            const int cnt = nblk * nn;
            Col<E, WNM> t_;
#pragma unroll
            for (int i = 0; i < WNM; ++i) t_.set(i, lane + 64 * i < cnt ? src[lane + 64 * i] : O::real(0));
#pragma unroll
            for (int i = 0; i < WNM; ++i) {
                const int e = lane + 64 * i;
                if (e < cnt) sl[e + e / nn] = t_.get(i);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
    }
    const E *U = ulds ? sl + s * ldu : a + mi * nn;
    auto u = [&](int r, int q) { return rm ? U[r * n + q] : U[r + q * n]; };
    // the diagonal's reciprocals from the matrix's own lanes (m >= n), else per lane
    const bool shared = m >= n;
    const int tl = t < n ? t : 0;
    const E rinv = O::inv(u(tl, tl));
    auto dinv = [&](int r) { return shared ? wshfl<E>(rinv, s * m + r) : O::inv(u(r, r)); };
    if (left) {
#pragma unroll
        for (int r = WNM - 1; r >= 0; --r) {
            if (r >= n) continue;
            E wv = scale_by<E>(v.get(r), alpha_re, alpha_im);
#pragma unroll
            for (int q = r + 1; q < WNM; ++q)
                if (q < n) wv = O::sub(wv, O::mul(u(r, q), v.get(q)));
            v.set(r, O::mul(wv, dinv(r)));
        }
    } else {
#pragma unroll
        for (int c = 0; c < WNM; ++c) {
            if (c >= n) continue;
            E wv = scale_by<E>(v.get(c), alpha_re, alpha_im);
#pragma unroll
            for (int q = 0; q < c; ++q) wv = O::sub(wv, O::mul(v.get(q), u(q, c)));
            v.set(c, O::mul(wv, dinv(c)));
        }
    }
    // every lane has read its x vector (and its factor) before any lane overwrites the slice
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    E *yb = sl + s * nm;
    if (live)
#pragma unroll
        for (int r = 0; r < WNM; ++r)
            if (r < n) yb[r * ysi + t * yst] = v.get(r);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    {
        Col<E, WNM> t_;
        const int cnt = nblk * nm;
#pragma unroll
        for (int i = 0; i < WNM; ++i) t_.set(i, lane + 64 * i < cnt ? sl[lane + 64 * i] : O::real(0));
#pragma unroll
        for (int i = 0; i < WNM; ++i)
            if (lane + 64 * i < cnt) y[mi0 * nm + lane + 64 * i] = t_.get(i);
    }
}

template <typename E> bool fits_lds(long n) { return n * n * (long)sizeof(E) <= DENSE_LDS_BYTES; }

template <typename E> void potrf_typed(void *a, long n, long k, InfoOut info, bool rm, hipStream_t s) {
    if (n <= WNMAX && g_dense_wave) {
        auto go = [&](auto kern) {
            const long per = 4 * (64 / n);
            hipLaunchKernelGGL(kern, dim3((unsigned)((k + per - 1) / per)), dim3(256), 0, s, (E *)a, (int)n, k, info,
                               rm ? 1 : 0);
        };
        if (n == 4) go(potrf_wave_kernel<E, 4, true>);
        else if (n < 4) go(potrf_wave_kernel<E, 4>);
        else if (n == 8) go(potrf_wave_kernel<E, 8, true>);
        else if (n < 8) go(potrf_wave_kernel<E, 8>);
        else if (n == 12) go(potrf_wave_kernel<E, 12, true>);
        else if (n < 12) go(potrf_wave_kernel<E, 12>);
        else if (n == 16) go(potrf_wave_kernel<E, 16, true>);
        else go(potrf_wave_kernel<E, 16>);
        SBX_HIP_CHECK(hipGetLastError());
        return;
    }
    if (rm) throw Error("dense: internal error (row-major matrices need the wave kernels)");
    const bool lds = fits_lds<E>(n);
    hipLaunchKernelGGL(potrf_kernel<E>, dim3((unsigned)k), dim3(DTH),
                       lds ? (size_t)(n * n * sizeof(E)) : 0, s, (E *)a, n, lds ? 1 : 0, info);
    SBX_HIP_CHECK(hipGetLastError());
}
struct GesvIO {
    const void *x = nullptr; // right-hand sides (nullptr: b itself)
    int xsi = 0, xst = 0, ysi = 0, yst = 0; // 0: the orientation of rm (row-major or column-major)
};

template <typename E>
void gesv_typed(void *a, long n, long k, void *b, long m, bool identity, const Scalar &alpha,
                int *ipiv, InfoOut info, bool rm, bool keep_lu, hipStream_t s, const GesvIO &io = GesvIO{}) {
    if (n <= WNMAX && g_dense_wave && identity && !keep_lu && alpha.re == 1 && alpha.im == 0) {
        // the inverse only (the factors not kept): Gauss-Jordan, a 16-lane row per matrix
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned)((k + 15) / 16)), dim3(256), 0, s, (const E *)a, (int)n, k,
                               (E *)b, info, rm ? 1 : 0);
        };
        if (n == 4) go(inv_wave_kernel<E, 4, true>);
        else if (n < 4) go(inv_wave_kernel<E, 4>);
        else if (n == 8) go(inv_wave_kernel<E, 8, true>);
        else if (n < 8) go(inv_wave_kernel<E, 8>);
        else if (n == 12) go(inv_wave_kernel<E, 12, true>);
        else if (n < 12) go(inv_wave_kernel<E, 12>);
        else if (n == 16) go(inv_wave_kernel<E, 16, true>);
        else go(inv_wave_kernel<E, 16>);
        SBX_HIP_CHECK(hipGetLastError());
        return;
    }
    if (n <= WNMAX && g_dense_wave) {
        const int xsi = io.xsi ? io.xsi : (rm ? (int)m : 1), xst = io.xst ? io.xst : (rm ? 1 : (int)n);
        const int ysi = io.ysi ? io.ysi : (rm ? (int)m : 1), yst = io.yst ? io.yst : (rm ? 1 : (int)n);
        auto go = [&](auto kern) {
            const long per = 4 * (64 / n);
            hipLaunchKernelGGL(kern, dim3((unsigned)((k + per - 1) / per)), dim3(256), 0, s, (E *)a, (int)n, k,
                               (const E *)(io.x ? io.x : b), (E *)b, m, identity ? 1 : 0, alpha.re, alpha.im,
                               info, rm ? 1 : 0, keep_lu ? 1 : 0, xsi, xst, ysi, yst);
        };
        if (n <= 4) go(gesv_wave_kernel<E, 4>);
        else if (n <= 8) go(gesv_wave_kernel<E, 8>);
        else if (n <= 12) go(gesv_wave_kernel<E, 12>);
        else go(gesv_wave_kernel<E, 16>);
        SBX_HIP_CHECK(hipGetLastError());
        return;
    }
    if (rm) throw Error("dense: internal error (row-major matrices need the wave kernels)");
    if (!keep_lu || a == b) throw Error("dense: internal error (in-place inversion needs the wave kernels)");
    if (io.x) throw Error("dense: internal error (separate right-hand sides need the wave kernels)");
    const bool lds = fits_lds<E>(n);
    hipLaunchKernelGGL(gesv_kernel<E>, dim3((unsigned)k), dim3(DTH),
                       lds ? (size_t)(n * n * sizeof(E)) : 0, s, (E *)a, n, (E *)b, m,
                       identity ? 1 : 0, alpha.re, alpha.im, lds ? 1 : 0, ipiv, info);
    SBX_HIP_CHECK(hipGetLastError());
}
template <typename E>
void trsm_typed(const void *a, long n, long k, void *x, long m, bool left, const Scalar &alpha,
                hipStream_t s) {
    if (n <= WNMAX && g_dense_wave >= 2) {
        const long per = 4 * (m <= 64 ? 64 / m : 1);
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned)((k + per - 1) / per)), dim3(256), 0, s, (const E *)a, (int)n,
                               k, (E *)x, m, left ? 1 : 0, alpha.re, alpha.im);
        };
        if (n <= 4) go(trsm_wave_kernel<E, 4>);
        else if (n <= 8) go(trsm_wave_kernel<E, 8>);
        else if (n <= 12) go(trsm_wave_kernel<E, 12>);
        else go(trsm_wave_kernel<E, 16>);
        SBX_HIP_CHECK(hipGetLastError());
        return;
    }
    const bool lds = fits_lds<E>(n);
    hipLaunchKernelGGL(trsm_kernel<E>, dim3((unsigned)k), dim3(DTH),
                       lds ? (size_t)(n * n * sizeof(E)) : 0, s, (const E *)a, n, (E *)x, m,
                       left ? 1 : 0, alpha.re, alpha.im, lds ? 1 : 0);
    SBX_HIP_CHECK(hipGetLastError());
}

/// res[0] <- the smallest matrix index with a nonzero info (res[0] starts at INT_MAX), and
/// res[1] <- that matrix's info by the thread that finds it when a single one is bad
__global__ void __launch_bounds__(256) first_bad_kernel(const int *info, long k, int *res) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < k; i += (long)gridDim.x * 256L)
        if (info[i] != 0) atomicMin(res, (int)i);
}

/// The calling thread's host-mapped failure flag (one per thread: every dense call synchronises
/// before it returns, so two calls never have it in flight together; kept for the thread's life)
volatile int *host_flag() {
    static thread_local int *flag = nullptr;
    if (!flag)
        SBX_HIP_CHECK(hipHostMalloc((void **)&flag, sizeof(int),
                                    hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent));
    return flag;
}
/// The info outputs of one launch over `v` (k ints), the flag cleared
InfoOut info_out(const Scratch &v) {
    volatile int *h = host_flag();
    *h = 0;
    int *dev = nullptr;
    SBX_HIP_CHECK(hipHostGetDevicePointer((void **)&dev, (void *)h, 0));
    return InfoOut{(int *)v.ptr, dev};
}

/// The first nonzero LAPACK info of the batch (synchronises the stream): with the host flag
/// clear, 0 at once; otherwise the index of the first failed matrix is found on the device, so
/// only 8 bytes cross to the host instead of the whole info array
int first_info(const int *info_d, long k, hipStream_t s, int device) {
    if (k >= 0x7fffffffL) throw Error("dense: too many matrices");
    SBX_HIP_CHECK(hipStreamSynchronize(s));
    if (*host_flag() == 0) return 0;
    Scratch res(sizeof(int), device);
    SBX_HIP_CHECK(hipMemsetAsync(res.ptr, 0x7f, sizeof(int), s));
    const long blocks = std::min((k + 255) / 256, 1024L);
    hipLaunchKernelGGL(first_bad_kernel, dim3((unsigned)blocks), dim3(256), 0, s, info_d, k, (int *)res.ptr);
    SBX_HIP_CHECK(hipGetLastError());
    int idx = 0;
    SBX_HIP_CHECK(hipMemcpyAsync(&idx, res.ptr, sizeof(int), hipMemcpyDeviceToHost, s));
    SBX_HIP_CHECK(hipStreamSynchronize(s));
    if (idx < 0 || idx >= k) return 0;
    int v = 0;
    SBX_HIP_CHECK(hipMemcpy(&v, info_d + idx, sizeof(int), hipMemcpyDeviceToHost));
    return v;
}

/// Calls f(E{}) with the element type of `t`
template <typename F> void dispatch(int t, F &&f) {
    switch (t) {
    case SBX_CDOUBLE: return f(double2{});
    case SBX_CFLOAT: return f(float2{});
    case SBX_DOUBLE: return f(double{});
    case SBX_FLOAT: return f(float{});
    default: throw Error("dense: unsupported type");
    }
}

} // namespace

bool dense_wave_rows(long n) { return n <= WNMAX && g_dense_wave; }

int launch_potrf(int t, void *a, long n, long k, int device, bool rm) {
    if (n == 0 || k == 0) return 0;
    if (k >= (1L << 31)) throw Error("dense: too many matrices");
    set_device(device);
    hipStream_t s = get_stream(device);
    Scratch info(sizeof(int) * k, device);
    const InfoOut iout = info_out(info);
    {
        KernelTimer timer("dense", s);
        dispatch(t, [&](auto z) { potrf_typed<decltype(z)>(a, n, k, iout, rm, s); });
    }
    return first_info((const int *)info.ptr, k, s, device);
}

int launch_gesv(int t, void *a, long n, long k, void *b, long m, bool identity,
                const Scalar &alpha, int device, bool rm, bool keep_lu) {
    if (n == 0 || k == 0) return 0;
    if (k >= (1L << 31)) throw Error("dense: too many matrices");
    set_device(device);
    hipStream_t s = get_stream(device);
    // (pivot indices only for the workgroup kernels: the wave kernels keep theirs in registers)
    Scratch info(sizeof(int) * k, device), ipiv(dense_wave_rows(n) ? 0 : sizeof(int) * k * n, device);
    const InfoOut iout = info_out(info);
    {
        KernelTimer timer("dense", s);
        dispatch(t, [&](auto z) {
            gesv_typed<decltype(z)>(a, n, k, b, m, identity, alpha, (int *)ipiv.ptr,
                                    iout, rm, keep_lu, s);
        });
    }
    return first_info((const int *)info.ptr, k, s, device);
}

bool trsm_io_fits(long n, long m) { return g_dense_wave >= 2 && n >= 1 && n <= WNMAX && m >= 1 && m <= 64; }

void launch_trsm_io(int t, const void *a, long n, long k, bool rm, const void *x, int xsi, int xst,
                    void *y, int ysi, int yst, long m, bool left, const Scalar &alpha, int device) {
    if (n == 0 || k == 0 || m == 0) return;
    if (!trsm_io_fits(n, m)) throw Error("dense: internal error (trsm_io shape)");
    if (k >= (1L << 31)) throw Error("dense: too many matrices");
    set_device(device);
    hipStream_t s = get_stream(device);
    KernelTimer timer("dense", s);
    dispatch(t, [&](auto z) {
        typedef decltype(z) E;
        const long per = 4 * (64 / m);
        auto go = [&](auto kern) {
            hipLaunchKernelGGL(kern, dim3((unsigned)((k + per - 1) / per)), dim3(256), 0, s, (const E *)a, (int)n, k,
                               rm ? 1 : 0, (const E *)x, xsi, xst, (E *)y, ysi, yst, (int)m, left ? 1 : 0,
                               alpha.re, alpha.im);
        };
        if (n <= 4) go(trsm_io_kernel<E, 4>);
        else if (n <= 8) go(trsm_io_kernel<E, 8>);
        else if (n <= 12) go(trsm_io_kernel<E, 12>);
        else go(trsm_io_kernel<E, 16>);
        SBX_HIP_CHECK(hipGetLastError());
    });
}

int launch_gesv_io(int t, const void *a, long n, long k, bool rm, const void *x, int xsi, int xst,
                   void *y, int ysi, int yst, long m, const Scalar &alpha, int device) {
    if (n == 0 || k == 0 || m == 0) return 0;
    if (!dense_wave_rows(n)) throw Error("dense: internal error (gesv_io shape)");
    if (k >= (1L << 31)) throw Error("dense: too many matrices");
    set_device(device);
    hipStream_t s = get_stream(device);
    Scratch info(sizeof(int) * k, device);
    const InfoOut iout = info_out(info);
    GesvIO io;
    io.x = x;
    io.xsi = xsi, io.xst = xst, io.ysi = ysi, io.yst = yst;
    {
        KernelTimer timer("dense", s);
        dispatch(t, [&](auto z) {
            gesv_typed<decltype(z)>(const_cast<void *>(a), n, k, y, m, false, alpha, nullptr, iout, rm,
                                    false, s, io);
        });
    }
    return first_info((const int *)info.ptr, k, s, device);
}

void launch_trsm(int t, const void *a, long n, long k, void *x, long m, bool left,
                 const Scalar &alpha, int device) {
    if (n == 0 || k == 0 || m == 0) return;
    if (k >= (1L << 31)) throw Error("dense: too many matrices");
    set_device(device);
    hipStream_t s = get_stream(device);
    KernelTimer timer("dense", s);
    dispatch(t, [&](auto z) { trsm_typed<decltype(z)>(a, n, k, x, m, left, alpha, s); });
}

} // namespace sbx
