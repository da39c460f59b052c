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
#include "sbx_internal.h"

#include <algorithm>

namespace sbx {
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
    void *y;
    long ldy;
    long ncols;
    double alpha_re, alpha_im;
    int add;
};

template <typename E> struct Ops;
template <> struct Ops<double2> {
    static __device__ __forceinline__ double2 zero() { return double2{0, 0}; }
    static __device__ __forceinline__ double2 fma(double2 a, double2 b, double2 c) {
        return double2{c.x + a.x * b.x - a.y * b.y, c.y + a.x * b.y + a.y * b.x};
    }
    static __device__ __forceinline__ double2 scale(double2 v, double ar, double ai) {
        return double2{ar * v.x - ai * v.y, ar * v.y + ai * v.x};
    }
    static __device__ __forceinline__ double2 add(double2 a, double2 b) {
        return double2{a.x + b.x, a.y + b.y};
    }
};
template <> struct Ops<float2> {
    static __device__ __forceinline__ float2 zero() { return float2{0, 0}; }
    static __device__ __forceinline__ float2 fma(float2 a, float2 b, float2 c) {
        return float2{c.x + a.x * b.x - a.y * b.y, c.y + a.x * b.y + a.y * b.x};
    }
    static __device__ __forceinline__ float2 scale(float2 v, double ar, double ai) {
        return float2{(float)ar * v.x - (float)ai * v.y, (float)ar * v.y + (float)ai * v.x};
    }
    static __device__ __forceinline__ float2 add(float2 a, float2 b) {
        return float2{a.x + b.x, a.y + b.y};
    }
};
template <> struct Ops<double> {
    static __device__ __forceinline__ double zero() { return 0; }
    static __device__ __forceinline__ double fma(double a, double b, double c) { return c + a * b; }
    static __device__ __forceinline__ double scale(double v, double ar, double) { return ar * v; }
    static __device__ __forceinline__ double add(double a, double b) { return a + b; }
};
template <> struct Ops<float> {
    static __device__ __forceinline__ float zero() { return 0; }
    static __device__ __forceinline__ float fma(float a, float b, float c) { return c + a * b; }
    static __device__ __forceinline__ float scale(float v, double ar, double) {
        return (float)ar * v;
    }
    static __device__ __forceinline__ float add(float a, float b) { return a + b; }
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

template <typename E, int BI, int BD>
void launch_layouts(const BsrArgs &a, bool yrow, bool xrow, long blocks, hipStream_t s) {
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

template <typename E> void launch_typed(const BsrArgs &a, bool yrow, bool xrow, hipStream_t s) {
    const long total = a.block_rows * a.bi * a.ncols;
    const long blocks = std::min((total + 255) / 256, 65536L);
    if (a.bi == 3 && a.bd == 3)
        launch_layouts<E, 3, 3>(a, yrow, xrow, blocks, s);
    else if (a.bi == 12 && a.bd == 12)
        launch_layouts<E, 12, 12>(a, yrow, xrow, blocks, s);
    else
        launch_layouts<E, 0, 0>(a, yrow, xrow, blocks, s);
}

} // namespace

void launch_bsr(const BsrDesc &d, int device) {
    if (d.block_rows == 0 || d.ncols == 0) return;
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
    a.y = d.y;
    a.ldy = d.ldy;
    a.ncols = d.ncols;
    a.alpha_re = d.alpha.re;
    a.alpha_im = d.alpha.im;
    a.add = d.add ? 1 : 0;
    switch (d.t) {
    case SBX_CDOUBLE: return launch_typed<double2>(a, d.y_row_major, d.x_row_major, s);
    case SBX_CFLOAT: return launch_typed<float2>(a, d.y_row_major, d.x_row_major, s);
    case SBX_DOUBLE: return launch_typed<double>(a, d.y_row_major, d.x_row_major, s);
    case SBX_FLOAT: return launch_typed<float>(a, d.y_row_major, d.x_row_major, s);
    default: throw Error("bsr: unsupported type");
    }
}

} // namespace sbx
