// Internal declarations shared by the superbblas_amd HIP library.
//
// The library is the MI355X-native replacement of superbblas's distributed tensor
// contraction hot path (reference: include/superbblas/{dist,tensor,copy_n,blas,bsr}.h).
// Everything user-visible goes through the C-ABI declared in include/superbblas_amd/sbx.h;
// this header is private to the .so.
#pragma once

#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <complex>
#include <cstdint>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/superbblas_amd/sbx.h"

namespace sbx {

/// Error type; the C-ABI layer turns it into a status code + sbx_last_error()
struct Error : public std::runtime_error {
    explicit Error(const std::string &s) : std::runtime_error(s) {}
};

#define SBX_HIP_CHECK(expr)                                                                        \
    do {                                                                                           \
        hipError_t sbx_e_ = (expr);                                                                \
        if (sbx_e_ != hipSuccess)                                                                  \
            throw ::sbx::Error(std::string("HIP error `") + hipGetErrorString(sbx_e_) + "` at " +  \
                               __FILE__ + ":" + std::to_string(__LINE__) + " in " #expr);          \
    } while (0)

/// Size in bytes of a scalar type
inline std::size_t dtype_size(int t) {
    switch (t) {
    case SBX_FLOAT: return 4;
    case SBX_DOUBLE: return 8;
    case SBX_CFLOAT: return 8;
    case SBX_CDOUBLE: return 16;
    case SBX_INT: return 4;
    case SBX_SIZE_T: return 8;
    default: throw Error("unsupported dtype");
    }
}
inline bool dtype_is_complex(int t) { return t == SBX_CFLOAT || t == SBX_CDOUBLE; }

/// A complex scalar carried through the host planner (alpha/beta)
struct Scalar {
    double re = 0, im = 0;
    bool is_zero() const { return re == 0 && im == 0; }
    bool is_one() const { return re == 1 && im == 0; }
};

//
// Runtime (runtime.cpp)
//

/// Library stream of a device (created lazily, or set by the user with sbx_stream_set)
hipStream_t get_stream(int device);
/// Make `device` current for the calling thread
void set_device(int device);
/// Second library stream of a device (exchanges that overlap work on get_stream)
hipStream_t get_side_stream(int device);
/// Order: work enqueued later on `to` waits for the work enqueued so far on `from`
void stream_after(hipStream_t to, hipStream_t from);
/// While alive, get_stream(device) returns `s` (the library's work is redirected to it)
struct StreamOverride {
    int device;
    hipStream_t prev;
    bool prev_user;
    StreamOverride(int device, hipStream_t s);
    ~StreamOverride();
};
/// Stream-ordered scratch allocation (caching allocator over hipMalloc, see runtime.cpp)
void *scratch_alloc(std::size_t bytes, int device);
void scratch_free(void *p, int device);
/// Caller-provided allocator hooks (getCustomAllocator / getCustomDeallocator, platform.h:129-139):
/// device memory the library needs comes from `alloc` when set (nullptr -> the library's own)
typedef void *(*AllocHook)(unsigned long long bytes, int device, void *user);
typedef void (*FreeHook)(void *p, int device, void *user);
void set_alloc_hooks(AllocHook a, FreeHook f, void *user);
/// Device memory through the hooks or hipMalloc / hipFree (not cached)
void *device_alloc(std::size_t bytes, int device);
void device_free(void *p, int device);
/// Bytes held by the scratch cache of `device`: idle (cached) and in use (live)
void cache_usage(int device, std::size_t *cached, std::size_t *live);
/// Allocator tune keys (alloc.max_cached, alloc.cross_stream_frees): read into *get, write *set
void alloc_tune(const char *key, long long *get, const long long *set);

/// RAII scratch buffer on a device, freed in stream order
struct Scratch {
    void *ptr = nullptr;
    int device = -1;
    std::size_t bytes = 0;
    Scratch() {}
    Scratch(std::size_t bytes, int device);
    Scratch(const Scratch &) = delete;
    Scratch &operator=(const Scratch &) = delete;
    Scratch(Scratch &&o) noexcept : ptr(o.ptr), device(o.device), bytes(o.bytes) {
        o.ptr = nullptr;
    }
    Scratch &operator=(Scratch &&o) noexcept {
        std::swap(ptr, o.ptr);
        std::swap(device, o.device);
        std::swap(bytes, o.bytes);
        return *this;
    }
    ~Scratch();
};

/// Device id owning a pointer, or -1 for host memory
int pointer_device(const void *p);

/// Per-kernel-family GPU timers (the reference's reportTimings / resetTimings,
/// performance.h:356-518, measured with HIP events on the launching stream).  When enabled,
/// a KernelTimer around a launch records an event pair; timings_get() synchronizes and sums.
void timings_enable(bool on);
bool timings_enabled();
void timings_reset();
/// total milliseconds and number of launches of `name` (0 if never timed)
void timings_get(const char *name, double *ms, long long *calls);
/// "name calls total_ms" lines of every timed family
std::string timings_report();
/// Time only the named kernel families (comma-separated; null or empty: all)
void timings_filter(const char *names);
struct KernelTimer {
    const char *name;
    hipStream_t stream;
    void *ev0 = nullptr;
    KernelTimer(const char *name, hipStream_t s);
    ~KernelTimer();
};

//
// Kernels (kernels_*.hip); all enqueue on get_stream(device)
//

/// Strided batched GEMM, BLAS column-major semantics (reference blas.h:662-810):
///   C_b = alpha * op(A_b) * op(B_b) + beta * C_b,  b < batch.
/// Generalised to arbitrary strides: op(A)(i,k) = A[i*sa_m + k*sa_k + b*sa_b] (conjugated if
/// conja), op(B)(k,j) = B[k*sb_k + j*sb_n + b*sb_b] (conj if conjb), C(i,j) = C[i*sc_m + j*sc_n +
/// b*sc_b].  `t` is one of SBX_FLOAT/DOUBLE/CFLOAT/CDOUBLE.
struct GemmDesc {
    int t;
    long m, n, k, batch;
    const void *a;
    long sa_m, sa_k, sa_b;
    bool conja;
    const void *b;
    long sb_k, sb_n, sb_b;
    bool conjb;
    void *c;
    long sc_m, sc_n, sc_b;
    Scalar alpha, beta;
    // optional split label groups (two runs of memory each): index i of M is (i / m_lo, i % m_lo)
    // with strides (sa_m_hi, sa_m) in A and (sc_m_hi, sc_m) in C; likewise N and K.  0 (or the
    // full extent) = one run.
    long m_lo = 0, n_lo = 0, k_lo = 0;
    long sa_m_hi = 0, sa_k_hi = 0, sb_k_hi = 0, sb_n_hi = 0, sc_m_hi = 0, sc_n_hi = 0;
};
void launch_gemm(const GemmDesc &d, int device);

/// N-dimensional strided box copy (the MI355X version of copy_n / copy_n_blocking,
/// reference copy_n.h:77-244, 584-950):
///   dst[sum_i c_i*dst_stride_i] (=|+=) alpha * src[sum_i c_i*src_stride_i],  c < size
/// with element type conversion src_t -> dst_t.
struct BoxCopyDesc {
    int src_t, dst_t;
    const void *src;
    void *dst;
    std::vector<long> size, src_stride, dst_stride; // in elements
    Scalar alpha;
    bool add;
    // optional masks (MaskType = float, laid out like the data they mask, at the box origin):
    // an element is written only where both given masks are nonzero (tensor.h:1019-1027)
    const float *src_mask = nullptr, *dst_mask = nullptr;
};
void launch_box_copy(const BoxCopyDesc &d, int device);
/// Drop the prepared box-copy launches (clearCaches)
void clear_copy_launch_cache();
/// The box-copy kernel the planner picks for a box (no GPU work; tests of the host planner):
/// 0 masked, 1 contiguous, 2 direct gather, 3 LDS tile, 4 site-block transpose, 5 block
/// transpose (-1: empty box); *blocks = its grid size
int copy_kernel_plan(const BoxCopyDesc &d, long *blocks);

/// Launch tape of one copy() call: the box-copy launches it issued, so that a later call of the
/// same shape on other pointers replays them without planning (the C ABI's copy fast path;
/// the reference's plan caches, dist.h:2303-2353).  While a tape is set on the calling thread,
/// launch_box_copy appends to it; work that is not a plain box-copy launch (masks, peer copies)
/// marks it invalid.
struct TapeLaunch {
    std::shared_ptr<const void> launch; // the prepared launch (kernels_copy.hip)
    const void *src;                    // pointers and alpha as recorded
    void *dst;
    int device;
    Scalar alpha;
    // resolved by the recorder's owner: argument (0: origin, 1: destination), component, byte
    // offset; alpha_is_call: alpha is the call's alpha (else the recorded constant)
    int src_arg = -1, src_comp = -1, dst_arg = -1, dst_comp = -1;
    long src_off = 0, dst_off = 0;
    bool alpha_is_call = false;
};
struct CopyTape {
    std::vector<TapeLaunch> launches;
    bool valid = true;
};
void set_copy_tape(CopyTape *t);
CopyTape *current_copy_tape();
/// Issue a recorded launch on new pointers / alpha (library stream of its device)
void replay_launch(const TapeLaunch &l, const void *src, void *dst, const Scalar &alpha);
/// Drop the cached copy plans (dist.cpp; clearCaches)
void clear_copy_plan_cache();
/// Kernel-shape overrides for tuning runs (0 = the library's choice); set through sbx_tune_set
struct CopyTune {
    long budget = 0; ///< elements per LDS tile
    long run = 0;    ///< target elements of a tile row's contiguous source run
    int nt = 0;      ///< row-mapped kernel stores: 0 = non-temporal for large outputs, 1 = always, -1 = never
    long max_elems = 0; ///< elements per launch before a box is cut into slabs (0 = 2^31 - 1)
    int pair = 0;  ///< tiled kernel, 8-byte elements: two elements per lane access where the runs allow (-1 = never)
    int order = 0; ///< ... with pairs, the source chain first when the destination chain would take the
                   ///< source's contiguous dim (-1 = always the destination chain first)
    int trans = 0; ///< the site-block transpose kernel for the boxes it takes (-1 = never)
    int btrans = 0; ///< the block transpose kernel for the boxes it takes (-1 = never)
    std::atomic<int> last_pair{0}; ///< read-back ("copy.last_pair"): the last box-copy launch -- the tile
                                   ///< kernel's paired phases (1 reads, 2 writes), 4 = the site-block
                                   ///< transpose kernel (| 1, 2 for its paired phases), 8 = the block
                                   ///< transpose kernel (| 2), 0 any other kernel
};
extern CopyTune g_copy_tune;
struct GemmTune {
    int m3 = 0; ///< complex products on the matrix cores (GEMM LDS-DMA and 12x12 BSR kernels): > 0 the
               ///< 3-multiplication (Gauss) form, else the 4-multiplication form (the default: BLAS rounding)
    int splits = 0; ///< LDS-DMA kernel split-K factor (0 = the library's choice)
    long max_bytes = 0; ///< operand bytes per batch entry before a GEMM is cut (0 = 2^31 - 1)
    int t48 = 5; ///< 4- and 8-byte elements, 33..48 rows and columns: 48x48 tiles (0 = off; 1..4 the
                 ///< round-2 forms; 6 k-group workgroups; 13 / 14 / 16 wave rings of 4 waves
                 ///< 8-deep, 4 waves 16-deep, 16 waves 8-deep; any other value the library's
                 ///< choice: wave rings of 8 waves, 8-deep slabs, for a tensor contracted with
                 ///< itself, else k-group workgroups)
    int share_ab = 1; ///< LDS-DMA kernel: one slab image for A and B when they are the same memory (0 = off)
    int loaders = 8; ///< complex<double> 128x128 LDS-DMA kernel, K-major operands: only this many waves
                     ///< (4, 8, 16) issue the slab DMA (0 = every wave its share); config 2: 1.491 ->
                     ///< 1.475 ms at 4 or 8 (tools/studies/gemm_loaders.py, profiles/r05_gemm_loaders.txt)
    int dma_spread = 1; ///< ... the loader waves spread their DMA over this many k-steps (1 or 4); 0 (8
                        ///< loaders): the early barrier -- a slab's barrier before its last k-step,
                        ///< whose fragments are already read, the next slab's first ones read after it
    int dma_nt = 0;     ///< ... with the non-temporal policy (0 = the default policy)
    int skinny = 1; ///< outputs with a dimension of <= 4 (and <= 16 with a short k): the dot / rows
                    ///< kernels instead of MFMA tiles (0 = off)
    int clock = 0; ///< LDS-DMA kernel clock meter (gemm_clock_meter, kernels_gemm.hip; 0 = off)
    int dot_wgs = 256; ///< gemm_dot_kernel (m, n <= 4): split-K to about this many workgroups (1024 / 2048:
                       ///< no faster, m = n = 4 slower; profiles/r06_gemm_dot_wgs.txt)
    int frag_uk = 0;      ///< ... gemm_frag_kernel: k-steps of 4 per load group (2, 4 or 8; 0 = by shape)
    int frag_waves = 4096; ///< ... split-K to about this many waves
    int frag = 1;  ///< small outputs (m, n <= 32) and tall-skinny products on gemm_frag_kernel (MFMA
                   ///< fragments straight from global memory); 2 also for m, n <= 4; 0 = off
    int frag_small = 32; ///< ... small outputs: m, n up to this
    int frag_nt = 0; ///< ... 16 x 16 tiles per wave along n (1, 2 or 4; 0 = 2 for 17-32-column small outputs)
    int frag_pair = 1; ///< ... 8-byte elements: k pairs of a unit-k-stride operand as one 16-byte load
    int frag_tall = 0; ///< ... tall-skinny products: the short output dimension up to this (k <= 64;
                       ///< 0 = 48 for complex<float>, else 16)
};
/// The S3T checksum (storage.cpp; storage.h:701-731): CRC-32 (zlib polynomial) of the bytes, or
/// with blocksize > 0 the CRC of the CRCs of blocksize chunks (prev must then be 0)
uint32_t storage_checksum(const void *p, std::size_t bytes, std::size_t blocksize, uint32_t prev);
/// The LDS-DMA GEMM's clock meter of a device: {shader clock cycles, 100 MHz ticks, launches}
/// summed since the last reset (zeros when the meter was never enabled)
void gemm_clock_read(int device, unsigned long long out[3], bool reset);
extern GemmTune g_gemm_tune;
struct BsrTune {
    int variant = 0; ///< BSR kernels: 0 = the library's choice, 1 = the generic kernels only (no 9-point
                     ///< or block-staged specialisation), 2 = no 12x12 block-staged kernel
    long row_max_cols = 3;  ///< 9-point 3x3 operators: one thread per nonzero block up to this many rhs columns (0 = off)
    long split_max_cols = 32; ///< 9-point 3x3 complex<double> operators, row-major x: rows split over their
                              ///< nonzero blocks (bsr_ell9_split_kernel) from row_max_cols + 1 to this many
                              ///< rhs columns (0 = off)
    int split_cw = 0;  ///< ... rhs columns per thread (1 or 2; 0 = by the column count)
    int split_jb = 0;  ///< ... nonzero blocks per thread (3 or 9; 0 = by the column count)
    int split_ilv = 2; ///< ... an XCD's rows visited as this many interleaved parts
    int kron_mfma = 1;          ///< Kronecker 3x3 (color) x 4x4 (spin) complex<double>: spin products on the
                                ///< matrix cores (bsr_kron_mfma_kernel) ...
    long kron_mfma_min_cols = 8; ///< ... from this many rhs columns
    int kron_pack = 1;           ///< ... below 16 rhs columns: a wave's 16 column slots span several rows (0 = off)
    int kron_xlds = 1;           ///< ... x staged by LDS-DMA, a column's 4 spins as one 64-B piece, this many
                                 ///< neighbours ahead (0 = off: per-lane loads one ahead; 1..3)
    int kron_ylds = 0;           ///< ... with x staged: y written through the same ring in whole pieces
    int kron_spin = 0;           ///< ... spin first on the VALU, a lane per (row, column): 1 bsr_kron_spin_kernel
                                 ///< (spin rows of at most two nonzeros, operands by LDS-DMA), 2 bsr_kron_xor_kernel
                                 ///< (diagonal + XOR-partner spin rows, plain loads); 0 = the MFMA forms (the
                                 ///< default: n = 12 142 us against 180 / 190)
    long kron_spin_min_cols = 8; ///< ... from this many rhs columns (at least 8)
    int kron_order = 1;          ///< ... rows in the operator's XCD order (bsr.cpp build_kron_order)
    int blk_pd = 1; ///< 12x12 blocks by LDS-DMA: blocks in flight ahead of the one in use (1..3)
    int tile = 0;   ///< 9-point 3x3 complex<double> operators, row-major x and y: site tiles with
                    ///< their halo staged in LDS (bsr_ell9_tile_kernel) ... 1: 16-site tiles, slices
                    ///< of 8 rhs columns (opt-in: 16^4 n = 64 180 vs 169 us for the row-chunk kernel,
                    ///< DESIGN 5.3 round 5); 2: 8-site tiles, slices of 16 columns (no LDS bank
                    ///< conflicts whatever the slots, round 6)
    long tile_min_cols = 33; ///< ... from this many rhs columns (a multiple of 8, or 16 for tile 2)
    int nt = 11; ///< the value stream's LDS-DMA loads with the non-temporal (streaming) policy, per
                ///< kernel: 1 12x12 blocks by LDS-DMA, 2 3x3 row chunks, 4 3x3 split rows, 8 3x3 one
                ///< thread per block.  Default 1 | 2 | 8 (tools/bsr_bound.py NTS, warm, interleaved:
                ///< 12x12 complex<double> 340 -> 328 us, complex<float> 179 -> 168 us, 3x3 n = 64
                ///< 161 -> 158 us, n = 1 19.0 -> 18.2 us; the split-row kernel 34.4 -> 42.5 us: off)
    /// read-back ("bsr.last_kernel"; atomic: launches may come from several host threads): the form
    /// of the last launch -- 1 one thread per block (3x3), 2 split rows (3x3), 3 row chunks (3x3),
    /// 4 site tiles (3x3),
    /// 5 Kronecker on MFMA, 6 the same with packed column slots, 7 12x12 blocks by LDS-DMA, 8 the
    /// same with packed slots, 9 Kronecker spin first (VALU), 10 12x12 fragment gathers (9 blocks
    /// per row), 11 12x12 generic rows, 12 Kronecker spin first with XOR-partner spin rows,
    /// 13 site tiles of 8 sites and 16 columns (3x3),
    /// 0 another kernel
    std::atomic<int> last{0};
};
extern BsrTune g_bsr_tune;
/// dense solvers: matrices up to 16 x 16 packed 64 / n per wave -- 1: Cholesky and LU
/// (inversion, gesm), 2: the triangular solves too (the default); 0 = the workgroup-per-matrix
/// kernels
extern int g_dense_wave;

/// The LDS-DMA overrun class (39cd2bc): a DMA pass writes a whole row of 16-B lanes into LDS --
/// lanes past the data included, they write zeros -- so a launch needs dynamic LDS for every pass
/// it issues, not only for the data.  Each LDS-DMA launcher checks its size against the passes
/// its kernel's loop issues (recomputed here from the loop bounds, independently of the sizing).
inline void check_dma_lds(const char *kernel, size_t lds, long passes, long lanes_per_pass,
                   long extra_bytes = 0) {
    const long need = passes * lanes_per_pass * 16 + extra_bytes;
    if ((long)lds < need)
        throw Error(std::string("bsr: internal LDS sizing error in ") + kernel + ": " +
                    std::to_string(lds) + " bytes for DMA passes needing " + std::to_string(need));
}

/// Fill `n` elements of type `t` with zeros
void launch_zero(void *p, std::size_t bytes, int device);

/// Gather / scatter of runs through index vectors (reference copy_n_blocking, copy_n.h:584-1050):
///   dst[(dst_idx ? dst_idx[d] : d*blocking) + r] (=|+=) alpha * src[(src_idx ? src_idx[d] :
///   d*blocking) + r],  d < n, r < blocking; all pointers on `device`
struct IndexCopyDesc {
    int src_t, dst_t;
    const void *src;
    void *dst;
    const int *src_idx = nullptr, *dst_idx = nullptr;
    long n = 0, blocking = 1;
    Scalar alpha;
    bool add = false;
};
void launch_index_copy(const IndexCopyDesc &d, int device);

/// BSR SpMM on one component (reference bsr.h:535-650 builtin loop, bsr.h:855-928 GPU):
///   y[row-block i] = alpha * sum_{j in row i} V_j * x[jj_j],  for every rhs column
/// A site-tile schedule of a 3x3 9-point operator (bsr.cpp build_tile_schedule): per tile of up
/// to tt sites its block rows [chunks][tt] (-1: none), its distinct block columns [chunks][umax]
/// (-1: none) and the slot of each nonzero block among them [chunks][tt][9] (255: skip)
struct TileSched {
    const int *rows = nullptr, *uniq = nullptr;
    const unsigned char *loc = nullptr;
    int umax = 0, tt = 0;
    long chunks = 0;
};

struct BsrDesc {
    int t;
    long block_rows; ///< number of block rows
    int bi, bd;      ///< block image / domain sizes
    const int *ii;   ///< CSR row pointer (block_rows+1), device
    const int *jj;   ///< first domain index of each nonzero block (-1 = skip), device
    const void *v;   ///< nonzero blocks, bi*bd each
    bool block_im_fast;
    int num_nnz_per_row; ///< >0 if all rows have the same count (ELL), else -1
    const void *x;
    long ldx;
    long x_rows = 0; ///< domain rows of x (the component's domain volume)
    bool x_row_major; ///< x(d, col) = x[d*ldx + col] if row major, else x[d + col*ldx]
    void *y;
    long ldy;
    bool y_row_major;
    long ncols;
    Scalar alpha;
    bool add; ///< y += (instead of y =)
    // Kronecker BSR (bsr.h:587-621): kron != nullptr; x is (site, bd, ncols, kd) and y is
    // (block row, bi, ncols, ki), both row major; jj holds the domain site of each nonzero
    int ki = 1, kd = 1;
    const void *kron = nullptr; ///< num_nnz_per_row matrices of ki x kd
    const int *kron_perm = nullptr; ///< block row per row slot in the XCD order (nullptr: none)
    const void *kron_terms = nullptr; ///< spin rows as two terms (nullptr: a row has more nonzeros)
    const void *kron_xor = nullptr;   ///< spin rows as diagonal + XOR partner (nullptr: not of that form)
    // site tiles of 3x3 9-point operators (bsr.cpp build_tile_schedule): [0] 16-site tiles (the
    // 8-column kernel), [1] 8-site tiles (the 16-column kernel); rows == nullptr: none
    TileSched tiles[2];
};
void launch_bsr(const BsrDesc &d, int device);
void launch_bsr_kron(const BsrDesc &d, int device);
/// Dense batched solvers on k column-major n x n matrices (kernels_dense.hip; rm: row-major
/// matrices and right-hand sides, possible when dense_wave_rows(n)); the int results are the
/// first nonzero LAPACK info of the batch (0: success)
bool dense_wave_rows(long n);
int launch_potrf(int t, void *a, long n, long k, int device, bool rm = false);
/// LU + solve: B (n x m per matrix) <- alpha A^-1 B (identity: B starts as I); A gets the LU
/// (keep_lu = false: A is left as it was -- the wave kernels only, where B may be A itself: the
/// in-place inversion)
int launch_gesv(int t, void *a, long n, long k, void *b, long m, bool identity,
                const Scalar &alpha, int device, bool rm = false, bool keep_lu = true);
/// left: X (n x m) <- alpha U^-1 X;  right: X (m x n) <- alpha X U^-1  (U upper, non-unit)
void launch_trsm(int t, const void *a, long n, long k, void *x, long m, bool left,
                 const Scalar &alpha, int device);
/// The same from x into y (both k contiguous blocks of n x m elements; the lane vector's
/// component i of right-hand side t at i * si + t * st of a block), U row-major when rm: the
/// small-matrix form only, when trsm_io_fits(n, m)
bool trsm_io_fits(long n, long m);
/// gesm from x into y (same block conventions as launch_trsm_io), the LU of A (row-major when rm)
/// kept in the kernel: A is not written (dense_wave_rows(n) only); the first nonzero info
int launch_gesv_io(int t, const void *a, long n, long k, bool rm, const void *x, int xsi, int xst,
                   void *y, int ysi, int yst, long m, const Scalar &alpha, int device);
void launch_trsm_io(int t, const void *a, long n, long k, bool rm, const void *x, int xsi, int xst,
                    void *y, int ysi, int yst, long m, bool left, const Scalar &alpha, int device);
/// dst block q = (conj if conj_values) src block perm[q], q < nblocks, blocks of block_elems
void launch_gather_blocks(int t, const void *src, const int *perm, long nblocks, long block_elems,
                          bool conj_values, void *dst, int device);

} // namespace sbx
