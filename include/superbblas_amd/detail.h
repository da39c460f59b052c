/*
 * detail.h -- the `superbblas::detail` surface of the drop-in header.
 *
 * The reference's tests and the lattice codes written against superbblas reach past the public
 * API into `superbblas::detail` for a handful of helpers: the device-tagged `vector<T, XPU>`, the
 * `Cpu` / `Gpu` contexts, the coordinate algebra (volume, strides, index <-> coordinate, periodic
 * normalisation and intersection, label permutations), the low-level copies (copy_n, zero_n,
 * copy_n_blocking with index vectors, makeSure) and the strided batched GEMM
 * (xgemm_batch_strided).  This header provides them with the reference's names and argument
 * meaning (cited per item) over the C ABI, so that code such as the reference's tests/bsr.cpp,
 * contract.cpp, dist.cpp and blas.cpp compiles unchanged against include/superbblas.h and runs
 * on libsuperbblas_amd.so.
 *
 * Design (MI355X-first, not the reference's):
 *  - `Gpu` (= `Hip`) is a device id; all work of a device goes to the library's stream of that
 *    device (sbx_stream_get), so a context carries no streams.  `device == CPU_DEVICE_ID` with a
 *    `backup_device` is pinned host memory ordered by that device (the reference's
 *    toCpuPinned(), platform.h:213-216).
 *  - Device memory comes from sbx_allocate (hipMalloc or the custom allocator hooks), pinned host
 *    memory from sbx_allocate on a CPU context (hipHostMalloc), plain host memory from operator
 *    new.  `vector` is a shared handle (operator= aliases), as the reference's (blas.h:236-358).
 *  - Every copy with a scale factor, a type conversion or index vectors runs as a HIP kernel
 *    (sbx_copy_n_blocking); host operands are mirrored through device scratch.  A host
 *    destination is complete when the call returns.
 *  - The integer algebra (intersection) is the library's own (plan.cpp), the one the
 *    distributed copies use, pinned against the reference's known answers.
 */
#ifndef SUPERBBLAS_AMD_DETAIL_H
#define SUPERBBLAS_AMD_DETAIL_H

#include <chrono>
#include <cstring>
#include <memory>
#include <new>
#include <sstream>
#include <type_traits>
#include <utility>

namespace superbblas {
namespace detail {

// ---- contexts (platform.h:171-260) ----

/// Host context (platform.h:173-184)
struct Cpu {
    Session session;
    Cpu(const Session &session = 0) : session(session) {}
    Cpu toCpu() const { return *this; }
    Cpu toCpuPinned() const { return *this; }
};

/// GPU context (platform.h:186-221): a device, or pinned host memory (device == CPU_DEVICE_ID)
/// ordered by `backup_device`
struct Hip {
    int device;
    int backup_device;
    Session session;
    Hip(int device = 0, int backup_device = -2, Session session = 0)
        : device(device), backup_device(backup_device == -2 ? device : backup_device),
          session(session) {}
    Cpu toCpu() const { return Cpu{session}; }
    Hip toCpuPinned() const {
        return Hip{CPU_DEVICE_ID, device == CPU_DEVICE_ID ? backup_device : device, session};
    }
};
using Gpu = Hip;

inline int deviceId(const Cpu &) { return CPU_DEVICE_ID; }
inline int deviceId(const Hip &xpu) { return xpu.device; }
inline int backupDeviceId(const Cpu &) { return CPU_DEVICE_ID; }
inline int backupDeviceId(const Hip &xpu) {
    return xpu.device == CPU_DEVICE_ID ? xpu.backup_device : xpu.device;
}

/// The C-ABI context of a low-level context: host memory or a device
inline sbx_context abi_context(const Cpu &) { return sbx_context{SBX_CPU, -1}; }
inline sbx_context abi_context(const Hip &xpu) {
    return xpu.device == CPU_DEVICE_ID ? sbx_context{SBX_CPU, -1}
                                       : sbx_context{SBX_GPU, xpu.device};
}

/// Wait for the work queued on a context (blas.h:965-974)
inline void sync(const Cpu &) {}
inline void sync(const Hip &xpu) {
    const int d = backupDeviceId(xpu);
    if (d >= 0) sbx_detail::check(sbx_sync(sbx_context{SBX_GPU, d}));
}

/// Wall-clock seconds (performance.h:228-236)
inline double w_time() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

/// Throw std::runtime_error (platform.h:718-753)
[[noreturn]] inline void gen_error(const std::string &s) { throw std::runtime_error(s); }

// ---- element-wise operation tags (blas.h:423-429) ----

namespace EWOp {
struct Copy {};
struct Add {};
} // namespace EWOp

inline int ewop_code(EWOp::Copy) { return SBX_COPY; }
inline int ewop_code(EWOp::Add) { return SBX_ADD; }

// ---- memory ----

namespace mem {
inline std::shared_ptr<char> bytes(std::size_t n, const Cpu &) {
    if (n == 0) return {};
    return std::shared_ptr<char>((char *)::operator new(n), [](char *p) { ::operator delete(p); });
}
inline std::shared_ptr<char> bytes(std::size_t n, const Hip &xpu) {
    if (n == 0) return {};
    const sbx_context c = abi_context(xpu);
    void *p = nullptr;
    sbx_detail::check(sbx_allocate((unsigned long long)n, c, &p));
    return std::shared_ptr<char>((char *)p, [c](char *q) { (void)sbx_deallocate(q, c); });
}
} // namespace mem

/// Array of `n` elements on a context; copies alias the same memory (blas.h:236-358).  Memory is
/// uninitialised.
template <typename T, typename XPU> struct vector {
    using T_no_const = typename std::remove_const<T>::type;
    using iterator = T *;

    vector() : vector(0, XPU{}) {}
    vector(std::size_t n, XPU xpu_) : n(n), xpu(xpu_) {
        ptr = mem::bytes(n * sizeof(T), xpu);
        ptr_aligned = (T *)ptr.get();
    }
    /// Alias of caller memory, never freed (blas.h:266-269)
    vector(std::size_t n, T *p, XPU xpu) : n(n), ptr_aligned(p), ptr(), xpu(xpu) {}
    vector(std::size_t n, T *p_aligned, std::shared_ptr<char> p, XPU xpu)
        : n(n), ptr_aligned(p_aligned), ptr(std::move(p)), xpu(xpu) {}
    /// vector<T> -> vector<const T>
    template <typename U = T_no_const,
              typename std::enable_if<!std::is_const<U>::value && std::is_const<T>::value &&
                                          std::is_same<const U, T>::value,
                                      bool>::type = true>
    vector(const vector<U, XPU> &v) : vector{v.n, (T *)v.ptr_aligned, v.ptr, v.xpu} {}

    void clear() {
        n = 0;
        ptr.reset();
        ptr_aligned = nullptr;
    }
    std::size_t size() const { return n; }
    T *data() const { return ptr_aligned; }
    T *begin() const { return ptr_aligned; }
    T *end() const { return ptr_aligned + n; }
    XPU ctx() const { return xpu; }
    /// Shrink (blas.h:304-308)
    void resize(std::size_t new_n) {
        if (new_n > n) throw std::runtime_error("Unsupported operation");
        n = new_n;
    }
    template <typename U = XPU, typename std::enable_if<std::is_same<U, Cpu>::value, bool>::type = true>
    const T &operator[](std::size_t i) const {
        return ptr_aligned[i];
    }
    template <typename U = XPU, typename std::enable_if<std::is_same<U, Cpu>::value, bool>::type = true>
    T &operator[](std::size_t i) {
        return ptr_aligned[i];
    }
    template <typename U = XPU, typename std::enable_if<std::is_same<U, Cpu>::value, bool>::type = true>
    const T &back() const {
        return ptr_aligned[n - 1];
    }
    template <typename U = XPU, typename std::enable_if<std::is_same<U, Cpu>::value, bool>::type = true>
    bool operator==(const vector<T, U> &v) const {
        if (n != v.size()) return false;
        for (std::size_t i = 0; i < n; ++i)
            if (!(ptr_aligned[i] == v.ptr_aligned[i])) return false;
        return true;
    }
    template <typename U = XPU, typename std::enable_if<std::is_same<U, Cpu>::value, bool>::type = true>
    bool operator!=(const vector<T, U> &v) const {
        return !operator==(v);
    }
    vector withNewContext(const XPU &new_xpu) const { return vector{n, ptr_aligned, ptr, new_xpu}; }

    std::size_t n;
    T *ptr_aligned = nullptr;
    std::shared_ptr<char> ptr;
    XPU xpu;
};

template <typename T> vector<T, Cpu> to_vector(T *ptr, std::size_t n, Cpu cpu) {
    return vector<T, Cpu>(ptr ? n : 0, ptr, cpu);
}
template <typename T> vector<T, Hip> to_vector(T *ptr, std::size_t n, Hip xpu) {
    return vector<T, Hip>(ptr ? n : 0, ptr, xpu);
}

/// Index vectors (tensor.h:89-90)
template <typename XPU> using Indices = vector<IndexType, XPU>;

/// v[0..n) -> w[0..n), any pair of contexts (blas.h:163-231)
template <typename T, typename XPU0, typename XPU1>
void copy_n(const T *v, XPU0 xpu0, std::size_t n, T *w, XPU1 xpu1) {
    if (n == 0 || v == w) return;
    sbx_detail::check(sbx_memcpy((void *)w, abi_context(xpu1), (const void *)v, abi_context(xpu0),
                                 (unsigned long long)(n * sizeof(T))));
}

/// v[0..n) = 0 (blas.h:431-490)
template <typename T, typename XPU> void zero_n(T *v, std::size_t n, const XPU &xpu) {
    if (n == 0) return;
    sbx_detail::check(
        sbx_memset_zero((void *)v, abi_context(xpu), (unsigned long long)(n * sizeof(T))));
}

namespace copy_detail {
template <typename XPU> sbx_context index_context(const void *idx, const XPU &xpu) {
    return idx ? abi_context(xpu) : sbx_context{SBX_CPU, -1};
}
} // namespace copy_detail

/// w[iw[d] + r] (=|+=) alpha * v[iv[d] + r] for d < n, r < blocking; a null index vector is
/// d * blocking (copy_n.h:1028-1050)
template <typename IndexType_, typename T, typename Q, typename XPUV, typename XPUIV,
          typename XPUW, typename XPUIW, typename EWOP>
void copy_n_blocking(typename elem<T>::type alpha, const T *v, const XPUV &xpuv,
                     IndexType_ blocking, const IndexType_ *indicesv, const XPUIV &xpuiv,
                     IndexType_ n, Q *w, const XPUW &xpuw, const IndexType_ *indicesw,
                     const XPUIW &xpuiw, EWOP) {
    static_assert(sizeof(IndexType_) == sizeof(int), "copy_n: 32-bit index vectors");
    if (n == 0 || blocking == 0) return;
    const auto a = sbx_detail::scalar(alpha);
    sbx_detail::check(sbx_copy_n_blocking(
        a.data(), sbx_detail::dtype<typename std::remove_const<T>::type>::value, (const void *)v,
        abi_context(xpuv), (long long)blocking, (const int *)indicesv,
        copy_detail::index_context(indicesv, xpuiv), (long long)n,
        sbx_detail::dtype<Q>::value, (void *)w, abi_context(xpuw), (const int *)indicesw,
        copy_detail::index_context(indicesw, xpuiw), ewop_code(EWOP{})));
}

/// w[iw[d]] (=|+=) alpha * v[iv[d]] for d < n (copy_n.h:540-583)
template <typename IndexType_, typename T, typename Q, typename XPUV, typename XPUIV,
          typename XPUW, typename XPUIW, typename EWOP>
void copy_n(typename elem<T>::type alpha, const T *v, const XPUV &xpuv,
            const IndexType_ *indicesv, const XPUIV &xpuiv, IndexType_ n, Q *w, const XPUW &xpuw,
            const IndexType_ *indicesw, const XPUIW &xpuiw, EWOP) {
    copy_n_blocking<IndexType_>(alpha, v, xpuv, IndexType_(1), indicesv, xpuiv, n, w, xpuw,
                                indicesw, xpuiw, EWOP{});
}

/// w[0..n) (=|+=) alpha * v[0..n) (copy_n.h:572-583)
template <typename IndexType_, typename T, typename Q, typename XPUV, typename XPUW, typename EWOP>
void copy_n(typename elem<T>::type alpha, const T *v, const XPUV &xpuv, IndexType_ n, Q *w,
            const XPUW &xpuw, EWOP) {
    copy_n_blocking<IndexType_>(alpha, v, xpuv, IndexType_(1), (const IndexType_ *)nullptr, xpuv,
                                n, w, xpuw, (const IndexType_ *)nullptr, xpuw, EWOP{});
}

/// The vector itself when it already lives on `xpu`'s device, else a copy there (blas.h:813-844)
template <typename T, typename XPU> vector<T, XPU> makeSure(const vector<T, XPU> &v, XPU xpu) {
    if (deviceId(v.ctx()) == deviceId(xpu)) return v;
    vector<T, XPU> r(v.size(), xpu);
    copy_n(v.data(), v.ctx(), v.size(), r.data(), r.ctx());
    return r;
}
template <typename T, typename XPU1, typename XPU0,
          typename std::enable_if<!std::is_same<XPU0, XPU1>::value, bool>::type = true>
vector<T, XPU1> makeSure(const vector<T, XPU0> &v, XPU1 xpu1) {
    vector<T, XPU1> r(v.size(), xpu1);
    copy_n(v.data(), v.ctx(), v.size(), r.data(), r.ctx());
    return r;
}

/// A new vector with the same content (blas.h:492-505)
template <typename T, typename XPU> vector<T, XPU> clone(const vector<T, XPU> &v) {
    vector<T, XPU> r(v.size(), v.ctx());
    copy_n(v.data(), v.ctx(), v.size(), r.data(), r.ctx());
    return r;
}

// ---- strided batched GEMM (blas.h:662-810; blas_cpu_tmpl.hpp:376-478) ----

/// C_b = alpha op(A_b) op(B_b) + beta C_b, column major, b < batch_size; trans in {N,T,C} (either
/// case).  On the FP64/FP32 matrix cores (kernels_gemm.hip); host operands are mirrored.
template <typename T, typename XPU>
void xgemm_batch_strided(char transa, char transb, int m, int n, int k, T alpha, const T *a,
                         int lda, int stridea, const T *b, int ldb, int strideb, T beta, T *c,
                         int ldc, int stridec, int batch_size, XPU xpu) {
    if (m == 0 || n == 0 || batch_size == 0) return;
    const auto al = sbx_detail::scalar(alpha), be = sbx_detail::scalar(beta);
    sbx_detail::check(sbx_xgemm_batch_strided_ctx(
        sbx_detail::dtype<T>::value, transa, transb, m, n, k, al.data(), (const void *)a, lda,
        stridea, (const void *)b, ldb, strideb, be.data(), (void *)c, ldc, stridec, batch_size,
        abi_context(xpu)));
}

// ---- coordinates (tensor.h:137-480, dist.h:78-560) ----

template <typename T, std::size_t N>
std::array<T, N> operator+(const std::array<T, N> &a, const std::array<T, N> &b) {
    std::array<T, N> r;
    for (std::size_t i = 0; i < N; ++i) r[i] = a[i] + b[i];
    return r;
}
template <typename T, std::size_t N>
std::array<T, N> operator-(const std::array<T, N> &a, const std::array<T, N> &b) {
    std::array<T, N> r;
    for (std::size_t i = 0; i < N; ++i) r[i] = a[i] - b[i];
    return r;
}
template <typename T, std::size_t N>
std::array<T, N> &operator+=(std::array<T, N> &a, const std::array<T, N> &b) {
    for (std::size_t i = 0; i < N; ++i) a[i] += b[i];
    return a;
}
template <typename T, std::size_t N> std::array<T, N> operator*(T a, const std::array<T, N> &b) {
    std::array<T, N> r;
    for (std::size_t i = 0; i < N; ++i) r[i] = a * b[i];
    return r;
}

/// Ranges: {from, size} (dist.h:78-82)
template <std::size_t N> using From_size_item = PartitionItem<N>;
template <std::size_t N> using From_size = std::vector<From_size_item<N>>;

/// Product of the dimensions (tensor.h:382-389); 0 for a rank-0 coordinate
template <std::size_t Nd, typename Idx> std::size_t volume(const Coor<Nd, Idx> &dim) {
    if (Nd == 0) return 0;
    std::size_t v = 1;
    for (std::size_t i = 0; i < Nd; ++i) v *= (std::size_t)dim[i];
    return v;
}
/// Total volume of a list of ranges (dist.h:320-324)
template <std::size_t Nd> std::size_t volume(const From_size<Nd> &fs) {
    std::size_t v = 0;
    for (const auto &r : fs) v += volume(r[1]);
    return v;
}

/// Jump to the next element of each dimension (tensor.h:279-299)
template <typename SIdx, std::size_t Nd, typename CIdx>
Coor<Nd, SIdx> get_strides(const Coor<Nd, CIdx> dim, CoorOrder co) {
    Coor<Nd, SIdx> s{};
    if (Nd == 0) return s;
    if (co == SlowToFast) {
        s[Nd - 1] = 1;
        for (std::size_t i = Nd - 1; i > 0; --i) s[i - 1] = s[i] * (SIdx)dim[i];
    } else {
        s[0] = 1;
        for (std::size_t i = 1; i < Nd; ++i) s[i] = s[i - 1] * (SIdx)dim[i - 1];
    }
    return s;
}

/// Linear index of a (periodic) coordinate (tensor.h:301-311)
template <std::size_t Nd, typename CIdx, typename SIdx>
SIdx coor2index(const Coor<Nd, CIdx> &coor, const Coor<Nd, CIdx> &dim,
                const Coor<Nd, SIdx> &stride) {
    SIdx r = 0;
    for (std::size_t j = 0; j < Nd; ++j) r += (SIdx)(coor[j] % dim[j]) * stride[j];
    return r;
}

/// Coordinate of a linear index (tensor.h:331-340)
template <std::size_t Nd, typename CIdx, typename SIdx>
Coor<Nd, CIdx> index2coor(const SIdx &index, const Coor<Nd, CIdx> &dim,
                          const Coor<Nd, SIdx> &stride) {
    Coor<Nd, CIdx> r;
    for (std::size_t j = 0; j < Nd; ++j) r[j] = (CIdx)((index / stride[j]) % (SIdx)dim[j]);
    return r;
}

/// coor mod dim into [0, dim) (dist.h:326-343)
inline IndexType normalize_coor(IndexType coor, IndexType dim) {
    if (dim == 0) return 0;
    const IndexType r = coor % dim;
    return r < 0 ? r + dim : r;
}
template <std::size_t Nd> Coor<Nd> normalize_coor(const Coor<Nd> &coor, const Coor<Nd> &dim) {
    Coor<Nd> r;
    for (std::size_t j = 0; j < Nd; ++j) r[j] = normalize_coor(coor[j], dim[j]);
    return r;
}

/// An array of Nd elements from a string of exactly Nd characters (tensor.h:262-277)
template <std::size_t Nd, typename T> std::array<T, Nd> toArray(const T *v, const char *name) {
    if ((v == nullptr && Nd > 0) || (v != nullptr && std::strlen(v) != Nd)) {
        std::stringstream ss;
        ss << "The length of the order should match the template argument; argument `" << name
           << "` should have length " << Nd;
        throw std::runtime_error(ss.str());
    }
    std::array<T, Nd> r{};
    for (std::size_t i = 0; i < Nd; ++i) r[i] = v[i];
    return r;
}

/// r[i] = coor[perm[i]], or `blank` where perm[i] < 0 (tensor.h:411-422)
template <std::size_t Nd0, std::size_t Nd1>
Coor<Nd1> reorder_coor(const Coor<Nd0> &coor, const Coor<Nd1> &perm, IndexType blank = 0) {
    Coor<Nd1> r;
    for (std::size_t i = 0; i < Nd1; ++i) r[i] = perm[i] >= 0 ? coor[perm[i]] : blank;
    return r;
}

/// Position in o0 of each label of o1, -1 when absent (tensor.h:464-478)
template <std::size_t Nd0, std::size_t Nd1>
Coor<Nd1> find_permutation(const Order<Nd0> &o0, const Order<Nd1> &o1) {
    Coor<Nd1> r;
    for (std::size_t i = 0; i < Nd1; ++i) {
        r[i] = -1;
        for (std::size_t j = 0; j < Nd0; ++j)
            if (o0[j] == o1[i]) {
                r[i] = (IndexType)j;
                break;
            }
    }
    return r;
}

/// Which range to return when two ranges cover a whole dimension (dist.h:361-363)
enum IntersectionDominant { FirstIntervalIsDominant, SecondIntervalIsDominant };

namespace range_detail {
/// All pieces of the intersection of two periodic ranges, first dimension fastest
template <std::size_t Nd>
From_size<Nd> pieces(const Coor<Nd> &from0, const Coor<Nd> &size0, const Coor<Nd> &from1,
                     const Coor<Nd> &size1, const Coor<Nd> &dim, IntersectionDominant d) {
    // full-support dimensions of both ranges: the dominant range's interval
    Coor<Nd> f0 = from0, s0 = size0, f1 = from1, s1 = size1;
    if (d == SecondIntervalIsDominant) {
        for (std::size_t i = 0; i < Nd; ++i)
            if (size0[i] == dim[i] && size1[i] == dim[i]) f0[i] = from1[i];
    }
    std::size_t cap = 1;
    for (std::size_t i = 0; i < Nd; ++i) cap *= 3;
    From_size<Nd> r(cap);
    int n = 0;
    sbx_detail::check(sbx_intersection((int)Nd, f0.data(), s0.data(), f1.data(), s1.data(),
                                       dim.data(), (int)cap, reinterpret_cast<int *>(r.data()),
                                       &n));
    r.resize(n);
    return r;
}
} // namespace range_detail

/// The intersection of two periodic ranges as one range (dist.h:425-451)
template <std::size_t Nd>
void intersection(const Coor<Nd> &from0, const Coor<Nd> &size0, const Coor<Nd> &from1,
                  const Coor<Nd> &size1, const Coor<Nd> &dim, Coor<Nd> &fromr, Coor<Nd> &sizer,
                  IntersectionDominant d = FirstIntervalIsDominant) {
    const From_size<Nd> r = range_detail::pieces(from0, size0, from1, size1, dim, d);
    if (r.empty()) {
        fromr = Coor<Nd>{{}};
        sizer = Coor<Nd>{{}};
    } else if (r.size() == 1) {
        fromr = r[0][0];
        sizer = r[0][1];
    } else {
        throw std::runtime_error("Not supported complex overlap of intervals");
    }
}

/// Every piece of the intersection of two periodic ranges (dist.h:453-486)
template <std::size_t Nd>
From_size<Nd> intersection(const Coor<Nd> &from0, const Coor<Nd> &size0, const Coor<Nd> &from1,
                           const Coor<Nd> &size1, const Coor<Nd> &dim,
                           IntersectionDominant d = FirstIntervalIsDominant) {
    return range_detail::pieces(from0, size0, from1, size1, dim, d);
}

/// Pieces of the intersection of each range of a list with a range (dist.h:488-522)
template <std::size_t Nd>
From_size<Nd> intersection(const From_size<Nd> &fs0, const Coor<Nd> &from1, const Coor<Nd> &size1,
                           const Coor<Nd> &dim, IntersectionDominant d = FirstIntervalIsDominant) {
    From_size<Nd> r;
    for (const auto &a : fs0) {
        const From_size<Nd> x = range_detail::pieces(a[0], a[1], from1, size1, dim, d);
        r.insert(r.end(), x.begin(), x.end());
    }
    return r;
}

/// Pieces of the intersections of every pair of ranges of two lists (dist.h:524-558)
template <std::size_t Nd>
From_size<Nd> intersection(const From_size<Nd> &fs0, const From_size<Nd> fs1, const Coor<Nd> &dim,
                           IntersectionDominant d = FirstIntervalIsDominant) {
    From_size<Nd> r;
    for (const auto &a : fs0)
        for (const auto &b : fs1) {
            const From_size<Nd> x = range_detail::pieces(a[0], a[1], b[0], b[1], dim, d);
            r.insert(r.end(), x.begin(), x.end());
        }
    return r;
}

} // namespace detail

// ---- Context -> low-level context (platform.h:765-773) ----

inline detail::Cpu Context::toCpu(Session session) const { return detail::Cpu{session}; }
inline detail::Gpu Context::toGpu(Session session) const {
    return plat == CPU ? detail::Gpu{CPU_DEVICE_ID, 0, session} : detail::Gpu{device, device, session};
}

} // namespace superbblas

#endif // SUPERBBLAS_AMD_DETAIL_H
