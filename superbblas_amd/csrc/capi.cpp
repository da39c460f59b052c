// extern "C" entry points (include/superbblas_amd/sbx.h).
//
// Converts the flat C descriptors into the planner's DistTensor form (SlowToFast internally),
// mirrors host (CPU-context) components through device scratch so that every data movement
// and every flop runs on the GPU, and turns C++ exceptions into status codes.
#include "plan.h"
#include <atomic>
#include <algorithm>
#include <functional>
#include <memory>
#include <unordered_map>

#include <rccl/rccl.h>

#include <cstdlib>
#include <cstring>
#include <mutex>

namespace sbx {
BsrOp *bsr_create(int nd, int ni, int dtype, const std::vector<std::vector<Range>> &pi,
                  const Coor &dimi, const std::vector<std::vector<Range>> &pd, const Coor &dimd,
                  const Coor &blocki, const Coor &blockd, bool block_im_fast,
                  const std::vector<const int *> &ii, const std::vector<const int *> &jj,
                  const std::vector<const void *> &v, const std::vector<int> &devs, bool reverse_jj,
                  const Comm &comm, const Coor *kroni = nullptr, const Coor *krond = nullptr,
                  const std::vector<const void *> *kronv = nullptr);
void bsr_destroy(BsrOp *op);
void bsr_krylov(const BsrOp &op, const Scalar &alpha, const std::string &oi,
                const std::string &od, const DistTensor &x, const Coor &fromx, const Coor &sizex,
                const Scalar &beta, const DistTensor &y, const Coor &fromy, const Coor &sizey,
                char okr, const Comm &comm, bool just_local = false,
                std::function<void()> *deferred = nullptr);
void set_user_stream(int device, hipStream_t s, bool has_user);
void destroy_streams();
void trim_pools();
} // namespace sbx

struct sbx_comm_s {
    sbx::Comm c;
    std::unique_ptr<sbx::HostStage> stage;
};
struct sbx_bsr_s {
    sbx::BsrOp *op = nullptr;
    int co = SBX_SLOW_TO_FAST;
    int nd = 0, ni = 0, dtype = 0;
    bool is_kron = false;
};

struct sbx_storage_s {
    sbx::StorageCtx *s = nullptr;
    int dtype = SBX_CDOUBLE;
    int nd = 0;
};

using namespace sbx;

namespace {

/// Device of the last host-context detail call (tune key "detail.last_device", for the tests)
std::atomic<int> g_detail_last_device{-1};

/// The calling thread's current device.  A detail call whose operands are all host memory runs
/// there (the reference runs such calls on the CPU of the calling rank, platform.h:757-816; here
/// they are mirrored through the GPU the caller selected, as pick_device does for the main path
/// through the communicator's device, and never silently on device 0)
int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0) d = 0;
    return d;
}

thread_local std::string g_last_error;

template <typename F> int guard(F &&f) {
    try {
        f();
        return SBX_OK;
    } catch (const std::exception &e) {
        g_last_error = e.what();
    } catch (...) {
        g_last_error = "unknown error";
    }
    return SBX_ERROR;
}

Coor to_coor(const int *p, int n, bool rev) {
    Coor c(n);
    for (int i = 0; i < n; ++i) c[i] = p ? p[rev ? n - 1 - i : i] : 0;
    return c;
}

/// Row / column label subsets of the dense solvers (reversed with the tensor for FastToSlow)
std::string sub_labels(const char *s, bool rev, const char *what) {
    if (!s) throw Error(std::string(what) + ": null labels");
    std::string r(s);
    if (rev) std::reverse(r.begin(), r.end());
    return r;
}

std::string to_labels(const char *o, int n, bool rev, const char *what) {
    if (!o) throw Error(std::string(what) + ": null labels");
    if ((int)std::strlen(o) != n)
        throw Error(std::string("the length of `") + what +
                    "` doesn't match the template parameter");
    std::string s(o, n);
    if (rev) std::reverse(s.begin(), s.end());
    for (int i = 0; i < n; ++i)
        for (int j = i + 1; j < n; ++j)
            if (s[i] == s[j]) throw Error(std::string(what) + " has repeated labels");
    return s;
}

Comm get_comm(sbx_comm c) { return c ? c->c : Comm{}; }

/// Partition array -> ranges per rank (dist.h:3251-3261)
std::vector<std::vector<Range>> to_ranges(const int *p, int nd, int ncomponents, const Comm &comm,
                                          bool rev) {
    if (!p) throw Error("null partition");
    if (ncomponents < 1) throw Error("invalid number of components");
    std::vector<std::vector<Range>> r(comm.nprocs);
    for (int rk = 0; rk < comm.nprocs; ++rk)
        for (int c = 0; c < ncomponents; ++c) {
            const int *item = p + (std::size_t)(rk * ncomponents + c) * 2 * nd;
            Range x{to_coor(item, nd, rev), to_coor(item + nd, nd, rev)};
            if (volume(x.size) == 0) {
                x.from.assign(nd, 0);
                x.size.assign(nd, 0);
            }
            r[rk].push_back(x);
        }
    return r;
}

/// Host components are mirrored through device scratch; this keeps the record to copy back
struct Mirror {
    std::vector<Scratch> bufs;
    struct Back {
        void *host;
        void *dev;
        std::size_t bytes;
        int device;
    };
    std::vector<Back> back;
    int device = 0;
    bool any = false;
};

int pick_device(std::initializer_list<std::pair<const sbx_context *, int>> ctxs, const Comm &comm) {
    if (comm.device >= 0) return comm.device;
    for (auto &c : ctxs)
        for (int i = 0; i < c.second; ++i)
            if (c.first[i].plat == SBX_GPU) return c.first[i].device;
    return 0;
}

DistTensor make_tensor(int nd, const char *o, const int *dim, const int *p, int ncomponents,
                       const void *const *v, const sbx_context *ctx, int dtype, const Comm &comm,
                       bool rev, Mirror &mirror, bool is_output, const char *what) {
    DistTensor t;
    t.labels = to_labels(o, nd, rev, what);
    t.dim = to_coor(dim, nd, rev);
    t.dtype = dtype;
    t.ranges = to_ranges(p, nd, ncomponents, comm, rev);
    for (int i = 0; i < nd; ++i)
        if (t.dim[i] < 0) throw Error("negative dimension");
    for (int c = 0; c < ncomponents; ++c) {
        const Range &r = t.ranges[comm.rank][c];
        for (int i = 0; i < nd; ++i)
            if (r.size[i] > t.dim[i] || r.from[i] < 0 || (t.dim[i] > 0 && r.from[i] >= t.dim[i] && r.size[i] > 0))
                throw Error(std::string(what) + ": invalid partition");
        const std::size_t bytes = volume(r.size) * dtype_size(dtype);
        void *ptr = const_cast<void *>(v ? v[c] : nullptr);
        if (ctx[c].plat == SBX_GPU) {
            t.ptr.push_back(ptr);
            t.dev.push_back(ctx[c].device);
        } else {
            // host component: mirror to the device
            mirror.any = true;
            mirror.bufs.emplace_back(bytes, mirror.device);
            void *d = mirror.bufs.back().ptr;
            if (bytes > 0) {
                set_device(mirror.device);
                SBX_HIP_CHECK(hipMemcpyAsync(d, ptr, bytes, hipMemcpyHostToDevice,
                                             get_stream(mirror.device)));
            }
            if (is_output && bytes > 0) mirror.back.push_back({ptr, d, bytes, mirror.device});
            t.ptr.push_back(d);
            t.dev.push_back(mirror.device);
        }
    }
    return t;
}

/// Masks of copy() (MaskType = float, one per component, laid out like its data); host masks
/// are mirrored to the device like host data
void attach_masks(DistTensor &t, const float *const *mask, int ncomponents,
                  const sbx_context *ctx, const Comm &comm, Mirror &mirror) {
    if (!mask) return;
    for (int c = 0; c < ncomponents; ++c) {
        const float *m = mask[c];
        const std::size_t bytes = volume(t.ranges[comm.rank][c].size) * sizeof(float);
        if (!m && bytes > 0) throw Error("copy: null mask pointer for a nonempty component");
        if (ctx[c].plat != SBX_GPU && bytes > 0) {
            mirror.any = true;
            mirror.bufs.emplace_back(bytes, mirror.device);
            set_device(mirror.device);
            SBX_HIP_CHECK(hipMemcpyAsync(mirror.bufs.back().ptr, m, bytes, hipMemcpyHostToDevice,
                                         get_stream(mirror.device)));
            m = (const float *)mirror.bufs.back().ptr;
        }
        t.mask.push_back(m);
    }
}

/// Element conversions of copy(): same type, real -> real, real -> complex, complex -> complex
/// (blas.h:57-65; never complex -> real), and int <-> size_t
void check_copy_types(int t0, int t1) {
    auto real = [](int t) { return t == SBX_FLOAT || t == SBX_DOUBLE; };
    auto index = [](int t) { return t == SBX_INT || t == SBX_SIZE_T; };
    if (t0 == t1 || (real(t0) && (real(t1) || dtype_is_complex(t1))) ||
        (dtype_is_complex(t0) && dtype_is_complex(t1)) || (index(t0) && index(t1)))
        return;
    throw Error("copy: unsupported type conversion");
}

void finish_mirror(Mirror &m) {
    if (!m.any) return;
    for (auto &b : m.back) {
        set_device(b.device);
        SBX_HIP_CHECK(
            hipMemcpyAsync(b.host, b.dev, b.bytes, hipMemcpyDeviceToHost, get_stream(b.device)));
    }
    set_device(m.device);
    SBX_HIP_CHECK(hipStreamSynchronize(get_stream(m.device)));
}

Scalar to_scalar(const double *a) { return a ? Scalar{a[0], a[1]} : Scalar{1, 0}; }

void check_session(int session) {
    if (session != 0) throw Error("only session 0 is supported");
}

sbx_storage_s &storage_of(sbx_storage sto) {
    if (!sto || !sto->s) throw Error("storage: invalid handle");
    return *sto;
}

} // namespace

struct sbx_request_s {
    std::function<void()> fn; // the pending part of the operation
};

namespace {
//
// copy() fast path: single process, device components, no masks.  The first call of a shape
// runs the planner with a launch tape on; later calls of the same shape (every argument but the
// data pointers and a nonzero alpha) replay the tape on the new pointers -- no planning, no
// allocations (the reference's copy-plan cache, dist.h:2303-2353).
//
struct TapeKeyHash {
    std::size_t operator()(const std::vector<long> &k) const {
        std::size_t h = 1469598103934665603ull;
        for (long v : k) h = (h ^ (std::size_t)v) * 1099511628211ull;
        return h;
    }
};
std::mutex g_tape_mutex;
std::unordered_map<std::vector<long>, std::shared_ptr<const CopyTape>, TapeKeyHash> &tapes() {
    static std::unordered_map<std::vector<long>, std::shared_ptr<const CopyTape>, TapeKeyHash> m;
    return m;
}

void key_ints(std::vector<long> &k, const int *p, long n) {
    for (long i = 0; i < n; ++i) k.push_back(p ? p[i] : 0);
}
void key_str(std::vector<long> &k, const char *o, int n) {
    for (int i = 0; i < n; ++i) k.push_back(o[i]);
}

/// Resolve a recorded pointer to (argument, component, byte offset) among the call's components;
/// false when it lies in none or in more than one (aliasing: not replayable)
bool resolve(const void *ptr, const void *const *v0, const int *p0, int nc0, int nd0, int t0,
             const void *const *v1, const int *p1, int nc1, int nd1, int t1, int &arg, int &comp,
             long &off) {
    int found = 0;
    auto scan = [&](const void *const *v, const int *p, int nc, int nd, int t, int a) {
        for (int c = 0; c < nc; ++c) {
            long vol = 1;
            for (int i = 0; i < nd; ++i) vol *= p[(long)c * 2 * nd + nd + i];
            const char *b = (const char *)v[c];
            const long bytes = vol * (long)dtype_size(t);
            if (b && (const char *)ptr >= b && (const char *)ptr < b + std::max(bytes, 1L)) {
                ++found;
                arg = a;
                comp = c;
                off = (long)((const char *)ptr - b);
            }
        }
    };
    scan(v0, p0, nc0, nd0, t0, 0);
    scan(v1, p1, nc1, nd1, t1, 1);
    return found == 1;
}
} // namespace

extern "C" {

const char *sbx_last_error(void) { return g_last_error.c_str(); }

int sbx_version(int *major, int *minor) {
    return guard([&] {
        if (major) *major = 0;
        if (minor) *minor = 2;
    });
}

int sbx_get_gpu_devices_count(int *n) {
    return guard([&] {
        int c = 0;
        if (hipGetDeviceCount(&c) != hipSuccess) {
            (void)hipGetLastError();
            c = 0;
        }
        *n = c;
    });
}

int sbx_sync(sbx_context ctx) {
    return guard([&] {
        if (ctx.plat != SBX_GPU) return;
        set_device(ctx.device);
        SBX_HIP_CHECK(hipStreamSynchronize(get_stream(ctx.device)));
    });
}

int sbx_stream_get(int device, void **stream) {
    return guard([&] { *stream = (void *)get_stream(device); });
}

int sbx_stream_set(int device, void *stream) {
    return guard([&] { set_user_stream(device, (hipStream_t)stream, true); });
}

int sbx_stream_reset(int device) {
    return guard([&] { set_user_stream(device, nullptr, false); });
}

int sbx_clear_caches(void) {
    return guard([&] {
        trim_pools();
        clear_copy_plan_cache();
        clear_copy_launch_cache();
        std::lock_guard<std::mutex> g(g_tape_mutex);
        tapes().clear();
    });
}

int sbx_clear_handles(void) {
    return guard([&] {
        trim_pools(); // cached scratch may name a library stream as its last user
        destroy_streams();
    });
}

int sbx_allocate(unsigned long long bytes, sbx_context ctx, void **ptr) {
    return guard([&] {
        if (ctx.plat == SBX_GPU) {
            *ptr = device_alloc(bytes, ctx.device);
        } else {
            SBX_HIP_CHECK(hipHostMalloc(ptr, bytes, hipHostMallocDefault));
        }
    });
}

int sbx_deallocate(void *ptr, sbx_context ctx) {
    return guard([&] {
        if (!ptr) return;
        if (ctx.plat == SBX_GPU) {
            set_device(ctx.device);
            SBX_HIP_CHECK(hipStreamSynchronize(get_stream(ctx.device)));
            device_free(ptr, ctx.device);
        } else {
            SBX_HIP_CHECK(hipHostFree(ptr));
        }
    });
}

int sbx_set_custom_allocator(sbx_alloc_fn alloc, sbx_free_fn dealloc, void *user) {
    return guard([&] {
        if ((alloc == nullptr) != (dealloc == nullptr))
            throw Error("set_custom_allocator: give both functions or neither");
        set_alloc_hooks(alloc, dealloc, user);
    });
}

int sbx_allocate_from_cache(unsigned long long bytes, sbx_context ctx, void **ptr) {
    return guard([&] {
        if (ctx.plat != SBX_GPU) throw Error("allocate_from_cache: GPU contexts only");
        *ptr = scratch_alloc(bytes, ctx.device);
    });
}

int sbx_release_to_cache(void *ptr, sbx_context ctx) {
    return guard([&] {
        if (ctx.plat != SBX_GPU) throw Error("release_to_cache: GPU contexts only");
        scratch_free(ptr, ctx.device);
    });
}

int sbx_cache_usage(int device, unsigned long long *cached, unsigned long long *live) {
    return guard([&] {
        std::size_t c = 0, l = 0;
        cache_usage(device, &c, &l);
        if (cached) *cached = c;
        if (live) *live = l;
    });
}

int sbx_tune_set(const char *key, long long value) {
    return guard([&] {
        if (!key) throw Error("tune_set: null key");
        const std::string k(key);
        if (k == "copy.budget") g_copy_tune.budget = (long)value;
        else if (k == "copy.run") g_copy_tune.run = (long)value;
        else if (k == "copy.nt") g_copy_tune.nt = (int)value;
        else if (k == "copy.max_elems") g_copy_tune.max_elems = (long)value;
        else if (k == "copy.pair") g_copy_tune.pair = (int)value;
        else if (k == "copy.order") g_copy_tune.order = (int)value;
        else if (k == "copy.trans") g_copy_tune.trans = (int)value;
        else if (k == "copy.btrans") g_copy_tune.btrans = (int)value;
        else if (k == "gemm.max_bytes") g_gemm_tune.max_bytes = (long)value;
        else if (k == "gemm.loaders") g_gemm_tune.loaders = (int)value;
        else if (k == "gemm.dma_spread") g_gemm_tune.dma_spread = (int)value;
        else if (k == "gemm.dma_nt") g_gemm_tune.dma_nt = (int)value;
        else if (k == "gemm.skinny") g_gemm_tune.skinny = (int)value;
        else if (k == "bsr.variant") g_bsr_tune.variant = (int)value;
        else if (k == "bsr.row_max_cols") g_bsr_tune.row_max_cols = (long)value;
        else if (k == "bsr.split_max_cols") g_bsr_tune.split_max_cols = (long)value;
        else if (k == "bsr.split_cw") g_bsr_tune.split_cw = (int)value;
        else if (k == "bsr.split_jb") g_bsr_tune.split_jb = (int)value;
        else if (k == "bsr.split_ilv") g_bsr_tune.split_ilv = (int)value;
        else if (k == "bsr.kron_mfma") g_bsr_tune.kron_mfma = (int)value;
        else if (k == "bsr.kron_mfma_min_cols") g_bsr_tune.kron_mfma_min_cols = (long)value;
        else if (k == "bsr.kron_pack") g_bsr_tune.kron_pack = (int)value;
        else if (k == "bsr.kron_xlds") g_bsr_tune.kron_xlds = (int)value;
        else if (k == "bsr.kron_ylds") g_bsr_tune.kron_ylds = (int)value;
        else if (k == "bsr.kron_spin") g_bsr_tune.kron_spin = (int)value;
        else if (k == "bsr.kron_spin_min_cols") g_bsr_tune.kron_spin_min_cols = (long)value;
        else if (k == "bsr.kron_order") g_bsr_tune.kron_order = (int)value;
        else if (k == "bsr.nt") g_bsr_tune.nt = (int)value;
        else if (k == "dense.wave") g_dense_wave = (int)value;
        else if (k == "bsr.blk_pd") g_bsr_tune.blk_pd = (int)value;
        else if (k == "bsr.tile") g_bsr_tune.tile = (int)value;
        else if (k == "bsr.tile_min_cols") g_bsr_tune.tile_min_cols = value;
        else if (k == "gemm.m3") g_gemm_tune.m3 = (int)value;
        else if (k == "gemm.splits") g_gemm_tune.splits = (int)value;
        else if (k == "gemm.t48") g_gemm_tune.t48 = (int)value;
        else if (k == "gemm.share_ab") g_gemm_tune.share_ab = (int)value;
        else if (k == "gemm.frag") g_gemm_tune.frag = (int)value;
        else if (k == "gemm.dot_wgs") g_gemm_tune.dot_wgs = (int)value;
        else if (k == "gemm.frag_tall") g_gemm_tune.frag_tall = (int)value;
        else if (k == "gemm.frag_pair") g_gemm_tune.frag_pair = (int)value;
        else if (k == "gemm.frag_nt") g_gemm_tune.frag_nt = (int)value;
        else if (k == "gemm.frag_small") g_gemm_tune.frag_small = (int)value;
        else if (k == "gemm.frag_uk") g_gemm_tune.frag_uk = (int)value;
        else if (k == "gemm.frag_waves") g_gemm_tune.frag_waves = (int)value;
        else if (k == "gemm.clock") {
            g_gemm_tune.clock = (int)value;
            unsigned long long v[3];
            gemm_clock_read(current_device(), v, true); // a new measurement starts at zero
        }
        else if (k == "dist.reduce") g_dist_reduce = (int)value;
        else if (k == "debug.level") g_debug_level = (int)value;
        else if (k == "debug.corrupt_copy") g_debug_corrupt = (int)value;
        else if (k == "dist.reduce_calls") g_dist_reduce_calls = value;
        else if (k == "dist.force_peer") g_dist_force_peer = (int)value;
        else if (k == "dist.peer_copies") g_dist_peer_copies = value;
        else if (k.compare(0, 6, "alloc.") == 0) alloc_tune(key, nullptr, &value);
        else throw Error("tune_set: unknown key " + k);
        if (k.compare(0, 5, "copy.") == 0) {
            // recorded launch tapes replay the kernel form chosen when they were recorded
            std::lock_guard<std::mutex> g(g_tape_mutex);
            tapes().clear();
        }
    });
}

int sbx_tune_get(const char *key, long long *value) {
    return guard([&] {
        if (!key || !value) throw Error("tune_get: null argument");
        const std::string k(key);
        if (k == "copy.budget") *value = g_copy_tune.budget;
        else if (k == "copy.run") *value = g_copy_tune.run;
        else if (k == "copy.nt") *value = g_copy_tune.nt;
        else if (k == "copy.max_elems") *value = g_copy_tune.max_elems;
        else if (k == "copy.pair") *value = g_copy_tune.pair;
        else if (k == "copy.order") *value = g_copy_tune.order;
        else if (k == "copy.trans") *value = g_copy_tune.trans;
        else if (k == "copy.btrans") *value = g_copy_tune.btrans;
        else if (k == "copy.last_pair") *value = g_copy_tune.last_pair;
        else if (k == "gemm.max_bytes") *value = g_gemm_tune.max_bytes;
        else if (k == "gemm.loaders") *value = g_gemm_tune.loaders;
        else if (k == "gemm.dma_spread") *value = g_gemm_tune.dma_spread;
        else if (k == "gemm.dma_nt") *value = g_gemm_tune.dma_nt;
        else if (k == "gemm.skinny") *value = g_gemm_tune.skinny;
        else if (k == "bsr.variant") *value = g_bsr_tune.variant;
        else if (k == "bsr.row_max_cols") *value = g_bsr_tune.row_max_cols;
        else if (k == "bsr.split_max_cols") *value = g_bsr_tune.split_max_cols;
        else if (k == "bsr.split_cw") *value = g_bsr_tune.split_cw;
        else if (k == "bsr.split_jb") *value = g_bsr_tune.split_jb;
        else if (k == "bsr.split_ilv") *value = g_bsr_tune.split_ilv;
        else if (k == "bsr.kron_mfma") *value = g_bsr_tune.kron_mfma;
        else if (k == "bsr.kron_mfma_min_cols") *value = g_bsr_tune.kron_mfma_min_cols;
        else if (k == "bsr.kron_pack") *value = g_bsr_tune.kron_pack;
        else if (k == "bsr.kron_xlds") *value = g_bsr_tune.kron_xlds;
        else if (k == "bsr.kron_ylds") *value = g_bsr_tune.kron_ylds;
        else if (k == "bsr.kron_spin") *value = g_bsr_tune.kron_spin;
        else if (k == "bsr.kron_spin_min_cols") *value = g_bsr_tune.kron_spin_min_cols;
        else if (k == "bsr.kron_order") *value = g_bsr_tune.kron_order;
        else if (k == "bsr.nt") *value = g_bsr_tune.nt;
        else if (k == "dense.wave") *value = g_dense_wave;
        else if (k == "bsr.blk_pd") *value = g_bsr_tune.blk_pd;
        else if (k == "bsr.tile") *value = g_bsr_tune.tile;
        else if (k == "bsr.tile_min_cols") *value = g_bsr_tune.tile_min_cols;
        else if (k == "bsr.last_kernel") *value = g_bsr_tune.last;
        else if (k == "gemm.m3") *value = g_gemm_tune.m3;
        else if (k == "gemm.splits") *value = g_gemm_tune.splits;
        else if (k == "gemm.t48") *value = g_gemm_tune.t48;
        else if (k == "gemm.share_ab") *value = g_gemm_tune.share_ab;
        else if (k == "gemm.frag") *value = g_gemm_tune.frag;
        else if (k == "gemm.dot_wgs") *value = g_gemm_tune.dot_wgs;
        else if (k == "gemm.frag_tall") *value = g_gemm_tune.frag_tall;
        else if (k == "gemm.frag_pair") *value = g_gemm_tune.frag_pair;
        else if (k == "gemm.frag_nt") *value = g_gemm_tune.frag_nt;
        else if (k == "gemm.frag_small") *value = g_gemm_tune.frag_small;
        else if (k == "gemm.frag_uk") *value = g_gemm_tune.frag_uk;
        else if (k == "gemm.frag_waves") *value = g_gemm_tune.frag_waves;
        else if (k == "gemm.clock") *value = g_gemm_tune.clock;
        else if (k == "gemm.clock_cycles" || k == "gemm.clock_ticks" || k == "gemm.clock_launches") {
            unsigned long long v[3];
            gemm_clock_read(current_device(), v, false);
            *value = (long long)v[k == "gemm.clock_cycles" ? 0 : k == "gemm.clock_ticks" ? 1 : 2];
        }
        else if (k == "dist.reduce") *value = g_dist_reduce;
        else if (k == "debug.level") *value = g_debug_level;
        else if (k == "debug.corrupt_copy") *value = g_debug_corrupt;
        else if (k == "dist.reduce_calls") *value = g_dist_reduce_calls;
        else if (k == "dist.force_peer") *value = g_dist_force_peer;
        else if (k == "dist.peer_copies") *value = g_dist_peer_copies;
        else if (k == "detail.last_device") *value = g_detail_last_device;
        else if (k.compare(0, 6, "alloc.") == 0) alloc_tune(key, value, nullptr);
        else throw Error("tune_get: unknown key " + k);
    });
}

int sbx_timings_enable(int on) {
    return guard([&] { timings_enable(on != 0); });
}

int sbx_timings_filter(const char *names) {
    return guard([&] { timings_filter(names && *names ? names : nullptr); });
}

int sbx_timings_reset(void) {
    return guard([&] { timings_reset(); });
}

int sbx_timings_get(const char *name, double *ms, long long *calls) {
    return guard([&] {
        if (!name || !ms || !calls) throw Error("timings_get: null argument");
        timings_get(name, ms, calls);
    });
}

int sbx_timings_report(char *buf, int len) {
    return guard([&] {
        const std::string r = timings_report();
        if (buf && len > 0) {
            const int n = std::min((int)r.size(), len - 1);
            std::memcpy(buf, r.data(), n);
            buf[n] = 0;
        }
    });
}

int sbx_comm_unique_id(unsigned char *id) {
    return guard([&] {
        ncclUniqueId u;
        ncclResult_t r = ncclGetUniqueId(&u);
        if (r != ncclSuccess) throw Error(std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
        static_assert(sizeof(ncclUniqueId) == 128, "unexpected ncclUniqueId size");
        std::memcpy(id, &u, sizeof(u));
    });
}

int sbx_comm_create(int nprocs, int rank, const unsigned char *id, int device, sbx_comm *comm) {
    return guard([&] {
        if (nprocs < 1 || rank < 0 || rank >= nprocs) throw Error("invalid rank/nprocs");
        std::unique_ptr<sbx_comm_s> c(new sbx_comm_s());
        c->c.nprocs = nprocs;
        c->c.rank = rank;
        c->c.device = device;
        if (nprocs > 1) {
            set_device(device);
            ncclUniqueId u;
            std::memcpy(&u, id, sizeof(u));
            ncclComm_t nc;
            ncclResult_t r = ncclCommInitRank(&nc, nprocs, u, rank);
            if (r != ncclSuccess)
                throw Error(std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
            c->c.nccl = nc;
        }
        *comm = c.release();
    });
}

int sbx_comm_create_host(int nprocs, int rank, int device, sbx_alltoallv_fn fn, void *user,
                         sbx_comm *comm) {
    return guard([&] {
        if (nprocs < 1 || rank < 0 || rank >= nprocs) throw Error("invalid rank/nprocs");
        if (!fn) throw Error("comm_create_host: null all-to-all callback");
        std::unique_ptr<sbx_comm_s> c(new sbx_comm_s());
        c->c.nprocs = nprocs;
        c->c.rank = rank;
        c->c.device = device;
        c->c.host_fn = fn;
        c->c.host_user = user;
        c->stage.reset(new HostStage());
        c->c.stage = c->stage.get();
        *comm = c.release();
    });
}

int sbx_comm_rank(sbx_comm comm, int *rank, int *nprocs) {
    return guard([&] {
        const Comm c = get_comm(comm);
        if (rank) *rank = c.rank;
        if (nprocs) *nprocs = c.nprocs;
    });
}

int sbx_copy_kernel_plan(int nd, const long long *size, const long long *src_stride,
                         const long long *dst_stride, int t0, int t1, int add, int masked,
                         int *kind, long long *blocks) {
    return guard([&] {
        check_copy_types(t0, t1);
        BoxCopyDesc d{};
        d.src_t = t0;
        d.dst_t = t1;
        d.add = add != 0;
        static const float mask_token = 1;
        if (masked) d.src_mask = d.dst_mask = &mask_token; // (only the presence matters here)
        for (int i = 0; i < nd; ++i) {
            if (size[i] < 0 || src_stride[i] < 0 || dst_stride[i] < 0)
                throw Error("copy_kernel_plan: negative size or stride");
            d.size.push_back((long)size[i]);
            d.src_stride.push_back((long)src_stride[i]);
            d.dst_stride.push_back((long)dst_stride[i]);
        }
        long b = 0;
        *kind = copy_kernel_plan(d, &b);
        if (blocks) *blocks = b;
    });
}

int sbx_comm_transport(sbx_comm comm, int *kind, int *count, int *user_rank) {
    return guard([&] {
        const Comm c = get_comm(comm);
        int k = 0, n = c.nprocs, r = c.rank;
        if (c.nccl) {
            k = 1;
            ncclResult_t e = ncclCommCount((ncclComm_t)c.nccl, &n);
            if (e == ncclSuccess) e = ncclCommUserRank((ncclComm_t)c.nccl, &r);
            if (e != ncclSuccess) throw Error(std::string("RCCL: ") + ncclGetErrorString(e));
        } else if (c.host_fn) {
            k = 2;
        }
        if (kind) *kind = k;
        if (count) *count = n;
        if (user_rank) *user_rank = r;
    });
}

int sbx_comm_destroy(sbx_comm comm) {
    return guard([&] {
        if (!comm) return;
        if (comm->c.nccl) ncclCommDestroy((ncclComm_t)comm->c.nccl);
        delete comm;
    });
}

int sbx_partitioning_distributed_procs(int nd, const char *order, const int *dim,
                                       const char *dist_labels, int nprocs, int *procs) {
    return guard([&] {
        Coor p = partitioning_distributed_procs(std::string(order, nd), to_coor(dim, nd, false),
                                                dist_labels ? dist_labels : "", (unsigned)nprocs);
        for (int i = 0; i < nd; ++i) procs[i] = p[i];
    });
}

int sbx_basic_partitioning(int nd, const char *order, const int *dim, const int *procs,
                           const char *dist_labels, int nprocs, int ncomponents, int *out) {
    return guard([&] {
        auto r = basic_partitioning(order, to_coor(dim, nd, false), to_coor(procs, nd, false),
                                    dist_labels, nprocs, ncomponents);
        for (std::size_t k = 0; k < r.size(); ++k)
            for (int i = 0; i < nd; ++i) {
                out[k * 2 * nd + i] = r[k].from[i];
                out[k * 2 * nd + nd + i] = r[k].size[i];
            }
    });
}

int sbx_basic_partitioning_ext(int nd, const int *dim, const int *procs, int nprocs,
                               int replicate, const int *ext_power, int *out) {
    return guard([&] {
        auto r = basic_partitioning_ext(to_coor(dim, nd, false), to_coor(procs, nd, false), nprocs,
                                        replicate != 0,
                                        ext_power ? to_coor(ext_power, nd, false) : Coor(nd, 0));
        for (std::size_t k = 0; k < r.size(); ++k)
            for (int i = 0; i < nd; ++i) {
                out[k * 2 * nd + i] = r[k].from[i];
                out[k * 2 * nd + nd + i] = r[k].size[i];
            }
    });
}

int sbx_make_hole(int nd, const int *from, const int *size, const int *hole_from,
                  const int *hole_size, const int *dim, int maxout, int *out, int *nout) {
    return guard([&] {
        auto r = make_hole(Range{to_coor(from, nd, false), to_coor(size, nd, false)},
                           Range{to_coor(hole_from, nd, false), to_coor(hole_size, nd, false)},
                           to_coor(dim, nd, false));
        if ((int)r.size() > maxout) throw Error("make_hole: output buffer too small");
        for (std::size_t k = 0; k < r.size(); ++k)
            for (int i = 0; i < nd; ++i) {
                out[k * 2 * nd + i] = r[k].from[i];
                out[k * 2 * nd + nd + i] = r[k].size[i];
            }
        *nout = (int)r.size();
    });
}

int sbx_wait(sbx_request request) {
    return guard([&] {
        if (!request) return;
        std::unique_ptr<sbx_request_s> r(request);
        if (r->fn) r->fn();
    });
}

int sbx_copy_masked(int nd0, int nd1, const double *alpha, int t0, int t1, const int *p0,
                    int ncomponents0, const char *o0, const int *from0, const int *size0,
                    const int *dim0, const void *const *v0, const float *const *mask0,
                    const sbx_context *ctx0, const int *p1, int ncomponents1, const char *o1,
                    const int *from1, const int *dim1, void *const *v1,
                    const float *const *mask1, const sbx_context *ctx1, sbx_comm comm, int co,
                    int copyadd, int session) {
    return sbx_copy_req(nd0, nd1, alpha, t0, t1, p0, ncomponents0, o0, from0, size0, dim0, v0,
                        mask0, ctx0, p1, ncomponents1, o1, from1, dim1, v1, mask1, ctx1, comm, co,
                        copyadd, session, nullptr);
}

namespace {
/// SB_DEBUG >= 1 (runtime_features.h:24-37): the GPU is synchronised and the ranks meet at a
/// barrier before and after every copy and contraction (the reference's debug mode, dist.h:2274-2280);
/// debug_level() is in debug.cpp (the tune key debug.level overrides SB_DEBUG)
struct DebugSync {
    const Comm &c;
    explicit DebugSync(const Comm &c_) : c(c_) { sync(); }
    ~DebugSync() {
        try {
            sync();
        } catch (...) {
        }
    }
    void sync() {
        if (debug_level() <= 0) return;
        SBX_HIP_CHECK(hipDeviceSynchronize());
        comm_barrier(c);
    }
};
} // namespace

int sbx_copy_req(int nd0, int nd1, const double *alpha, int t0, int t1, const int *p0,
                 int ncomponents0, const char *o0, const int *from0, const int *size0,
                 const int *dim0, const void *const *v0, const float *const *mask0,
                 const sbx_context *ctx0, const int *p1, int ncomponents1, const char *o1,
                 const int *from1, const int *dim1, void *const *v1, const float *const *mask1,
                 const sbx_context *ctx1, sbx_comm comm, int co, int copyadd, int session,
                 sbx_request *request) {
    if (request) *request = nullptr;
    return guard([&] {
        check_session(session);
        check_copy_types(t0, t1);
        if (mask0 && !mask1)
            throw Error("copy: a destination mask (mask1) is required with an origin mask");
        const Comm c = get_comm(comm);
        const DebugSync dbg(c);
        const Scalar a_call = to_scalar(alpha);
        // fast path (see above): the shape key excludes the data pointers and alpha's value
        // (SB_DEBUG >= 2 checks every copy through dist_copy: no replay)
        bool fast = !mask0 && !mask1 && c.nprocs == 1 && debug_level() < 2 &&
                    g_debug_corrupt.load() == 0 && p0 && p1 && v0 &&
                    v1 && o0 && o1 &&
                    ncomponents0 >= 1 && ncomponents1 >= 1 && ctx0 && ctx1 &&
                    (int)std::strlen(o0) == nd0 && (int)std::strlen(o1) == nd1;
        for (int i = 0; fast && i < ncomponents0; ++i) fast = ctx0[i].plat == SBX_GPU;
        for (int i = 0; fast && i < ncomponents1; ++i) fast = ctx1[i].plat == SBX_GPU;
        std::vector<long> key;
        if (fast) {
            key.reserve(32 + 6 * (nd0 + nd1) + 2 * (ncomponents0 * nd0 + ncomponents1 * nd1));
            key.insert(key.end(), {nd0, nd1, t0, t1, ncomponents0, ncomponents1, co, copyadd,
                                   (long)a_call.is_zero(), comm ? 1L : 0L, c.device,
                                   g_copy_tune.budget, g_copy_tune.run,
                                   g_copy_tune.nt, g_copy_tune.max_elems, (long)g_copy_tune.pair,
                                   (long)g_copy_tune.order});
            key_str(key, o0, nd0);
            key_str(key, o1, nd1);
            key_ints(key, p0, 2L * nd0 * ncomponents0);
            key_ints(key, p1, 2L * nd1 * ncomponents1);
            key_ints(key, from0, nd0);
            key_ints(key, size0, nd0);
            key_ints(key, dim0, nd0);
            key_ints(key, from1, nd1);
            key_ints(key, dim1, nd1);
            for (int i = 0; i < ncomponents0; ++i) key.push_back(ctx0[i].device);
            for (int i = 0; i < ncomponents1; ++i) key.push_back(ctx1[i].device);
            std::shared_ptr<const CopyTape> tape;
            {
                std::lock_guard<std::mutex> g(g_tape_mutex);
                auto it = tapes().find(key);
                if (it != tapes().end()) tape = it->second;
            }
            if (tape) {
                for (const TapeLaunch &l : tape->launches) {
                    const char *sb = l.src_arg == 0 ? (const char *)v0[l.src_comp]
                                                    : (const char *)v1[l.src_comp];
                    char *db = l.dst_arg == 0 ? (char *)const_cast<void *>(v0[l.dst_comp])
                                              : (char *)v1[l.dst_comp];
                    replay_launch(l, sb + l.src_off, db + l.dst_off, l.alpha_is_call ? a_call : l.alpha);
                }
                return;
            }
        }
        const bool rev = co == SBX_FAST_TO_SLOW;
        check_copy_args(to_labels(o0, nd0, rev, "o0"), to_coor(from0, nd0, rev),
                        to_coor(size0, nd0, rev), to_coor(dim0, nd0, rev),
                        to_labels(o1, nd1, rev, "o1"), to_coor(from1, nd1, rev),
                        to_coor(dim1, nd1, rev));
        Mirror m;
        m.device = pick_device({{ctx0, ncomponents0}, {ctx1, ncomponents1}}, c);
        DistTensor a = make_tensor(nd0, o0, dim0, p0, ncomponents0, v0, ctx0, t0, c, rev, m, false, "o0");
        DistTensor b = make_tensor(nd1, o1, dim1, p1, ncomponents1, (const void *const *)v1, ctx1,
                                   t1, c, rev, m, true, "o1");
        attach_masks(a, mask0, ncomponents0, ctx0, c, m);
        attach_masks(b, mask1, ncomponents1, ctx1, c, m);
        auto tape = fast ? std::make_shared<CopyTape>() : nullptr;
        set_copy_tape(tape.get());
        std::function<void()> pending;
        try {
            dist_copy(a_call, a, to_coor(from0, nd0, rev), to_coor(size0, nd0, rev), b,
                      to_coor(from1, nd1, rev), copyadd == SBX_ADD, c,
                      request && !m.any ? &pending : nullptr);
        } catch (...) {
            set_copy_tape(nullptr);
            throw;
        }
        set_copy_tape(nullptr);
        if (pending) *request = new sbx_request_s{pending};
        finish_mirror(m);
        if (tape && tape->valid) {
            // resolve the recorded pointers against the components (p0/p1 in the caller's
            // order; the byte extents do not depend on it)
            for (TapeLaunch &l : tape->launches) {
                bool ok = resolve(l.src, v0, p0, ncomponents0, nd0, t0, (const void *const *)v1, p1,
                                  ncomponents1, nd1, t1, l.src_arg, l.src_comp, l.src_off) &&
                          resolve(l.dst, v0, p0, ncomponents0, nd0, t0, (const void *const *)v1, p1,
                                  ncomponents1, nd1, t1, l.dst_arg, l.dst_comp, l.dst_off);
                const bool is_call = l.alpha.re == a_call.re && l.alpha.im == a_call.im;
                // a launch whose alpha matches neither the call nor zero would be ambiguous
                if (!is_call && !l.alpha.is_zero()) ok = false;
                l.alpha_is_call = is_call;
                if (!ok) {
                    tape->valid = false;
                    break;
                }
            }
            if (tape->valid) {
                std::lock_guard<std::mutex> g(g_tape_mutex);
                if (tapes().size() >= 4096) tapes().clear();
                tapes().emplace(std::move(key), tape);
            }
        }
    });
}

int sbx_copy(int nd0, int nd1, const double *alpha, int t0, int t1, const int *p0,
             int ncomponents0, const char *o0, const int *from0, const int *size0, const int *dim0,
             const void *const *v0, const sbx_context *ctx0, const int *p1, int ncomponents1,
             const char *o1, const int *from1, const int *dim1, void *const *v1,
             const sbx_context *ctx1, sbx_comm comm, int co, int copyadd, int session) {
    return sbx_copy_masked(nd0, nd1, alpha, t0, t1, p0, ncomponents0, o0, from0, size0, dim0, v0,
                           nullptr, ctx0, p1, ncomponents1, o1, from1, dim1, v1, nullptr, ctx1,
                           comm, co, copyadd, session);
}

int sbx_copy_plan(int nd0, int nd1, const int *p0, int ncomponents0, const char *o0,
                  const int *from0, const int *size0, const int *dim0, const int *p1,
                  int ncomponents1, const char *o1, const int *from1, const int *dim1, int nprocs,
                  int rank, int co, int copyadd, long long *send, long long *recv,
                  long long *local) {
    return guard([&] {
        if (nprocs < 1 || rank < 0 || rank >= nprocs) throw Error("copy_plan: invalid rank");
        const bool rev = co == SBX_FAST_TO_SLOW;
        Comm c;
        c.nprocs = nprocs;
        c.rank = rank;
        DistTensor a, b;
        a.labels = to_labels(o0, nd0, rev, "o0");
        a.dim = to_coor(dim0, nd0, rev);
        a.ranges = to_ranges(p0, nd0, ncomponents0, c, rev);
        b.labels = to_labels(o1, nd1, rev, "o1");
        b.dim = to_coor(dim1, nd1, rev);
        b.ranges = to_ranges(p1, nd1, ncomponents1, c, rev);
        std::vector<long> s, r;
        long l = 0;
        copy_plan_counts(a, to_coor(from0, nd0, rev), to_coor(size0, nd0, rev), b,
                         to_coor(from1, nd1, rev), copyadd == SBX_ADD, rank, s, r, l);
        for (int q = 0; q < nprocs; ++q) {
            send[q] = s[q];
            recv[q] = r[q];
        }
        *local = l;
    });
}

int sbx_local_copy(int nd0, int nd1, const double *alpha, int t0, int t1, const char *o0,
                   const int *from0, const int *size0, const int *dim0, const void *v0,
                   const char *o1, const int *from1, const int *dim1, void *v1, int co,
                   int copyadd, int device) {
    return guard([&] {
        const bool rev = co == SBX_FAST_TO_SLOW;
        DistTensor a, b;
        a.labels = to_labels(o0, nd0, rev, "o0");
        a.dim = to_coor(dim0, nd0, rev);
        a.dtype = t0;
        a.ranges = {{Range{Coor(nd0, 0), a.dim}}};
        a.ptr = {const_cast<void *>(v0)};
        a.dev = {device};
        b.labels = to_labels(o1, nd1, rev, "o1");
        b.dim = to_coor(dim1, nd1, rev);
        b.dtype = t1;
        b.ranges = {{Range{Coor(nd1, 0), b.dim}}};
        b.ptr = {v1};
        b.dev = {device};
        dist_copy(to_scalar(alpha), a, to_coor(from0, nd0, rev), to_coor(size0, nd0, rev), b,
                  to_coor(from1, nd1, rev), copyadd == SBX_ADD, Comm{});
    });
}

int sbx_contraction(int nd0, int nd1, int ndr, int t, const double *alpha, const int *p0,
                    const int *from0, const int *size0, const int *dim0, int ncomponents0,
                    const char *o0, int conj0, const void *const *v0, const sbx_context *ctx0,
                    const int *p1, const int *from1, const int *size1, const int *dim1,
                    int ncomponents1, const char *o1, int conj1, const void *const *v1,
                    const sbx_context *ctx1, const double *beta, const int *pr,
                    const int *fromr, const int *sizer, const int *dimr, int ncomponentsr,
                    const char *o_r, void *const *vr, const sbx_context *ctxr, sbx_comm comm,
                    int co, int session) {
    return guard([&] {
        check_session(session);
        if (t != SBX_FLOAT && t != SBX_DOUBLE && t != SBX_CFLOAT && t != SBX_CDOUBLE)
            throw Error("contraction: unsupported type");
        const Comm c = get_comm(comm);
        const DebugSync dbg(c);
        const bool rev = co == SBX_FAST_TO_SLOW;
        check_contraction_args(to_labels(o0, nd0, rev, "o0"), to_coor(size0, nd0, rev),
                               to_labels(o1, nd1, rev, "o1"), to_coor(size1, nd1, rev),
                               to_labels(o_r, ndr, rev, "o_r"), to_coor(sizer, ndr, rev), t, t, t);
        Mirror m;
        m.device = pick_device({{ctx0, ncomponents0}, {ctx1, ncomponents1}, {ctxr, ncomponentsr}}, c);
        DistTensor a = make_tensor(nd0, o0, dim0, p0, ncomponents0, v0, ctx0, t, c, rev, m, false, "o0");
        DistTensor b = make_tensor(nd1, o1, dim1, p1, ncomponents1, v1, ctx1, t, c, rev, m, false, "o1");
        DistTensor r = make_tensor(ndr, o_r, dimr, pr, ncomponentsr, (const void *const *)vr, ctxr,
                                   t, c, rev, m, true, "o_r");
        dist_contraction(to_scalar(alpha), a, to_coor(from0, nd0, rev), to_coor(size0, nd0, rev),
                         conj0 != 0, b, to_coor(from1, nd1, rev), to_coor(size1, nd1, rev),
                         conj1 != 0, to_scalar(beta), r, to_coor(fromr, ndr, rev),
                         to_coor(sizer, ndr, rev), c);
        finish_mirror(m);
    });
}

namespace {
int create_bsr_any(int nd, int ni, int t, const int *pim, const int *dimi, const int *pdm,
                   const int *dimd, int ncomponents, const int *blockim, const int *blockdm,
                   const int *kronim, const int *krondm, int blockImFast, const int *const *ii,
                   const int *const *jj, const void *const *v, const void *const *kronv,
                   const sbx_context *ctx, sbx_comm comm, int co, sbx_bsr *bsrh, int session) {
    return guard([&] {
        check_session(session);
        if (!bsrh) throw Error("create_bsr: null handle output");
        const Comm c = get_comm(comm);
        const bool rev = co == SBX_FAST_TO_SLOW;
        std::vector<const int *> vii, vjj;
        std::vector<const void *> vv, vk;
        std::vector<int> devs;
        for (int i = 0; i < ncomponents; ++i) {
            vii.push_back(ii[i]);
            vjj.push_back(jj[i]);
            vv.push_back(v[i]);
            if (kronv) vk.push_back(kronv[i]);
            devs.push_back(ctx[i].plat == SBX_GPU ? ctx[i].device : -1); // -1: host component
        }
        const Coor ki = kronv ? to_coor(kronim, ni, rev) : Coor(), kd = kronv ? to_coor(krondm, nd, rev) : Coor();
        std::unique_ptr<sbx_bsr_s> h(new sbx_bsr_s());
        h->op = bsr_create(nd, ni, t, to_ranges(pim, ni, ncomponents, c, rev), to_coor(dimi, ni, rev),
                           to_ranges(pdm, nd, ncomponents, c, rev), to_coor(dimd, nd, rev),
                           to_coor(blockim, ni, rev), to_coor(blockdm, nd, rev), blockImFast != 0,
                           vii, vjj, vv, devs, rev, c, kronv ? &ki : nullptr,
                           kronv ? &kd : nullptr, kronv ? &vk : nullptr);
        h->co = co;
        h->nd = nd;
        h->ni = ni;
        h->dtype = t;
        h->is_kron = kronv != nullptr;
        *bsrh = h.release();
    });
}
} // namespace

int sbx_create_bsr(int nd, int ni, int t, const int *pim, const int *dimi, const int *pdm,
                   const int *dimd, int ncomponents, const int *blockim, const int *blockdm,
                   int blockImFast, const int *const *ii, const int *const *jj,
                   const void *const *v, const sbx_context *ctx, sbx_comm comm, int co,
                   sbx_bsr *bsrh, int session) {
    return create_bsr_any(nd, ni, t, pim, dimi, pdm, dimd, ncomponents, blockim, blockdm, nullptr,
                          nullptr, blockImFast, ii, jj, v, nullptr, ctx, comm, co, bsrh, session);
}

int sbx_create_kron_bsr(int nd, int ni, int t, const int *pim, const int *dimi, const int *pdm,
                        const int *dimd, int ncomponents, const int *blockim, const int *blockdm,
                        const int *kronim, const int *krondm, int blockImFast,
                        const int *const *ii, const int *const *jj, const void *const *v,
                        const void *const *kronv, const sbx_context *ctx, sbx_comm comm, int co,
                        sbx_bsr *bsrh, int session) {
    if (!kronv || !kronim || !krondm) {
        g_last_error = "create_kron_bsr: null Kronecker values or dimensions";
        return SBX_ERROR;
    }
    return create_bsr_any(nd, ni, t, pim, dimi, pdm, dimd, ncomponents, blockim, blockdm, kronim,
                          krondm, blockImFast, ii, jj, v, kronv, ctx, comm, co, bsrh, session);
}

int sbx_bsr_krylov(sbx_bsr bsrh, int nd, int ni, int nx, int ny, int t, const double *alpha,
                   const char *oim, const char *odm, const int *px, int ncomponents,
                   const char *ox, const int *fromx, const int *sizex, const int *dimx,
                   const void *const *vx, const double *beta, const int *py, const char *oy,
                   const int *fromy, const int *sizey, const int *dimy, char okr,
                   void *const *vy, const sbx_context *ctx, sbx_comm comm, int co, int session) {
    return sbx_bsr_krylov_req(bsrh, nd, ni, nx, ny, t, alpha, oim, odm, px, ncomponents, ox,
                              fromx, sizex, dimx, vx, beta, py, oy, fromy, sizey, dimy, okr, vy,
                              ctx, comm, co, session, 0, nullptr);
}

int sbx_bsr_krylov_req(sbx_bsr bsrh, int nd, int ni, int nx, int ny, int t, const double *alpha,
                       const char *oim, const char *odm, const int *px, int ncomponents,
                       const char *ox, const int *fromx, const int *sizex, const int *dimx,
                       const void *const *vx, const double *beta, const int *py, const char *oy,
                       const int *fromy, const int *sizey, const int *dimy, char okr,
                       void *const *vy, const sbx_context *ctx, sbx_comm comm, int co,
                       int session, int just_local, sbx_request *request) {
    if (request) *request = nullptr;
    return guard([&] {
        check_session(session);
        if (!bsrh || !bsrh->op) throw Error("bsr_krylov: invalid handle");
        if (bsrh->nd != nd || bsrh->ni != ni || bsrh->dtype != t)
            throw Error("Given BSR handle doesn't match the template parameters Nd, Ni, or T");
        if (co != bsrh->co)
            throw Error("Unsupported to use a different coordinate ordering that one used to "
                        "create the matrix");
        const Comm c = get_comm(comm);
        const bool rev = co == SBX_FAST_TO_SLOW;
        Mirror m;
        m.device = pick_device({{ctx, ncomponents}}, c);
        DistTensor x = make_tensor(nx, ox, dimx, px, ncomponents, vx, ctx, t, c, rev, m, false, "ox");
        DistTensor y = make_tensor(ny, oy, dimy, py, ncomponents, (const void *const *)vy, ctx, t,
                                   c, rev, m, true, "oy");
        std::function<void()> pending;
        bsr_krylov(*bsrh->op, to_scalar(alpha), to_labels(oim, ni, rev, "oim"),
                   to_labels(odm, nd, rev, "odm"), x, to_coor(fromx, nx, rev),
                   to_coor(sizex, nx, rev), to_scalar(beta), y, to_coor(fromy, ny, rev),
                   to_coor(sizey, ny, rev), okr, c, just_local != 0,
                   request && !m.any ? &pending : nullptr);
        if (pending) *request = new sbx_request_s{pending};
        finish_mirror(m);
    });
}

int sbx_bsr_get_preferred_layout(sbx_bsr bsrh, int ncomponents, const sbx_context *ctx,
                                 sbx_comm comm, int co, int *layout_x, int *layout_y) {
    return guard([&] {
        (void)ctx;
        (void)comm;
        (void)co;
        if (!bsrh) throw Error("invalid handle");
        for (int i = 0; i < ncomponents; ++i) {
            layout_x[i] = SBX_ROW_MAJOR;
            layout_y[i] = SBX_ROW_MAJOR;
        }
    });
}

int sbx_destroy_bsr(sbx_bsr bsrh) {
    return guard([&] {
        if (!bsrh) return;
        bsr_destroy(bsrh->op);
        delete bsrh;
    });
}

/* ---- dense batched solvers (dense.h) ---- */

int sbx_cholesky(int nd, int t, const int *p, const int *dim, int ncomponents, const char *o,
                 void *const *v, const char *orows, const char *ocols, const sbx_context *ctx,
                 sbx_comm comm, int co, int session) {
    return guard([&] {
        check_session(session);
        const Comm c = get_comm(comm);
        const bool rev = co == SBX_FAST_TO_SLOW;
        Mirror m;
        m.device = pick_device({{ctx, ncomponents}}, c);
        DistTensor a = make_tensor(nd, o, dim, p, ncomponents, (const void *const *)v, ctx, t, c,
                                   rev, m, true, "o");
        dense_cholesky(a, sub_labels(orows, rev, "orows"), sub_labels(ocols, rev, "ocols"), c);
        finish_mirror(m);
    });
}

int sbx_inversion(int nd, int t, const int *p, const int *dim, int ncomponents, const char *o,
                  void *const *v, const char *orows, const char *ocols, const sbx_context *ctx,
                  sbx_comm comm, int co, int session) {
    return guard([&] {
        check_session(session);
        const Comm c = get_comm(comm);
        const bool rev = co == SBX_FAST_TO_SLOW;
        Mirror m;
        m.device = pick_device({{ctx, ncomponents}}, c);
        DistTensor a = make_tensor(nd, o, dim, p, ncomponents, (const void *const *)v, ctx, t, c,
                                   rev, m, true, "o");
        dense_inversion(a, sub_labels(orows, rev, "orows"), sub_labels(ocols, rev, "ocols"), c);
        finish_mirror(m);
    });
}

namespace {
int solve_any(bool gesm, int ndc, int ndx, int ndy, int t, const double *alpha, const int *pc,
              const int *dimc, int ncomponentsc, const char *oc, const void *const *vc,
              const char *orows, const char *ocols, const sbx_context *ctxc, const int *px,
              const int *dimx, int ncomponentsx, const char *ox, const void *const *vx,
              const sbx_context *ctxx, const int *py, const int *dimy, int ncomponentsy,
              const char *oy, void *const *vy, const sbx_context *ctxy, sbx_comm comm, int co,
              int session) {
    return guard([&] {
        check_session(session);
        const Comm c = get_comm(comm);
        const bool rev = co == SBX_FAST_TO_SLOW;
        Mirror m;
        m.device = pick_device({{ctxc, ncomponentsc}, {ctxx, ncomponentsx}, {ctxy, ncomponentsy}}, c);
        DistTensor a = make_tensor(ndc, oc, dimc, pc, ncomponentsc, vc, ctxc, t, c, rev, m, false, "oc");
        DistTensor x = make_tensor(ndx, ox, dimx, px, ncomponentsx, vx, ctxx, t, c, rev, m, false, "ox");
        DistTensor y = make_tensor(ndy, oy, dimy, py, ncomponentsy, (const void *const *)vy, ctxy,
                                   t, c, rev, m, true, "oy");
        dense_solve(gesm, to_scalar(alpha), a, sub_labels(orows, rev, "orows"),
                    sub_labels(ocols, rev, "ocols"), x, y, c);
        finish_mirror(m);
    });
}
} // namespace

int sbx_trsm(int ndc, int ndx, int ndy, int t, const double *alpha, const int *pc, const int *dimc,
             int ncomponentsc, const char *oc, const void *const *vc, const char *orows,
             const char *ocols, const sbx_context *ctxc, const int *px, const int *dimx,
             int ncomponentsx, const char *ox, const void *const *vx, const sbx_context *ctxx,
             const int *py, const int *dimy, int ncomponentsy, const char *oy, void *const *vy,
             const sbx_context *ctxy, sbx_comm comm, int co, int session) {
    return solve_any(false, ndc, ndx, ndy, t, alpha, pc, dimc, ncomponentsc, oc, vc, orows, ocols,
                     ctxc, px, dimx, ncomponentsx, ox, vx, ctxx, py, dimy, ncomponentsy, oy, vy,
                     ctxy, comm, co, session);
}

int sbx_gesm(int ndc, int ndx, int ndy, int t, const double *alpha, const int *pc, const int *dimc,
             int ncomponentsc, const char *oc, const void *const *vc, const char *orows,
             const char *ocols, const sbx_context *ctxc, const int *px, const int *dimx,
             int ncomponentsx, const char *ox, const void *const *vx, const sbx_context *ctxx,
             const int *py, const int *dimy, int ncomponentsy, const char *oy, void *const *vy,
             const sbx_context *ctxy, sbx_comm comm, int co, int session) {
    return solve_any(true, ndc, ndx, ndy, t, alpha, pc, dimc, ncomponentsc, oc, vc, orows, ocols,
                     ctxc, px, dimx, ncomponentsx, ox, vx, ctxx, py, dimy, ncomponentsy, oy, vy,
                     ctxy, comm, co, session);
}

int sbx_xgemm_batch_strided(int t, char transa, char transb, int m, int n, int k,
                            const double *alpha, const void *a, int lda, long long stridea,
                            const void *b, int ldb, long long strideb, const double *beta,
                            void *c, int ldc, long long stridec, int batch, int device) {
    return guard([&] {
        auto norm = [](char x) {
            if (x == 'n' || x == 'N') return 'N';
            if (x == 't' || x == 'T') return 'T';
            if (x == 'c' || x == 'C') return 'C';
            throw Error("Not valid value of trans");
        };
        const char ta = norm(transa), tb = norm(transb);
        GemmDesc d;
        d.t = t;
        d.m = m;
        d.n = n;
        d.k = k;
        d.batch = batch;
        d.a = a;
        d.sa_m = ta == 'N' ? 1 : lda;
        d.sa_k = ta == 'N' ? lda : 1;
        d.sa_b = stridea;
        d.conja = ta == 'C';
        d.b = b;
        d.sb_k = tb == 'N' ? 1 : ldb;
        d.sb_n = tb == 'N' ? ldb : 1;
        d.sb_b = strideb;
        d.conjb = tb == 'C';
        d.c = c;
        d.sc_m = 1;
        d.sc_n = ldc;
        d.sc_b = stridec;
        d.alpha = to_scalar(alpha);
        d.beta = to_scalar(beta);
        launch_gemm(d, device);
    });
}

//
// Low-level memory entry points of the superbblas::detail surface (include/superbblas_amd/
// detail.h): the reference's copy_n / zero_n / copy_n_blocking / xgemm_batch_strided on a
// context (blas.h:170-231, 436-490, 662-810; copy_n.h:584-1050).  Host operands are mirrored
// through device scratch like the host components of the distributed calls: every flop and
// every element conversion runs on the GPU; host destinations are complete on return.
//

namespace {

bool on_host(const sbx_context &c) { return c.plat != SBX_GPU; }

/// The one device an entry point runs on: the device of its GPU operands (all must agree), or
/// the calling thread's current device when every operand is host memory
int single_device(std::initializer_list<sbx_context> ctxs, const char *what) {
    int dev = -1;
    for (const auto &c : ctxs) {
        if (on_host(c)) continue;
        if (c.device < 0) throw Error(std::string(what) + ": invalid device");
        if (dev >= 0 && dev != c.device)
            throw Error(std::string(what) + ": operands on different devices are not supported");
        dev = c.device;
    }
    if (dev < 0) {
        dev = current_device();
        g_detail_last_device = dev;
    }
    return dev;
}

/// Largest index of an index vector (read from the host or the device)
long index_max(const int *idx, const sbx_context &c, long n) {
    std::vector<int> h;
    const int *p = idx;
    if (!on_host(c)) {
        h.resize(n);
        set_device(c.device);
        SBX_HIP_CHECK(hipStreamSynchronize(get_stream(c.device)));
        SBX_HIP_CHECK(hipMemcpy(h.data(), idx, sizeof(int) * n, hipMemcpyDeviceToHost));
        p = h.data();
    }
    long m = -1;
    for (long i = 0; i < n; ++i) {
        if (p[i] < 0) throw Error("copy_n: negative index");
        m = std::max(m, (long)p[i]);
    }
    return m;
}

/// Host memory mirrored into device scratch for the length of one call
const void *upload(std::vector<Scratch> &bufs, const void *host, std::size_t bytes, int device) {
    bufs.emplace_back(bytes, device);
    if (bytes > 0)
        SBX_HIP_CHECK(hipMemcpyAsync(bufs.back().ptr, host, bytes, hipMemcpyHostToDevice,
                                     get_stream(device)));
    return bufs.back().ptr;
}

/// Elements spanned by a column-major strided batch of rows x cols matrices
long gemm_span(long rows, long cols, long ld, long stride, long batch) {
    if (rows <= 0 || cols <= 0 || batch <= 0) return 0;
    return (batch - 1) * stride + (cols - 1) * ld + rows;
}

} // namespace

int sbx_memcpy(void *dst, sbx_context dctx, const void *src, sbx_context sctx,
               unsigned long long bytes) {
    return guard([&] {
        if (bytes == 0 || dst == src) return;
        if (!dst || !src) throw Error("copy_n: null pointer");
        if (on_host(dctx) && on_host(sctx)) {
            std::memcpy(dst, src, bytes);
        } else if (on_host(sctx)) {
            set_device(dctx.device);
            hipStream_t s = get_stream(dctx.device);
            SBX_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
            SBX_HIP_CHECK(hipStreamSynchronize(s)); // the host source may change on return
        } else if (on_host(dctx)) {
            set_device(sctx.device);
            hipStream_t s = get_stream(sctx.device);
            SBX_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
            SBX_HIP_CHECK(hipStreamSynchronize(s));
        } else if (sctx.device == dctx.device) {
            set_device(sctx.device);
            SBX_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice,
                                         get_stream(sctx.device)));
        } else {
            // peer copy on the source's stream; the destination's stream then waits for it
            // (the reference's causalConnectTo, blas.h:218-228)
            set_device(dctx.device);
            stream_after(get_stream(sctx.device), get_stream(dctx.device));
            set_device(sctx.device);
            SBX_HIP_CHECK(hipMemcpyPeerAsync(dst, dctx.device, src, sctx.device, bytes,
                                             get_stream(sctx.device)));
            stream_after(get_stream(dctx.device), get_stream(sctx.device));
        }
    });
}

int sbx_memset_zero(void *ptr, sbx_context ctx, unsigned long long bytes) {
    return guard([&] {
        if (bytes == 0) return;
        if (!ptr) throw Error("zero_n: null pointer");
        if (on_host(ctx))
            std::memset(ptr, 0, bytes);
        else
            launch_zero(ptr, bytes, ctx.device);
    });
}

int sbx_copy_n_blocking(const double *alpha, int tv, const void *v, sbx_context vctx,
                        long long blocking, const int *iv, sbx_context ivctx, long long n, int tw,
                        void *w, sbx_context wctx, const int *iw, sbx_context iwctx,
                        int copyadd) {
    return guard([&] {
        if (n < 0 || blocking < 0) throw Error("copy_n: negative size");
        if (n == 0 || blocking == 0) return;
        check_copy_types(tv, tw);
        if (!v || !w) throw Error("copy_n: null pointer");
        const int dev = single_device({vctx, wctx, iv ? ivctx : vctx, iw ? iwctx : wctx},
                                      "copy_n");
        set_device(dev);
        hipStream_t s = get_stream(dev);
        std::vector<Scratch> bufs;
        const std::size_t esv = dtype_size(tv), esw = dtype_size(tw);
        const long extv = iv ? index_max(iv, ivctx, n) + blocking : n * blocking;
        const long extw = iw ? index_max(iw, iwctx, n) + blocking : n * blocking;
        if (extv > 0x7fffffffL || extw > 0x7fffffffL)
            throw Error("copy_n: index vectors address at most 2^31 elements");
        IndexCopyDesc d;
        d.src_t = tv;
        d.dst_t = tw;
        d.n = n;
        d.blocking = blocking;
        d.alpha = to_scalar(alpha);
        d.add = copyadd == SBX_ADD;
        d.src_idx = iv && on_host(ivctx)
                        ? (const int *)upload(bufs, iv, sizeof(int) * n, dev) : iv;
        d.dst_idx = iw && on_host(iwctx)
                        ? (const int *)upload(bufs, iw, sizeof(int) * n, dev) : iw;
        d.src = on_host(vctx) ? upload(bufs, v, esv * extv, dev) : v;
        // a host destination is mirrored whole (its untouched elements come back unchanged)
        d.dst = on_host(wctx) ? const_cast<void *>(upload(bufs, w, esw * extw, dev)) : w;
        launch_index_copy(d, dev);
        if (on_host(wctx))
            SBX_HIP_CHECK(hipMemcpyAsync(w, d.dst, esw * extw, hipMemcpyDeviceToHost, s));
        if (!bufs.empty()) SBX_HIP_CHECK(hipStreamSynchronize(s));
    });
}

int sbx_checksum(const void *p, unsigned long long bytes, unsigned long long blocksize,
                 unsigned prev, unsigned *out) {
    return guard([&] {
        if (!out || (!p && bytes > 0)) throw Error("do_checksum: null argument");
        *out = storage_checksum(p, bytes, blocksize, prev);
    });
}

int sbx_intersection(int nd, const int *from0, const int *size0, const int *from1,
                     const int *size1, const int *dim, int maxout, int *out, int *nout) {
    return guard([&] {
        const Range a{to_coor(from0, nd, false), to_coor(size0, nd, false)};
        const Range b{to_coor(from1, nd, false), to_coor(size1, nd, false)};
        const std::vector<Range> r = intersection(a, b, to_coor(dim, nd, false));
        *nout = (int)r.size();
        if ((int)r.size() > maxout) throw Error("intersection: output too small");
        for (std::size_t i = 0; i < r.size(); ++i)
            for (int j = 0; j < nd; ++j) {
                out[i * 2 * nd + j] = r[i].from[j];
                out[i * 2 * nd + nd + j] = r[i].size[j];
            }
    });
}

int sbx_xgemm_batch_strided_ctx(int t, char transa, char transb, int m, int n, int k,
                                const double *alpha, const void *a, int lda, long long stridea,
                                const void *b, int ldb, long long strideb, const double *beta,
                                void *c, int ldc, long long stridec, int batch, sbx_context ctx) {
    if (!on_host(ctx))
        return sbx_xgemm_batch_strided(t, transa, transb, m, n, k, alpha, a, lda, stridea, b, ldb,
                                       strideb, beta, c, ldc, stridec, batch, ctx.device);
    std::vector<Scratch> bufs;
    const void *da = nullptr, *db = nullptr;
    void *dc = nullptr;
    long span_c = 0;
    const int dev = current_device();
    g_detail_last_device = dev;
    const int rc = guard([&] {
        const std::size_t es = dtype_size(t);
        const bool na = transa == 'n' || transa == 'N', nb = transb == 'n' || transb == 'N';
        const long span_a = gemm_span(na ? m : k, na ? k : m, lda, stridea, batch);
        const long span_b = gemm_span(nb ? k : n, nb ? n : k, ldb, strideb, batch);
        span_c = gemm_span(m, n, ldc, stridec, batch);
        set_device(dev);
        da = upload(bufs, a, es * span_a, dev);
        db = upload(bufs, b, es * span_b, dev);
        dc = const_cast<void *>(upload(bufs, c, es * span_c, dev));
    });
    if (rc != SBX_OK) return rc;
    const int rg = sbx_xgemm_batch_strided(t, transa, transb, m, n, k, alpha, da, lda, stridea, db,
                                           ldb, strideb, beta, dc, ldc, stridec, batch, dev);
    if (rg != SBX_OK) return rg;
    return guard([&] {
        hipStream_t s = get_stream(dev);
        if (span_c > 0)
            SBX_HIP_CHECK(hipMemcpyAsync(c, dc, dtype_size(t) * span_c, hipMemcpyDeviceToHost, s));
        SBX_HIP_CHECK(hipStreamSynchronize(s));
    });
}

//
// Tensor storage (storage.cpp)
//


int sbx_storage_create(int nd, const int *dim, int co, const char *filename,
                       const char *metadata, int metadata_length, int checksum, int t,
                       sbx_comm comm, sbx_storage *sto) {
    return guard([&] {
        if (!filename || !sto) throw Error("storage: null argument");
        std::unique_ptr<sbx_storage_s> h(new sbx_storage_s());
        h->dtype = t;
        h->nd = nd;
        h->s = storage_create(t, to_coor(dim, nd, co == SBX_FAST_TO_SLOW), filename, metadata,
                              metadata_length, checksum, get_comm(comm));
        *sto = h.release();
    });
}

int sbx_storage_read_header(const char *filename, int co, int *t, char *metadata,
                            int metadata_cap, int *metadata_length, int *nd, int *dim,
                            int dim_cap) {
    return guard([&] {
        if (!filename) throw Error("storage: null file name");
        int dt;
        std::string meta;
        Coor d;
        storage_read_header(filename, dt, meta, d);
        if (co == SBX_FAST_TO_SLOW) std::reverse(d.begin(), d.end());
        if (t) *t = dt;
        if (metadata && metadata_cap > 0)
            std::memcpy(metadata, meta.data(), std::min<std::size_t>(metadata_cap, meta.size()));
        if (metadata_length) *metadata_length = (int)meta.size();
        if (nd) *nd = (int)d.size();
        if (dim)
            for (int i = 0; i < std::min(dim_cap, (int)d.size()); ++i) dim[i] = d[i];
    });
}

int sbx_storage_open(int nd, int t, const char *filename, int allow_writing, sbx_comm comm,
                     sbx_storage *sto) {
    return guard([&] {
        if (!filename || !sto) throw Error("storage: null argument");
        std::unique_ptr<sbx_storage_s> h(new sbx_storage_s());
        h->dtype = t;
        h->nd = nd;
        h->s = storage_open(nd, t, filename, allow_writing != 0, get_comm(comm));
        *sto = h.release();
    });
}

int sbx_storage_append_blocks(int nd0, int nd1, const int *p0, int num_blocks, const char *o0,
                              const int *from0, const int *size0, const int *dim0,
                              const char *o1, const int *from1, sbx_storage sto, sbx_comm comm,
                              int co) {
    return guard([&] {
        sbx_storage_s &h = storage_of(sto);
        if (nd1 != h.nd) throw Error("storage: invalid number of dimensions");
        if (num_blocks < 0 || (num_blocks > 0 && !p0)) throw Error("storage: invalid blocks");
        const bool rev = co == SBX_FAST_TO_SLOW;
        std::vector<Range> blocks;
        for (int i = 0; i < num_blocks; ++i)
            blocks.push_back(Range{to_coor(p0 + (std::size_t)i * 2 * nd0, nd0, rev),
                                   to_coor(p0 + (std::size_t)i * 2 * nd0 + nd0, nd0, rev)});
        storage_append_blocks(*h.s, blocks, to_labels(o0, nd0, rev, "o0"),
                              to_coor(from0, nd0, rev), to_coor(size0, nd0, rev),
                              to_coor(dim0, nd0, rev), to_labels(o1, nd1, rev, "o1"),
                              to_coor(from1, nd1, rev), get_comm(comm));
    });
}

int sbx_storage_save(int nd0, int nd1, const double *alpha, int t0, const int *p0,
                     int ncomponents0, const char *o0, const int *from0, const int *size0,
                     const int *dim0, const void *const *v0, const sbx_context *ctx0,
                     const char *o1, const int *from1, sbx_storage sto, sbx_comm comm, int co,
                     int session) {
    return guard([&] {
        check_session(session);
        sbx_storage_s &h = storage_of(sto);
        if (nd1 != h.nd) throw Error("storage: invalid number of dimensions");
        check_copy_types(t0, h.dtype);
        const Comm c = get_comm(comm);
        const bool rev = co == SBX_FAST_TO_SLOW;
        Mirror m;
        m.device = pick_device({{ctx0, ncomponents0}}, c);
        DistTensor a = make_tensor(nd0, o0, dim0, p0, ncomponents0, v0, ctx0, t0, c, rev, m, false,
                                   "o0");
        storage_save(*h.s, to_scalar(alpha), a, to_coor(from0, nd0, rev), to_coor(size0, nd0, rev),
                     to_labels(o1, nd1, rev, "o1"), to_coor(from1, nd1, rev), c);
        finish_mirror(m);
    });
}

int sbx_storage_load(int nd0, int nd1, const double *alpha, sbx_storage sto, const char *o0,
                     const int *from0, const int *size0, int t1, const int *p1, int ncomponents1,
                     const char *o1, const int *from1, const int *dim1, void *const *v1,
                     const sbx_context *ctx1, sbx_comm comm, int co, int copyadd, int session) {
    return guard([&] {
        check_session(session);
        (void)copyadd;
        sbx_storage_s &h = storage_of(sto);
        if (nd0 != h.nd) throw Error("storage: invalid number of dimensions");
        check_copy_types(h.dtype, t1);
        const Comm c = get_comm(comm);
        const bool rev = co == SBX_FAST_TO_SLOW;
        Mirror m;
        m.device = pick_device({{ctx1, ncomponents1}}, c);
        DistTensor b = make_tensor(nd1, o1, dim1, p1, ncomponents1, (const void *const *)v1, ctx1,
                                   t1, c, rev, m, true, "o1");
        storage_load(*h.s, to_scalar(alpha), to_labels(o0, nd0, rev, "o0"),
                     to_coor(from0, nd0, rev), to_coor(size0, nd0, rev), b,
                     to_coor(from1, nd1, rev), c);
        finish_mirror(m);
    });
}

int sbx_storage_get_blocks(sbx_storage sto, int nd0, int nd1, const char *o0, const char *o1,
                           const int *from1, const int *size1, int co, int *blocks, int cap,
                           int *nblocks) {
    return guard([&] {
        sbx_storage_s &h = storage_of(sto);
        if (nd0 != h.nd) throw Error("storage: invalid number of dimensions");
        // only the storage labels follow `co` (storage.h:1404)
        const std::vector<Range> r =
            storage_get_blocks(*h.s, to_labels(o0, nd0, co == SBX_FAST_TO_SLOW, "o0"),
                               to_labels(o1, nd1, false, "o1"), to_coor(from1, nd1, false),
                               to_coor(size1, nd1, false));
        if (nblocks) *nblocks = (int)r.size();
        for (int i = 0; blocks && i < std::min(cap, (int)r.size()); ++i)
            for (int k = 0; k < nd1; ++k) {
                blocks[(std::size_t)i * 2 * nd1 + k] = r[i].from[k];
                blocks[(std::size_t)i * 2 * nd1 + nd1 + k] = r[i].size[k];
            }
    });
}

int sbx_storage_info(sbx_storage sto, int *nd, int *t) {
    return guard([&] {
        const sbx_storage_s &h = storage_of(sto);
        if (nd) *nd = h.nd;
        if (t) *t = h.dtype;
    });
}

int sbx_storage_check(sbx_storage sto, sbx_comm comm) {
    return guard([&] { storage_checksums(*storage_of(sto).s, get_comm(comm), false); });
}

int sbx_storage_flush(sbx_storage sto) {
    return guard([&] { storage_flush(*storage_of(sto).s); });
}

int sbx_storage_preallocate(sbx_storage sto, unsigned long long size) {
    return guard([&] { storage_preallocate(*storage_of(sto).s, (std::size_t)size); });
}

int sbx_storage_close(sbx_storage sto, sbx_comm comm) {
    return guard([&] {
        std::unique_ptr<sbx_storage_s> h(sto);
        if (!h) throw Error("storage: invalid handle");
        StorageCtx *s = h->s;
        h->s = nullptr;
        storage_close(s, get_comm(comm));
    });
}

} // extern "C"

