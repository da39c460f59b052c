// Device runtime: per-device library streams, the scratch-memory cache and kernel timers.
//
// Reference: platform.h:173-221 (Gpu context), 304-409 (stream helpers), 448-467
// (getGpuAllocStream: every GPU op of a device is enqueued on one library stream),
// alloc.h:91-391 (cached scratch buffers) and performance.h:356-518 (timings).
#include "sbx_internal.h"

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>

namespace sbx {

namespace {
struct DeviceState {
    hipStream_t own = nullptr;  // stream created by the library
    hipStream_t side = nullptr; // second library stream (overlapped exchanges)
    hipStream_t user = nullptr; // stream set by the caller (sbx_stream_set); may be the null stream
    bool has_user = false;
};
std::mutex g_mutex;
std::vector<DeviceState> &states() {
    static std::vector<DeviceState> s;
    return s;
}
DeviceState &state(int device) {
    auto &s = states();
    if (device < 0) throw Error("invalid device id");
    if ((int)s.size() <= device) s.resize(device + 1);
    return s[device];
}
} // namespace

void set_device(int device) {
    int cur = -1;
    SBX_HIP_CHECK(hipGetDevice(&cur));
    if (cur != device) SBX_HIP_CHECK(hipSetDevice(device));
}

hipStream_t get_stream(int device) {
    std::lock_guard<std::mutex> g(g_mutex);
    DeviceState &st = state(device);
    if (st.has_user) return st.user;
    if (!st.own) {
        set_device(device);
        SBX_HIP_CHECK(hipStreamCreateWithFlags(&st.own, hipStreamNonBlocking));
    }
    return st.own;
}

hipStream_t get_side_stream(int device) {
    std::lock_guard<std::mutex> g(g_mutex);
    DeviceState &st = state(device);
    if (!st.side) {
        set_device(device);
        SBX_HIP_CHECK(hipStreamCreateWithFlags(&st.side, hipStreamNonBlocking));
    }
    return st.side;
}

/// A stream that lives as long as the library's handles: the null stream and the library's own
/// streams (sbx_clear_handles releases the scratch cache before destroying them)
bool durable_stream(int device, hipStream_t s) {
    if (s == nullptr) return true;
    std::lock_guard<std::mutex> g(g_mutex);
    const DeviceState &st = state(device);
    return s == st.own || s == st.side;
}

void stream_after(hipStream_t to, hipStream_t from) {
    if (to == from) return;
    hipEvent_t ev;
    SBX_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    SBX_HIP_CHECK(hipEventRecord(ev, from));
    SBX_HIP_CHECK(hipStreamWaitEvent(to, ev, 0));
    SBX_HIP_CHECK(hipEventDestroy(ev));
}

StreamOverride::StreamOverride(int dev, hipStream_t s) : device(dev) {
    std::lock_guard<std::mutex> g(g_mutex);
    DeviceState &st = state(dev);
    prev = st.user;
    prev_user = st.has_user;
    st.user = s;
    st.has_user = true;
}

StreamOverride::~StreamOverride() {
    std::lock_guard<std::mutex> g(g_mutex);
    DeviceState &st = state(device);
    st.user = prev;
    st.has_user = prev_user;
}

void set_user_stream(int device, hipStream_t s, bool has_user) {
    std::lock_guard<std::mutex> g(g_mutex);
    state(device).user = s;
    state(device).has_user = has_user;
}

void destroy_streams() {
    std::lock_guard<std::mutex> g(g_mutex);
    for (std::size_t d = 0; d < states().size(); ++d) {
        DeviceState &st = states()[d];
        if (st.own) {
            (void)hipSetDevice((int)d);
            (void)hipStreamSynchronize(st.own);
            (void)hipStreamDestroy(st.own);
            st.own = nullptr;
        }
        if (st.side) {
            (void)hipSetDevice((int)d);
            (void)hipStreamSynchronize(st.side);
            (void)hipStreamDestroy(st.side);
            st.side = nullptr;
        }
    }
}

//
// Scratch memory: a caching allocator over hipMalloc (the reference's allocateBufferResouce
// cache, alloc.h:323-391).  A freed block goes back to a per-device free list together with the
// stream that last used it; a later allocation reuses it at once on the same stream (stream
// order) or, from another stream, after waiting on that stream.  A block freed on a caller's
// stream also carries an event recorded at the free (the caller may destroy its stream); one
// freed on the null stream or a library stream does not: an event record is a marker packet the
// GPU processes between two kernels (~4 us of stream time per GEMM call that used split-K
// scratch), and those streams outlive the cache (sbx_clear_handles trims it first).  Blocks stay
// mapped for the life of the cache: hipMallocAsync's pool was measured to hand back reused
// memory with stale contents after many queued launches on this platform, so it is not used.
//
// The idle blocks of a device are capped (the reference's LRU cache bound, cache.h:237-294):
// SB_CACHEGB_GPU GiB when set (runtime_features.h:147-158), otherwise 10 % of the device's
// memory; past the cap the least recently freed blocks go back to the driver.
//
// A block is freed on the stream current at the free.  When that is not the stream it was
// allocated on (a buffer made under a StreamOverride and released after the override ended, e.g.
// a deferred exchange whose request is dropped without wait), the free first makes the current
// stream wait for the allocation stream, so a reuse in the current stream's order never overlaps
// work still queued on the other one.  Such frees are counted (tune key alloc.cross_stream_frees).
//
namespace {
struct Block {
    void *p;
    std::size_t bytes;
    hipStream_t stream;
    hipEvent_t ev;
    unsigned long long seq; // free order (LRU eviction)
};
struct Live {
    std::size_t bytes;
    hipStream_t stream; // allocation stream
};
struct Cache {
    std::multimap<std::size_t, Block> free_blocks;
    std::map<void *, Live> live;
    std::size_t cached_bytes = 0;
    long long max_cached = -1; // bytes; < 0: not yet decided
};
unsigned long long g_free_seq = 0;
long long g_max_cached_override = -1; // tune key alloc.max_cached (bytes; < 0: the policy above)
long long g_cross_stream_frees = 0;
std::mutex g_cache_mutex;
std::vector<Cache> &caches() {
    static std::vector<Cache> c;
    return c;
}
Cache &cache(int device) {
    auto &c = caches();
    if ((int)c.size() <= device) c.resize(device + 1);
    return c[device];
}
struct Hooks {
    AllocHook alloc = nullptr;
    FreeHook free = nullptr;
    void *user = nullptr;
};
Hooks &hooks() {
    static Hooks h;
    return h;
}
std::size_t round_bytes(std::size_t b) {
    if (b <= 256) return 256;
    if (b < (2u << 20)) {
        std::size_t r = 256;
        while (r < b) r <<= 1;
        return r;
    }
    return (b + (2u << 20) - 1) / (2u << 20) * (2u << 20);
}
/// The cap of `device`'s idle blocks in bytes (callers hold g_cache_mutex)
long long max_cached(int device) {
    if (g_max_cached_override >= 0) return g_max_cached_override;
    Cache &c = cache(device);
    if (c.max_cached < 0) {
        const char *l = std::getenv("SB_CACHEGB_GPU");
        const double gib = l ? std::atof(l) : -1.0;
        if (gib >= 0) {
            c.max_cached = (long long)(gib * 1073741824.0);
        } else {
            std::size_t fr = 0, total = 0;
            // (hipMemGetInfo reports the current device: make it `device`, then restore)
            int prev = -1;
            (void)hipGetDevice(&prev);
            if (prev != device) (void)hipSetDevice(device);
            const hipError_t e = hipMemGetInfo(&fr, &total);
            if (prev != device && prev >= 0) (void)hipSetDevice(prev);
            if (e != hipSuccess) {
                (void)hipGetLastError();
                total = 0;
            }
            c.max_cached = total > 0 ? (long long)(total / 10) : (1LL << 34);
        }
    }
    return c.max_cached;
}
/// Take the least recently freed blocks out of the cache until the idle bytes are within the cap
/// (callers hold g_cache_mutex); the caller returns them to the driver with release_blocks after
/// dropping the lock, so a small cap does not serialise every thread behind a host sync
std::vector<Block> take_over_cap(int device) {
    std::vector<Block> out;
    Cache &c = cache(device);
    const long long cap = max_cached(device);
    while ((long long)c.cached_bytes > cap && !c.free_blocks.empty()) {
        auto oldest = c.free_blocks.begin();
        for (auto it = c.free_blocks.begin(); it != c.free_blocks.end(); ++it)
            if (it->second.seq < oldest->second.seq) oldest = it;
        out.push_back(oldest->second);
        c.cached_bytes -= oldest->second.bytes;
        c.free_blocks.erase(oldest);
    }
    return out;
}
/// Return blocks taken out of the cache to the driver (without g_cache_mutex held)
void release_blocks(const std::vector<Block> &blocks, int device) {
    for (const Block &b : blocks) {
        if (b.ev) {
            (void)hipEventSynchronize(b.ev); // its last use is done
            (void)hipEventDestroy(b.ev);
        } else {
            (void)hipStreamSynchronize(b.stream);
        }
        device_free(b.p, device);
    }
}
int log_level() {
    static const int v = [] {
        const char *l = std::getenv("SB_LOG");
        return l ? std::max(0, std::atoi(l)) : 0;
    }();
    return v;
}
/// Return every cached block of `device` to the driver (callers hold g_cache_mutex)
void release_cached(int device) {
    Cache &c = cache(device);
    if (c.free_blocks.empty()) return;
    (void)hipDeviceSynchronize();
    for (auto &e : c.free_blocks) {
        if (e.second.ev) (void)hipEventDestroy(e.second.ev);
        device_free(e.second.p, device);
    }
    c.free_blocks.clear();
    c.cached_bytes = 0;
}
} // namespace

void *scratch_alloc(std::size_t bytes, int device) {
    if (bytes == 0) return nullptr;
    set_device(device);
    const hipStream_t s = get_stream(device);
    const std::size_t rb = round_bytes(bytes);
    std::lock_guard<std::mutex> g(g_cache_mutex);
    Cache &c = cache(device);
    auto it = c.free_blocks.lower_bound(rb);
    if (it != c.free_blocks.end() && it->first <= 2 * rb) {
        Block b = it->second;
        c.free_blocks.erase(it);
        c.cached_bytes -= b.bytes;
        if (b.ev) {
            if (b.stream != s) SBX_HIP_CHECK(hipStreamWaitEvent(s, b.ev, 0));
            SBX_HIP_CHECK(hipEventDestroy(b.ev));
        } else if (b.stream != s) {
            stream_after(s, b.stream); // (a durable stream: the null or a library stream)
        }
        c.live[b.p] = Live{b.bytes, s};
        return b.p;
    }
    void *p = nullptr;
    try {
        p = device_alloc(rb, device);
    } catch (const Error &) {
        // out of memory: give the cached blocks back and retry once (alloc.h:104-168)
        (void)hipGetLastError();
        release_cached(device);
        try {
            p = device_alloc(rb, device);
        } catch (const Error &) {
            if (log_level() > 0) {
                std::size_t l = 0;
                for (auto &e : c.live) l += e.second.bytes;
                std::fprintf(stderr,
                             "superbblas_amd: error allocating %zu bytes on device %d; scratch in "
                             "use %zu MiB\n",
                             rb, device, l >> 20);
            }
            throw;
        }
    }
    c.live[p] = Live{rb, s};
    return p;
}

void set_alloc_hooks(AllocHook a, FreeHook f, void *user) {
    std::lock_guard<std::mutex> g(g_cache_mutex);
    // blocks obtained from the previous allocator go back to it before the switch
    for (int d = 0; d < (int)caches().size(); ++d) {
        (void)hipSetDevice(d);
        release_cached(d);
    }
    hooks() = Hooks{a, f, user};
}

namespace {
std::mutex g_hook_mutex;
std::map<void *, Hooks> &hook_owned() { // blocks that came from a caller's allocator
    static std::map<void *, Hooks> m;
    return m;
}
} // namespace

void *device_alloc(std::size_t bytes, int device) {
    set_device(device);
    const Hooks h = hooks();
    if (h.alloc) {
        if (void *p = h.alloc(bytes, device, h.user)) {
            std::lock_guard<std::mutex> g(g_hook_mutex);
            hook_owned()[p] = h;
            return p;
        }
        // a null answer means "use the library's allocation" (as an empty std::function)
    }
    void *p = nullptr;
    SBX_HIP_CHECK(hipMalloc(&p, bytes));
    return p;
}

void device_free(void *p, int device) {
    if (!p) return;
    set_device(device);
    Hooks h;
    bool owned = false;
    {
        std::lock_guard<std::mutex> g(g_hook_mutex);
        auto it = hook_owned().find(p);
        if (it != hook_owned().end()) {
            h = it->second;
            owned = true;
            hook_owned().erase(it);
        }
    }
    if (owned) {
        SBX_HIP_CHECK(hipDeviceSynchronize()); // the hook is not stream-ordered
        h.free(p, device, h.user);
        return;
    }
    SBX_HIP_CHECK(hipFree(p));
}

void cache_usage(int device, std::size_t *cached, std::size_t *live) {
    std::lock_guard<std::mutex> g(g_cache_mutex);
    Cache &c = cache(device);
    *cached = c.cached_bytes;
    std::size_t l = 0;
    for (auto &e : c.live) l += e.second.bytes;
    *live = l;
}

void scratch_free(void *p, int device) {
    if (!p) return;
    set_device(device);
    const hipStream_t s = get_stream(device);
    const bool durable = durable_stream(device, s);
    std::vector<Block> evict;
    {
    std::lock_guard<std::mutex> g(g_cache_mutex);
    Cache &c = cache(device);
    auto it = c.live.find(p);
    if (it == c.live.end()) throw Error("scratch_free: unknown pointer");
    Block b{p, it->second.bytes, s, nullptr, ++g_free_seq};
    if (it->second.stream != s) {
        // freed away from its allocation stream: the reuse order is this stream's, so it first
        // waits for the allocation stream's queued work
        stream_after(s, it->second.stream);
        ++g_cross_stream_frees;
    }
    c.live.erase(it);
    if (!durable) {
        SBX_HIP_CHECK(hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
        SBX_HIP_CHECK(hipEventRecord(b.ev, s));
    }
    c.free_blocks.emplace(b.bytes, b);
    c.cached_bytes += b.bytes;
    evict = take_over_cap(device);
    }
    release_blocks(evict, device);
}

void alloc_tune(const char *key, long long *get, const long long *set) {
    std::lock_guard<std::mutex> g(g_cache_mutex);
    const std::string k(key);
    if (k == "alloc.max_cached") {
        if (set) g_max_cached_override = *set;
        if (get) *get = g_max_cached_override >= 0 ? g_max_cached_override : max_cached(0);
    } else if (k == "alloc.cross_stream_frees") {
        if (set) g_cross_stream_frees = *set;
        if (get) *get = g_cross_stream_frees;
    } else {
        throw Error(std::string("tune: unknown key ") + key);
    }
}

void trim_pools() {
    std::lock_guard<std::mutex> g(g_cache_mutex);
    for (int d = 0; d < (int)caches().size(); ++d) {
        (void)hipSetDevice(d);
        release_cached(d);
    }
}

Scratch::Scratch(std::size_t bytes_, int device_) : device(device_), bytes(bytes_) {
    ptr = scratch_alloc(bytes, device);
}
Scratch::~Scratch() {
    if (ptr) {
        try {
            scratch_free(ptr, device);
        } catch (...) {
        }
    }
}

int pointer_device(const void *p) {
    if (!p) return -1;
    hipPointerAttribute_t attr;
    if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) return attr.device;
    return -1;
}

//
// Kernel timers
//
namespace {
struct TimerState {
    // SB_TRACK_TIME (runtime_features.h:55-68) turns the timers on from the start
    std::atomic<bool> on{[] {
        const char *l = std::getenv("SB_TRACK_TIME");
        return l && std::atoi(l) != 0;
    }()};
    std::string only; // comma-separated kernel families to time (empty: all)
    struct Pending {
        std::string name;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending;
    std::map<std::string, std::pair<double, long long>> totals;
};
TimerState &timers() {
    static TimerState t;
    return t;
}
std::mutex g_timer_mutex;
void drain_timers() {
    TimerState &t = timers();
    for (auto &p : t.pending) {
        float ms = 0;
        SBX_HIP_CHECK(hipEventSynchronize(p.b));
        SBX_HIP_CHECK(hipEventElapsedTime(&ms, p.a, p.b));
        auto &e = t.totals[p.name];
        e.first += ms;
        e.second += 1;
        (void)hipEventDestroy(p.a);
        (void)hipEventDestroy(p.b);
    }
    t.pending.clear();
}
} // namespace

void timings_enable(bool on) {
    std::lock_guard<std::mutex> g(g_timer_mutex);
    timers().on = on;
}
bool timings_enabled() { return timers().on; }
void timings_reset() {
    std::lock_guard<std::mutex> g(g_timer_mutex);
    drain_timers();
    timers().totals.clear();
}
void timings_get(const char *name, double *ms, long long *calls) {
    std::lock_guard<std::mutex> g(g_timer_mutex);
    drain_timers();
    auto it = timers().totals.find(name);
    *ms = it == timers().totals.end() ? 0.0 : it->second.first;
    *calls = it == timers().totals.end() ? 0 : it->second.second;
}
std::string timings_report() {
    std::lock_guard<std::mutex> g(g_timer_mutex);
    drain_timers();
    std::string r;
    for (auto &e : timers().totals)
        r += e.first + " " + std::to_string(e.second.second) + " " +
             std::to_string(e.second.first) + "\n";
    return r;
}
void timings_filter(const char *names) {
    std::lock_guard<std::mutex> g(g_timer_mutex);
    timers().only = names ? std::string(",") + names + "," : std::string();
}
KernelTimer::KernelTimer(const char *n, hipStream_t s) : name(n), stream(s) {
    if (!timers().on) return; // the common case: no lock per launch
    {
        // the switch and the family filter are written under the lock (timings_enable/filter)
        std::lock_guard<std::mutex> g(g_timer_mutex);
        if (!timers().on) return;
        // each timed launch adds two event records to the stream (~4 us of stream time each)
        if (!timers().only.empty() &&
            timers().only.find(std::string(",") + n + ",") == std::string::npos)
            return;
    }
    hipEvent_t a;
    SBX_HIP_CHECK(hipEventCreate(&a));
    SBX_HIP_CHECK(hipEventRecord(a, s));
    ev0 = a;
}
KernelTimer::~KernelTimer() {
    if (!ev0) return;
    hipEvent_t b;
    if (hipEventCreate(&b) != hipSuccess) return;
    (void)hipEventRecord(b, stream);
    std::lock_guard<std::mutex> g(g_timer_mutex);
    timers().pending.push_back({name, (hipEvent_t)ev0, b});
}

} // namespace sbx
