// Device runtime: per-device library streams and the stream-ordered scratch pool.
//
// Reference: platform.h:173-221 (Gpu context), 304-409 (stream helpers), 448-467
// (getGpuAllocStream: every GPU op of a device is enqueued on one library stream) and
// alloc.h:91-391 (hipMallocAsync on the alloc stream + a cached scratch-buffer pool).
// On ROCm the stream-ordered allocator already is a caching pool; raising its release
// threshold keeps freed scratch resident so steady-state calls do no driver allocations.
#include "sbx_internal.h"

#include <map>
#include <mutex>

namespace sbx {

namespace {
struct DeviceState {
    hipStream_t own = nullptr;  // stream created by the library
    hipStream_t side = nullptr; // second library stream (overlapped exchanges)
    hipStream_t user = nullptr; // stream set by the caller (sbx_stream_set); may be the null stream
    bool has_user = false;
    bool pool_configured = false;
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

void *scratch_alloc(std::size_t bytes, int device) {
    if (bytes == 0) return nullptr;
    set_device(device);
    {
        std::lock_guard<std::mutex> g(g_mutex);
        DeviceState &st = state(device);
        if (!st.pool_configured) {
            hipMemPool_t pool;
            if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) {
                uint64_t threshold = UINT64_MAX;
                (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &threshold);
            }
            st.pool_configured = true;
        }
    }
    void *p = nullptr;
    hipError_t e = hipMallocAsync(&p, bytes, get_stream(device));
    if (e != hipSuccess) {
        // Mirror alloc.h:104-168: release the cached memory and retry once
        (void)hipGetLastError();
        (void)hipStreamSynchronize(get_stream(device));
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess) (void)hipMemPoolTrimTo(pool, 0);
        SBX_HIP_CHECK(hipMallocAsync(&p, bytes, get_stream(device)));
    }
    return p;
}

void scratch_free(void *p, int device) {
    if (!p) return;
    set_device(device);
    SBX_HIP_CHECK(hipFreeAsync(p, get_stream(device)));
}

void trim_pools() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return;
    for (int d = 0; d < n && d < (int)states().size(); ++d) {
        (void)hipSetDevice(d);
        (void)hipDeviceSynchronize();
        hipMemPool_t pool;
        if (hipDeviceGetDefaultMemPool(&pool, d) == hipSuccess) (void)hipMemPoolTrimTo(pool, 0);
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
    bool on = false;
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
KernelTimer::KernelTimer(const char *n, hipStream_t s) : name(n), stream(s) {
    if (!timers().on) return;
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
