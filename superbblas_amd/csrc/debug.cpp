// SB_DEBUG self-checks (the reference's debug mode, runtime_features.h:24-37):
//  * level >= 1: every rank's call arguments are hashed and compared across the communicator
//    (check_consistency, dist.h:702-736) -- a rank making a different collective call is caught
//    before it can deadlock an exchange;
//  * level >= 2: every copy first runs on index-valued size_t mock tensors through the same
//    planner, pack / exchange / unpack and kernels, and the destination is checked exactly,
//    periodic wraps, Add multiplicity of replicated origins and masks included
//    (ns_copy_test, dist.h:1919-2116, triggered at dist.h:2282-2285).
// Deviation, on purpose: the reference's check_consistency constructs its error without throwing
// it (dist.h:735); here a mismatch throws.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <sstream>

#include "plan.h"

namespace sbx {

namespace {
int env_debug_level() {
    const char *l = std::getenv("SB_DEBUG");
    return l ? std::max(0, std::atoi(l)) : 0;
}
thread_local bool t_in_mock = false; // the mock copy itself is not tested again
} // namespace

std::atomic<int> g_debug_level{env_debug_level()};
std::atomic<int> g_debug_corrupt{0};

int debug_level() { return g_debug_level.load(std::memory_order_relaxed); }

//
// check_consistency
//

void Hasher::add_bytes(const void *p, std::size_t n) {
    // FNV-1a, 64 bit
    const unsigned char *c = (const unsigned char *)p;
    for (std::size_t i = 0; i < n; ++i) {
        h ^= c[i];
        h *= 1099511628211ull;
    }
}
void Hasher::add(const Coor &c) {
    add((long)c.size());
    for (int x : c) add((long)x);
}
void Hasher::add(const std::string &s) {
    add((long)s.size());
    add_bytes(s.data(), s.size());
}
void Hasher::add(const Scalar &s) {
    add_bytes(&s.re, sizeof(double));
    add_bytes(&s.im, sizeof(double));
}
void Hasher::add(const DistTensor &t) {
    add(t.labels);
    add(t.dim);
    add((long)t.dtype);
    add((long)t.ranges.size());
    for (const auto &rk : t.ranges) {
        add((long)rk.size());
        for (const Range &r : rk) {
            add(r.from);
            add(r.size);
        }
    }
    add((long)!t.mask.empty());
}

void check_consistency(const Hasher &h, const char *what, const Comm &comm) {
    if (debug_level() <= 0 || comm.nprocs <= 1) return;
    if (!comm_all_equal(comm, h.h + (unsigned long long)comm.nprocs))
        throw Error(std::string("check_consistency failed! (") + what + ": the ranks were called "
                    "with different arguments; seen on rank " + std::to_string(comm.rank) + ")");
}

//
// Mock-index copy test
//

namespace {

/// The global SlowToFast index of every element of a component of `t` (range r), periodic
std::vector<unsigned long long> global_indices(const Range &r, const Coor &dim) {
    const long n = volume(r.size);
    std::vector<unsigned long long> out(n);
    const int nd = (int)dim.size();
    const std::vector<long> gst = strides_slow_to_fast(dim);
    std::vector<int> c(nd, 0);
    for (long i = 0; i < n; ++i) {
        unsigned long long g = 0;
        for (int d = 0; d < nd; ++d) g += (unsigned long long)normalize_coor((long)r.from[d] + c[d], dim[d]) * gst[d];
        out[i] = g;
        for (int d = nd - 1; d >= 0; --d) {
            if (++c[d] < r.size[d]) break;
            c[d] = 0;
        }
    }
    return out;
}

bool in_interval(const Coor &from, const Coor &size, const Coor &dim, const Coor &c) {
    for (std::size_t d = 0; d < c.size(); ++d)
        if (normalize_coor((long)c[d] - from[d], dim[d]) >= size[d]) return false;
    return true;
}

} // namespace

void copy_mock_test(const DistTensor &src, const Coor &from0, const Coor &size0,
                    const DistTensor &dst, const Coor &from1, bool add, const Comm &comm) {
    if (debug_level() < 2 || t_in_mock || volume(size0) == 0) return;
    struct Flag {
        Flag() { t_in_mock = true; }
        ~Flag() { t_in_mock = false; }
    } flag;
    const int nd0 = src.nd(), nd1 = dst.nd();
    // the mock tensors: same partitions, masks and devices, size_t values
    DistTensor s = src, d = dst;
    s.dtype = d.dtype = SBX_SIZE_T;
    std::vector<Scratch> bufs;
    bufs.reserve(s.ptr.size() + d.ptr.size());
    for (std::size_t i = 0; i < s.ptr.size(); ++i) {
        const Range &r = src.ranges[comm.rank][i];
        const std::vector<unsigned long long> g = global_indices(r, src.dim);
        bufs.emplace_back(g.size() * 8, s.dev[i]);
        s.ptr[i] = bufs.back().ptr;
        if (!g.empty()) {
            set_device(s.dev[i]);
            SBX_HIP_CHECK(hipMemcpyAsync(s.ptr[i], g.data(), g.size() * 8, hipMemcpyHostToDevice,
                                         get_stream(s.dev[i])));
            SBX_HIP_CHECK(hipStreamSynchronize(get_stream(s.dev[i])));
        }
    }
    for (std::size_t i = 0; i < d.ptr.size(); ++i) {
        const std::size_t bytes = volume(dst.ranges[comm.rank][i].size) * 8;
        bufs.emplace_back(bytes, d.dev[i]);
        d.ptr[i] = bufs.back().ptr;
        if (bytes) launch_zero(d.ptr[i], bytes, d.dev[i]);
    }
    dist_copy(Scalar{1, 0}, s, from0, size0, d, from1, add, comm);

    // expected values (test_copy_check, dist.h:1997-2044)
    std::vector<int> perm1(nd0, -1); // position in dst of each src label
    for (int k = 0; k < nd0; ++k) {
        auto j = dst.labels.find(src.labels[k]);
        if (j != std::string::npos) perm1[k] = (int)j;
    }
    Coor size1(nd1, 1);
    for (int k = 0; k < nd0; ++k)
        if (perm1[k] >= 0) size1[perm1[k]] = size0[k];
    const std::vector<long> st0 = strides_slow_to_fast(src.dim);
    // the first mismatch of this rank; every rank learns whether any rank failed before throwing
    // (a rank throwing alone would leave the others in the real copy's exchange)
    std::string fail;
    for (std::size_t i = 0; i < d.ptr.size() && fail.empty(); ++i) {
        const Range &rb = dst.ranges[comm.rank][i];
        const long n = volume(rb.size);
        if (n == 0) continue;
        std::vector<unsigned long long> got(n);
        std::vector<float> mask;
        set_device(d.dev[i]);
        SBX_HIP_CHECK(hipStreamSynchronize(get_stream(d.dev[i])));
        SBX_HIP_CHECK(hipMemcpy(got.data(), d.ptr[i], n * 8, hipMemcpyDeviceToHost));
        if (const float *m = dst.mask_of((int)i)) {
            mask.resize(n);
            SBX_HIP_CHECK(hipMemcpy(mask.data(), m, n * sizeof(float), hipMemcpyDeviceToHost));
        }
        Coor lc(nd1, 0), c1(nd1), c0(nd0);
        for (long e = 0; e < n; ++e) {
            for (int j = 0; j < nd1; ++j) c1[j] = normalize_coor((long)rb.from[j] + lc[j], dst.dim[j]);
            unsigned long long want = 0;
            if (in_interval(from1, size1, dst.dim, c1)) {
                for (int k = 0; k < nd0; ++k)
                    c0[k] = perm1[k] < 0 ? from0[k]
                                         : normalize_coor((long)from0[k] + c1[perm1[k]] - from1[perm1[k]],
                                                          src.dim[k]);
                unsigned long long idx = 0;
                for (int k = 0; k < nd0; ++k) idx += (unsigned long long)c0[k] * st0[k];
                int rep = 0;
                for (const auto &rk : src.ranges)
                    for (const Range &r : rk)
                        if (volume(r.size) > 0 && in_interval(r.from, r.size, src.dim, c0)) ++rep;
                want = add ? idx * rep : (rep == 0 ? 0 : idx);
                if (!mask.empty() && mask[e] == 0) want = 0;
            }
            if (got[e] != want) {
                std::ostringstream os;
                os << "test_copy_check does not pass! (SB_DEBUG mock-index copy check: rank "
                   << comm.rank << ", destination component " << i << ", coordinate (";
                for (int j = 0; j < nd1; ++j) os << (j ? "," : "") << c1[j];
                os << ") of '" << dst.labels << "' holds " << got[e] << ", expected " << want << ")";
                fail = os.str();
                break;
            }
            for (int j = nd1 - 1; j >= 0; --j) {
                if (++lc[j] < rb.size[j]) break;
                lc[j] = 0;
            }
        }
    }
    const bool ok = fail.empty();
    if (!comm_all_equal(comm, ok ? 1ull : 0ull) && ok)
        throw Error("test_copy_check does not pass! (SB_DEBUG mock-index copy check failed on "
                    "another rank)");
    if (!ok) throw Error(fail);
}

} // namespace sbx
