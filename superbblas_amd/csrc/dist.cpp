// Distributed copy and contraction over partitioned tensors.
//
// Reference behaviour (restated, not translated):
//  * copy_request (dist.h:2264-2438): every (origin component, destination component) pair
//    copies the overlap of their ranges; the pieces on other ranks travel through the remap
//    communicator; `Copy` zeroes destination elements without an origin (has_full_support,
//    dist.h:666-700); `Add` adds the contribution of every origin component.
//  * send_receive (dist.h:1426-1573): pack per destination rank -> MPI_Ialltoallv -> unpack.
//    Here: pack kernels on the device stream -> RCCL grouped ncclSend/ncclRecv (an all-to-all
//    with per-peer byte counts over xGMI) -> unpack kernels, all stream ordered: no host sync.
//  * contraction_normalized (dist.h:3092-3196): scale the output by beta, partition the work
//    like the larger operand (repetitions removed), bring the other operand to that partition,
//    contract locally, reduce the partial outputs into the output with an Add copy.
//
// MI355X-specific choices:
//  * `Copy` pieces are de-duplicated per destination (a replicated origin is read once, the
//    local replica first), which gives the reference's values with less traffic.
//  * operands already laid out so that every label group (T, contracted, free) is a single
//    stride are used in place: no normalising copies (the reference's `reorder_tensor` copies
//    whenever the order differs from its preferred one).
//  * the common single-process case runs the GEMM directly into the output with beta.
#include "plan.h"

#include <rccl/rccl.h>

#include <algorithm>
#include <cassert>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>

namespace sbx {

namespace {

//
// Helpers
//

/// One box to copy between two local arrays
struct Piece {
    int a, b;      // global component index of the origin / destination
    Coor src_from; // local coordinates in the origin component (origin labels)
    Coor dst_from; // local coordinates in the destination component (destination labels)
    Coor size;     // in origin labels
};

struct CompRef {
    int rank, idx; // rank and index within the rank
};

std::vector<CompRef> flatten_components(const DistTensor &t) {
    std::vector<CompRef> r;
    for (int rk = 0; rk < (int)t.ranges.size(); ++rk)
        for (int i = 0; i < (int)t.ranges[rk].size(); ++i) r.push_back({rk, i});
    return r;
}

/// Split a piece where its box wraps around the local (periodic, full-dimension) component
void split_wraps(Piece p, const Coor &src_comp_size, const Coor &dst_comp_size,
                 const std::vector<int> &perm_s2d, std::vector<Piece> &out) {
    for (std::size_t k = 0; k < p.size.size(); ++k) {
        if (p.src_from[k] + p.size[k] > src_comp_size[k]) {
            const int t = src_comp_size[k] - p.src_from[k];
            Piece p1 = p, p2 = p;
            p1.size[k] = t;
            p2.size[k] -= t;
            p2.src_from[k] = 0;
            if (perm_s2d[k] >= 0) {
                const int kd = perm_s2d[k];
                p2.dst_from[kd] = normalize_coor((long)p.dst_from[kd] + t, dst_comp_size[kd]);
            }
            split_wraps(p1, src_comp_size, dst_comp_size, perm_s2d, out);
            split_wraps(p2, src_comp_size, dst_comp_size, perm_s2d, out);
            return;
        }
    }
    for (std::size_t k = 0; k < p.size.size(); ++k) {
        if (perm_s2d[k] < 0) continue;
        const int kd = perm_s2d[k];
        if (p.dst_from[kd] + p.size[k] > dst_comp_size[kd]) {
            const int t = dst_comp_size[kd] - p.dst_from[kd];
            Piece p1 = p, p2 = p;
            p1.size[k] = t;
            p2.size[k] -= t;
            p2.dst_from[kd] = 0;
            p2.src_from[k] = normalize_coor((long)p.src_from[k] + t, src_comp_size[k]);
            split_wraps(p1, src_comp_size, dst_comp_size, perm_s2d, out);
            split_wraps(p2, src_comp_size, dst_comp_size, perm_s2d, out);
            return;
        }
    }
    out.push_back(p);
}

/// Plan all the pieces of a distributed copy (every rank computes the same global list)
std::vector<Piece> plan_copy(const DistTensor &src, const Coor &from0, const Coor &size0,
                             const DistTensor &dst, const Coor &from1, bool add, int my_rank) {
    const std::vector<CompRef> sc = flatten_components(src), dc = flatten_components(dst);
    // perm_s2d[k]: destination dim of origin dim k (-1 if absent)
    std::vector<int> perm_s2d(src.nd(), -1);
    for (int k = 0; k < src.nd(); ++k) {
        auto j = dst.labels.find(src.labels[k]);
        if (j != std::string::npos) perm_s2d[k] = (int)j;
    }
    const Range region0{from0, size0};

    std::vector<Piece> out;
    for (int bi = 0; bi < (int)dc.size(); ++bi) {
        const Range &rb = dst.ranges[dc[bi].rank][dc[bi].idx];
        if (volume(rb.size) == 0) continue;
        // Origin components in priority order: same rank first (for Copy de-duplication)
        std::vector<int> order(sc.size());
        for (int i = 0; i < (int)sc.size(); ++i) order[i] = i;
        if (!add) {
            auto prio = [&](int x) {
                if (sc[x].rank != dc[bi].rank) return 2;
                return sc[x].idx == dc[bi].idx ? 0 : 1;
            };
            std::stable_sort(order.begin(), order.end(),
                             [&](int x, int y) { return prio(x) < prio(y); });
        }
        std::vector<Range> covered; // destination global ranges already assigned (Copy)
        for (int ai : order) {
            const Range &ra = src.ranges[sc[ai].rank][sc[ai].idx];
            if (volume(ra.size) == 0) continue;
            for (const Range &s : intersection(region0, ra, src.dim)) {
                const Range t =
                    translate(s, src.labels, from0, src.dim, dst.labels, from1, dst.dim);
                std::vector<Range> ds = intersection(t, rb, dst.dim);
                if (!add) {
                    // remove what other origins already provide
                    for (const Range &cv : covered) {
                        std::vector<Range> nds;
                        for (const Range &d : ds) {
                            if (intersection(d, cv, dst.dim).empty()) {
                                nds.push_back(d);
                            } else {
                                auto h = make_hole(d, cv, dst.dim);
                                nds.insert(nds.end(), h.begin(), h.end());
                            }
                        }
                        ds.swap(nds);
                    }
                }
                for (const Range &d : ds) {
                    if (volume(d.size) == 0) continue;
                    if (!add) covered.push_back(d);
                    const Range sback =
                        translate(d, dst.labels, from1, dst.dim, src.labels, from0, src.dim);
                    Piece p;
                    p.a = ai;
                    p.b = bi;
                    p.size.resize(src.nd());
                    p.src_from.resize(src.nd());
                    p.dst_from.resize(dst.nd());
                    for (int k = 0; k < src.nd(); ++k) {
                        p.size[k] = perm_s2d[k] >= 0 ? d.size[perm_s2d[k]] : 1;
                        p.src_from[k] =
                            normalize_coor((long)sback.from[k] - ra.from[k], src.dim[k]);
                    }
                    for (int k = 0; k < dst.nd(); ++k)
                        p.dst_from[k] = normalize_coor((long)d.from[k] - rb.from[k], dst.dim[k]);
                    split_wraps(p, ra.size, rb.size, perm_s2d, out);
                }
            }
        }
        (void)my_rank;
    }
    return out;
}

long offset_of(const Coor &from, const std::vector<long> &strides) {
    long o = 0;
    for (std::size_t i = 0; i < from.size(); ++i) o += (long)from[i] * strides[i];
    return o;
}

/// Box copy between two local arrays on the same device
void local_piece_copy(const Scalar &alpha, int src_t, const void *src, const Coor &src_size,
                      const Coor &src_from, int dst_t, void *dst, const Coor &dst_size,
                      const Coor &dst_from, const Coor &box, const std::vector<int> &perm_s2d,
                      bool add, int device, const float *src_mask = nullptr,
                      const float *dst_mask = nullptr) {
    const std::vector<long> ss = strides_slow_to_fast(src_size), ds = strides_slow_to_fast(dst_size);
    BoxCopyDesc d;
    d.src_t = src_t;
    d.dst_t = dst_t;
    d.src = (const char *)src + dtype_size(src_t) * offset_of(src_from, ss);
    d.dst = (char *)dst + dtype_size(dst_t) * offset_of(dst_from, ds);
    if (src_mask) d.src_mask = src_mask + offset_of(src_from, ss);
    if (dst_mask) d.dst_mask = dst_mask + offset_of(dst_from, ds);
    d.size.resize(box.size());
    d.src_stride = ss;
    d.dst_stride.resize(box.size());
    for (std::size_t k = 0; k < box.size(); ++k) {
        d.size[k] = box[k];
        d.dst_stride[k] = perm_s2d[k] >= 0 ? ds[perm_s2d[k]] : 0;
    }
    d.alpha = alpha;
    d.add = add;
    launch_box_copy(d, device);
}

/// Cross-device stream ordering: make `to` wait for the work enqueued so far on `from`
void stream_wait(int from, int to) {
    if (from == to && !g_dist_force_peer) return; // (forced peer path: the events run too)
    hipEvent_t ev;
    set_device(from);
    SBX_HIP_CHECK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    SBX_HIP_CHECK(hipEventRecord(ev, get_stream(from)));
    set_device(to);
    SBX_HIP_CHECK(hipStreamWaitEvent(get_stream(to), ev, 0));
    SBX_HIP_CHECK(hipEventDestroy(ev));
}

void nccl_check(ncclResult_t r, const char *what) {
    if (r != ncclSuccess)
        throw Error(std::string("RCCL error in ") + what + ": " + ncclGetErrorString(r));
}

/// Exchange packed per-peer buffers through the host callback of a host-staged communicator
void host_exchange(const Comm &comm, const void *sdev, const std::vector<std::size_t> &send_bytes,
                   const std::vector<std::size_t> &send_off, void *rdev,
                   const std::vector<std::size_t> &recv_bytes,
                   const std::vector<std::size_t> &recv_off, hipStream_t s) {
    HostStage &st = *comm.stage;
    const std::size_t ns = send_off.back(), nr = recv_off.back();
    if (st.send_cap < ns) {
        if (st.send) SBX_HIP_CHECK(hipHostFree(st.send));
        st.send = nullptr;
        st.send_cap = 0;
        SBX_HIP_CHECK(hipHostMalloc(&st.send, ns, hipHostMallocDefault));
        st.send_cap = ns;
    }
    if (st.recv_cap < nr) {
        if (st.recv) SBX_HIP_CHECK(hipHostFree(st.recv));
        st.recv = nullptr;
        st.recv_cap = 0;
        SBX_HIP_CHECK(hipHostMalloc(&st.recv, nr, hipHostMallocDefault));
        st.recv_cap = nr;
    }
    if (ns) SBX_HIP_CHECK(hipMemcpyAsync(st.send, sdev, ns, hipMemcpyDeviceToHost, s));
    SBX_HIP_CHECK(hipStreamSynchronize(s));
    std::vector<unsigned long long> sb(comm.nprocs), sd(comm.nprocs), rb(comm.nprocs),
        rd(comm.nprocs);
    for (int q = 0; q < comm.nprocs; ++q) {
        const bool self = q == comm.rank;
        sb[q] = self ? 0 : send_bytes[q];
        sd[q] = send_off[q];
        rb[q] = self ? 0 : recv_bytes[q];
        rd[q] = recv_off[q];
    }
    const int rc = comm.host_fn(st.send, sb.data(), sd.data(), st.recv, rb.data(), rd.data(),
                                comm.host_user);
    if (rc != 0) throw Error("copy: the host all-to-all callback failed (" + std::to_string(rc) + ")");
    if (nr) SBX_HIP_CHECK(hipMemcpyAsync(rdev, st.recv, nr, hipMemcpyHostToDevice, s));
}

/// The planner's result for one copy shape: the pieces and whether they cover this rank's
/// destination region (no zero-fill needed).  Cached by shape (the reference caches its copy
/// plans the same way, dist.h:2303-2353), so a repeated copy skips the interval algebra.
struct CopyPlan {
    std::vector<Piece> pieces;
    bool full = true;
};

struct PlanKeyHash {
    std::size_t operator()(const std::vector<long> &k) const {
        std::size_t h = 1469598103934665603ull;
        for (long v : k) h = (h ^ (std::size_t)v) * 1099511628211ull;
        return h;
    }
};

std::mutex g_plan_mutex;
std::unordered_map<std::vector<long>, std::shared_ptr<const CopyPlan>, PlanKeyHash> &plan_cache() {
    static std::unordered_map<std::vector<long>, std::shared_ptr<const CopyPlan>, PlanKeyHash> c;
    return c;
}

void key_tensor(std::vector<long> &k, const DistTensor &t) {
    k.push_back(t.nd());
    for (char c : t.labels) k.push_back(c);
    for (int d : t.dim) k.push_back(d);
    k.push_back((long)t.ranges.size());
    for (const auto &rk : t.ranges) {
        k.push_back((long)rk.size());
        for (const Range &r : rk) {
            for (int v : r.from) k.push_back(v);
            for (int v : r.size) k.push_back(v);
        }
    }
}

std::shared_ptr<const CopyPlan> get_copy_plan(const DistTensor &src, const Coor &from0,
                                              const Coor &size0, const DistTensor &dst,
                                              const Coor &from1, const Range &region1, bool add,
                                              int rank) {
    std::vector<long> key;
    key.reserve(64);
    key.push_back(rank);
    key.push_back(add);
    key_tensor(key, src);
    key_tensor(key, dst);
    for (int v : from0) key.push_back(v);
    for (int v : size0) key.push_back(v);
    for (int v : from1) key.push_back(v);
    {
        std::lock_guard<std::mutex> g(g_plan_mutex);
        auto it = plan_cache().find(key);
        if (it != plan_cache().end()) return it->second;
    }
    auto plan = std::make_shared<CopyPlan>();
    plan->pieces = plan_copy(src, from0, size0, dst, from1, add, rank);
    if (!add) {
        // covered volume per local destination component vs. the region's volume
        const std::vector<CompRef> dc = flatten_components(dst);
        std::vector<long> need(dst.ranges[rank].size(), 0), got(need.size(), 0);
        for (int i = 0; i < (int)need.size(); ++i) {
            const Range &rb = dst.ranges[rank][i];
            if (volume(rb.size) == 0) continue;
            for (const Range &z : intersection(region1, rb, dst.dim)) need[i] += volume(z.size);
        }
        for (const Piece &p : plan->pieces)
            if (dc[p.b].rank == rank) got[dc[p.b].idx] += volume(p.size);
        for (std::size_t i = 0; i < need.size(); ++i) plan->full &= (need[i] == got[i]);
    }
    std::lock_guard<std::mutex> g(g_plan_mutex);
    if (plan_cache().size() >= 4096) plan_cache().clear();
    plan_cache().emplace(std::move(key), plan);
    return plan;
}

} // namespace

void clear_copy_plan_cache() {
    std::lock_guard<std::mutex> g(g_plan_mutex);
    plan_cache().clear();
}

HostStage::~HostStage() {
    if (send) (void)hipHostFree(send);
    if (recv) (void)hipHostFree(recv);
}

//
// Distributed copy
//

void check_copy_args(const std::string &l0, const Coor &from0, const Coor &size0,
                     const Coor &dim0, const std::string &l1, const Coor &from1,
                     const Coor &dim1) {
    if (from0.size() != l0.size() || size0.size() != l0.size() || dim0.size() != l0.size() ||
        from1.size() != l1.size() || dim1.size() != l1.size())
        throw Error("copy: invalid coordinates");
    for (std::size_t k = 0; k < l0.size(); ++k) {
        if (size0[k] < 0 || size0[k] > dim0[k]) throw Error("copy: invalid size0");
        const auto j = l1.find(l0[k]);
        if (j == std::string::npos) {
            if (size0[k] > 1) throw Error("Invalid copy operation");
        } else if (size0[k] > dim1[j]) {
            throw Error("Invalid copy operation");
        }
    }
}

void copy_plan_counts(const DistTensor &src, const Coor &from0, const Coor &size0,
                      const DistTensor &dst, const Coor &from1, bool add, int rank,
                      std::vector<long> &send, std::vector<long> &recv, long &local) {
    const int nprocs = (int)src.ranges.size();
    send.assign(nprocs, 0);
    recv.assign(nprocs, 0);
    local = 0;
    if (volume(size0) == 0) return;
    const std::vector<CompRef> sc = flatten_components(src), dc = flatten_components(dst);
    for (const Piece &p : plan_copy(src, from0, size0, dst, from1, add, rank)) {
        const int ra = sc[p.a].rank, rb = dc[p.b].rank;
        const long n = volume(p.size);
        if (ra == rank && rb == rank) local += n;
        else if (ra == rank) send[rb] += n;
        else if (rb == rank) recv[ra] += n;
    }
}

void dist_copy(const Scalar &alpha, const DistTensor &src, const Coor &from0, const Coor &size0,
               const DistTensor &dst, const Coor &from1, bool add, const Comm &comm,
               std::function<void()> *deferred) {
    if (deferred) *deferred = nullptr;
    if ((int)src.ranges.size() != comm.nprocs || (int)dst.ranges.size() != comm.nprocs)
        throw Error("copy: partition is incompatible with the communicator");
    if (src.nd() != (int)from0.size() || src.nd() != (int)size0.size() ||
        dst.nd() != (int)from1.size())
        throw Error("copy: invalid coordinates");
    // check_isomorphic (tensor.h:495-507): origin labels absent in the destination have size 1
    for (int k = 0; k < src.nd(); ++k) {
        auto j = dst.labels.find(src.labels[k]);
        if (j == std::string::npos) {
            if (size0[k] > 1) throw Error("Invalid copy operation");
        } else if (size0[k] > dst.dim[j]) {
            throw Error("Invalid copy operation");
        }
    }
    if (debug_level() > 0 && comm.nprocs > 1) {
        Hasher h;
        h.add(std::string("copy"));
        h.add(alpha);
        h.add(src);
        h.add(from0);
        h.add(size0);
        h.add(dst);
        h.add(from1);
        h.add((long)add);
        check_consistency(h, "copy", comm);
    }
    copy_mock_test(src, from0, size0, dst, from1, add, comm);
    if (volume(size0) == 0) return;

    const std::vector<CompRef> sc = flatten_components(src), dc = flatten_components(dst);
    std::vector<int> perm_s2d(src.nd(), -1);
    for (int k = 0; k < src.nd(); ++k) {
        auto j = dst.labels.find(src.labels[k]);
        if (j != std::string::npos) perm_s2d[k] = (int)j;
    }

    // Zero the destination region when copying (the reference zeroes it when the origin lacks
    // full support, dist.h:2356-2382; zeroing always is equivalent and simpler)
    const bool zero_all = !add && (alpha.is_zero());
    const Range region1 = translate(Range{from0, size0}, src.labels, from0, src.dim, dst.labels,
                                    from1, dst.dim);
    // local destination components on this rank
    auto zero_region = [&]() {
        for (int i = 0; i < (int)dst.ranges[comm.rank].size(); ++i) {
            const Range &rb = dst.ranges[comm.rank][i];
            if (volume(rb.size) == 0) continue;
            for (const Range &z : intersection(region1, rb, dst.dim)) {
                Piece p;
                p.size = z.size;
                p.dst_from.resize(dst.nd());
                for (int k = 0; k < dst.nd(); ++k)
                    p.dst_from[k] = normalize_coor((long)z.from[k] - rb.from[k], dst.dim[k]);
                p.src_from = p.dst_from;
                std::vector<int> id(dst.nd());
                for (int k = 0; k < dst.nd(); ++k) id[k] = k;
                std::vector<Piece> ps;
                split_wraps(p, rb.size, rb.size, id, ps);
                for (const Piece &q : ps)
                    local_piece_copy(Scalar{0, 0}, dst.dtype, dst.ptr[i], rb.size, q.dst_from,
                                     dst.dtype, dst.ptr[i], rb.size, q.dst_from, q.size, id,
                                     false, dst.dev[i], nullptr, dst.mask_of(i));
            }
        }
    };
    if (zero_all) {
        zero_region();
        return;
    }
    // Add with alpha == 0 leaves the destination untouched (copy_n.h:92, dist.h:2383)
    if (add && alpha.is_zero()) return;

    const std::shared_ptr<const CopyPlan> plan =
        get_copy_plan(src, from0, size0, dst, from1, region1, add, comm.rank);
    const std::vector<Piece> &pieces = plan->pieces;
    // Zero the part of the local destination not covered by any piece
    if (!add && !plan->full) zero_region();

    // Local pieces
    int local_no = 0;
    const int corrupt = g_debug_corrupt.load(std::memory_order_relaxed);
    for (const Piece &p : pieces) {
        const CompRef &ca = sc[p.a], &cb = dc[p.b];
        if (ca.rank != comm.rank || cb.rank != comm.rank) continue;
        if (++local_no == corrupt) continue; // a deliberately wrong plan (debug.corrupt_copy)
        const Range &ra = src.ranges[ca.rank][ca.idx];
        const Range &rb = dst.ranges[cb.rank][cb.idx];
        const int da = src.dev[ca.idx], db = dst.dev[cb.idx];
        if (da == db && !g_dist_force_peer) {
            local_piece_copy(alpha, src.dtype, src.ptr[ca.idx], ra.size, p.src_from, dst.dtype,
                             dst.ptr[cb.idx], rb.size, p.dst_from, p.size, perm_s2d, add, db,
                             src.mask_of(ca.idx), dst.mask_of(cb.idx));
        } else {
            // pack on the origin device, peer copy, unpack on the destination device
            if (CopyTape *t = current_copy_tape()) t->valid = false; // not replayable
            const long n = volume(p.size);
            const std::size_t bytes = n * dtype_size(src.dtype);
            Scratch sbuf(bytes, da);
            std::vector<int> id(src.nd());
            for (int k = 0; k < src.nd(); ++k) id[k] = k;
            local_piece_copy(Scalar{1, 0}, src.dtype, src.ptr[ca.idx], ra.size, p.src_from,
                             src.dtype, sbuf.ptr, p.size, Coor(src.nd(), 0), p.size, id, false, da);
            Scratch dbuf(bytes, db);
            stream_wait(da, db);
            set_device(db);
            SBX_HIP_CHECK(hipMemcpyPeerAsync(dbuf.ptr, db, sbuf.ptr, da, bytes, get_stream(db)));
            ++g_dist_peer_copies;
            local_piece_copy(alpha, src.dtype, dbuf.ptr, p.size, Coor(src.nd(), 0), dst.dtype,
                             dst.ptr[cb.idx], rb.size, p.dst_from, p.size, perm_s2d, add, db,
                             nullptr, dst.mask_of(cb.idx));
            stream_wait(db, da); // keep sbuf alive until the peer copy is done
        }
    }

    if (comm.nprocs == 1) return;

    // Remote pieces: pack per peer, RCCL all-to-all (grouped send/recv), unpack
    const int device = comm.device;
    const std::size_t es = dtype_size(src.dtype);
    std::vector<std::size_t> send_bytes(comm.nprocs, 0), recv_bytes(comm.nprocs, 0);
    for (const Piece &p : pieces) {
        const CompRef &ca = sc[p.a], &cb = dc[p.b];
        if (ca.rank == cb.rank) continue;
        if (ca.rank == comm.rank) send_bytes[cb.rank] += volume(p.size) * es;
        if (cb.rank == comm.rank) recv_bytes[ca.rank] += volume(p.size) * es;
    }
    std::vector<std::size_t> send_off(comm.nprocs + 1, 0), recv_off(comm.nprocs + 1, 0);
    for (int q = 0; q < comm.nprocs; ++q) {
        send_off[q + 1] = send_off[q] + (send_bytes[q] + 255) / 256 * 256;
        recv_off[q + 1] = recv_off[q] + (recv_bytes[q] + 255) / 256 * 256;
    }
    if (!comm.nccl && !(comm.host_fn && comm.stage))
        throw Error("copy: the communicator has no transport");
    std::vector<int> id(src.nd());
    for (int k = 0; k < src.nd(); ++k) id[k] = k;
    set_device(device);
    const hipStream_t main_s = get_stream(device);
    // deferred RCCL exchange: pack, send and receive on the side stream (after the work queued so
    // far on the library stream), so that later library-stream work overlaps the transfer
    const bool side = deferred && comm.nccl;
    const hipStream_t ex_s = side ? get_side_stream(device) : main_s;
    if (side) stream_after(ex_s, main_s);
    auto sbuf = std::make_shared<Scratch>(), rbuf = std::make_shared<Scratch>();
    {
        std::unique_ptr<StreamOverride> so(side ? new StreamOverride(device, ex_s) : nullptr);
        *sbuf = Scratch(send_off[comm.nprocs], device);
        *rbuf = Scratch(recv_off[comm.nprocs], device);
        std::vector<std::size_t> cur(send_off.begin(), send_off.end() - 1);
        for (const Piece &p : pieces) {
            const CompRef &ca = sc[p.a], &cb = dc[p.b];
            if (ca.rank != comm.rank || cb.rank == comm.rank) continue;
            const int da = src.dev[ca.idx];
            char *slot = (char *)sbuf->ptr + cur[cb.rank];
            const std::size_t bytes = volume(p.size) * es;
            cur[cb.rank] += bytes;
            if (da == device && !g_dist_force_peer) {
                local_piece_copy(Scalar{1, 0}, src.dtype, src.ptr[ca.idx],
                                 src.ranges[ca.rank][ca.idx].size, p.src_from, src.dtype, slot,
                                 p.size, Coor(src.nd(), 0), p.size, id, false, device);
                continue;
            }
            // a component on another GPU of this rank (several components per rank, the
            // reference's --components, dist.h:205-241): packed on its own device, then peer-
            // copied (xGMI) into the communicator device's send buffer
            if (CopyTape *t = current_copy_tape()) t->valid = false;
            Scratch tmp(bytes, da);
            local_piece_copy(Scalar{1, 0}, src.dtype, src.ptr[ca.idx],
                             src.ranges[ca.rank][ca.idx].size, p.src_from, src.dtype, tmp.ptr,
                             p.size, Coor(src.nd(), 0), p.size, id, false, da);
            stream_wait(da, device);
            set_device(device);
            SBX_HIP_CHECK(hipMemcpyPeerAsync(slot, device, tmp.ptr, da, bytes, get_stream(device)));
            ++g_dist_peer_copies;
            stream_wait(device, da); // tmp is reused on `da` only after the peer copy
        }
        if (comm.nccl) {
            // RCCL: grouped point-to-point send/recv straight from/to device memory (xGMI)
            ncclComm_t nc = (ncclComm_t)comm.nccl;
            nccl_check(ncclGroupStart(), "ncclGroupStart");
            for (int q = 0; q < comm.nprocs; ++q) {
                if (q == comm.rank) continue;
                if (send_bytes[q] > 0)
                    nccl_check(ncclSend((char *)sbuf->ptr + send_off[q], send_bytes[q], ncclChar,
                                        q, nc, ex_s),
                               "ncclSend");
                if (recv_bytes[q] > 0)
                    nccl_check(ncclRecv((char *)rbuf->ptr + recv_off[q], recv_bytes[q], ncclChar,
                                        q, nc, ex_s),
                               "ncclRecv");
            }
            nccl_check(ncclGroupEnd(), "ncclGroupEnd");
        }
    }
    // completion of the side-stream exchange (shared by the copies of the closure; consumed once)
    auto done = std::make_shared<hipEvent_t>(nullptr);
    if (side) {
        SBX_HIP_CHECK(hipEventCreateWithFlags(done.get(), hipEventDisableTiming));
        SBX_HIP_CHECK(hipEventRecord(*done, ex_s));
    }
    // the rest: (host-staged) exchange through the caller's all-to-all, then the unpack with the
    // destination permutation, alpha and Copy/Add fused, on the library stream
    auto plan_ref = plan;
    const DistTensor src_c = src, dst_c = dst;
    auto finish = [=]() {
        set_device(device);
        const hipStream_t s = get_stream(device);
        if (*done) {
            // the unpack (and the later free of the pack buffers, recorded on this stream)
            // follow the exchange
            SBX_HIP_CHECK(hipStreamWaitEvent(s, *done, 0));
            SBX_HIP_CHECK(hipEventDestroy(*done));
            *done = nullptr;
        }
        if (!comm.nccl)
            // Host-staged: device -> pinned host, the caller's all-to-all, pinned host -> device
            // (the reference's non-GPU-aware MPI path, dist.h:1426-1500)
            host_exchange(comm, sbuf->ptr, send_bytes, send_off, rbuf->ptr, recv_bytes, recv_off, s);
        const std::vector<CompRef> sc2 = flatten_components(src_c), dc2 = flatten_components(dst_c);
        std::vector<std::size_t> cur(recv_off.begin(), recv_off.end() - 1);
        for (const Piece &p : plan_ref->pieces) {
            const CompRef &ca = sc2[p.a], &cb = dc2[p.b];
            if (cb.rank != comm.rank || ca.rank == comm.rank) continue;
            const int db = dst_c.dev[cb.idx];
            const char *slot = (const char *)rbuf->ptr + cur[ca.rank];
            const std::size_t bytes = volume(p.size) * es;
            cur[ca.rank] += bytes;
            if (db == device && !g_dist_force_peer) {
                local_piece_copy(alpha, src_c.dtype, slot, p.size, Coor(src_c.nd(), 0),
                                 dst_c.dtype, dst_c.ptr[cb.idx], dst_c.ranges[cb.rank][cb.idx].size,
                                 p.dst_from, p.size, perm_s2d, add, device, nullptr,
                                 dst_c.mask_of(cb.idx));
                continue;
            }
            // a destination component on another GPU of this rank: peer copy of the received
            // piece to that device, unpacked there
            Scratch tmp(bytes, db);
            stream_wait(device, db);
            set_device(db);
            SBX_HIP_CHECK(hipMemcpyPeerAsync(tmp.ptr, db, slot, device, bytes, get_stream(db)));
            ++g_dist_peer_copies;
            local_piece_copy(alpha, src_c.dtype, tmp.ptr, p.size, Coor(src_c.nd(), 0), dst_c.dtype,
                             dst_c.ptr[cb.idx], dst_c.ranges[cb.rank][cb.idx].size, p.dst_from,
                             p.size, perm_s2d, add, db, nullptr, dst_c.mask_of(cb.idx));
            stream_wait(db, device); // the receive buffer outlives the peer copy
            set_device(device);
        }
    };
    if (deferred)
        *deferred = finish;
    else
        finish();
}

int g_dist_force_peer = 0;
std::atomic<long long> g_dist_peer_copies{0};
int g_dist_reduce = 1; // tune key dist.reduce: 1 collective reductions where they fit, 0 never
std::atomic<long long> g_dist_reduce_calls{0}; // read-back dist.reduce_calls: collectives issued

bool dist_reduce_collective(const DistTensor &part, const Coor &f0, const Coor &s0,
                            const DistTensor &dst, const Coor &f1, const Comm &comm) {
    if (!comm.nccl || comm.nprocs < 2 || g_dist_reduce <= 0) return false;
    ncclDataType_t nt;
    int reals = 1;
    switch (part.dtype) {
    case SBX_CDOUBLE: nt = ncclDouble; reals = 2; break;
    case SBX_DOUBLE: nt = ncclDouble; break;
    case SBX_CFLOAT: nt = ncclFloat; reals = 2; break;
    case SBX_FLOAT: nt = ncclFloat; break;
    default: return false;
    }
    if (part.dtype != dst.dtype || volume(s0) == 0 || (int)part.ranges.size() != comm.nprocs ||
        (int)dst.ranges.size() != comm.nprocs)
        return false;
    const int nd = part.nd();
    // every rank: one partial component, the same range, holding the box as one contiguous run
    // (the box spans the component in every dimension but the slowest)
    const Range &r0 = part.ranges[0].size() == 1 ? part.ranges[0][0] : Range{};
    if (part.ranges[0].size() != 1) return false;
    for (int q = 1; q < comm.nprocs; ++q)
        if (part.ranges[q].size() != 1 || part.ranges[q][0].from != r0.from ||
            part.ranges[q][0].size != r0.size)
            return false;
    Coor off(nd, 0);
    for (int d = 0; d < nd; ++d) {
        off[d] = normalize_coor((long)f0[d] - r0.from[d], part.dim[d]);
        if (off[d] + s0[d] > r0.size[d]) return false;
        if (d > 0 && (off[d] != 0 || s0[d] != r0.size[d])) return false;
    }
    // the destination box: owned by one rank (reduce) or whole on every rank (all-reduce)
    Coor size1(dst.nd(), 1);
    for (int d = 0; d < nd; ++d) {
        const auto j = dst.labels.find(part.labels[d]);
        if (j == std::string::npos) return false;
        size1[j] = s0[d];
    }
    const Range box1{f1, size1};
    const long vbox = volume(size1);
    int owners = 0, root = -1, whole = 0;
    for (int q = 0; q < comm.nprocs; ++q) {
        long covered = 0;
        for (const Range &r : dst.ranges[q])
            for (const Range &x : intersection(r, box1, dst.dim)) covered += volume(x.size);
        if (covered > 0) {
            ++owners;
            root = q;
        }
        if (covered == vbox && dst.ranges[q].size() == 1) ++whole;
    }
    const bool all = whole == comm.nprocs;
    if (!(owners == 1 || all)) return false;
    const int device = comm.device;
    set_device(device);
    const hipStream_t s = get_stream(device);
    const std::size_t es = dtype_size(part.dtype);
    const long n = volume(s0);
    const std::vector<long> st = strides_slow_to_fast(r0.size);
    const char *send = (const char *)part.ptr[0] + es * offset_of(off, st);
    const bool mine = all || comm.rank == root;
    Scratch sum(mine ? n * es : 0, device);
    ncclComm_t nc = (ncclComm_t)comm.nccl;
    ++g_dist_reduce_calls;
    if (all)
        nccl_check(ncclAllReduce(send, sum.ptr, (size_t)n * reals, nt, ncclSum, nc, s),
                   "ncclAllReduce");
    else
        nccl_check(ncclReduce(send, mine ? sum.ptr : nullptr, (size_t)n * reals, nt, ncclSum, root,
                              nc, s),
                   "ncclReduce");
    if (!mine) return true;
    // Add the sum into this rank's destination components (a local copy: one process, one box)
    DistTensor sl;
    sl.labels = part.labels;
    sl.dim = part.dim;
    sl.dtype = part.dtype;
    sl.ranges = {{Range{f0, s0}}};
    sl.ptr = {sum.ptr};
    sl.dev = {device};
    DistTensor dl;
    dl.labels = dst.labels;
    dl.dim = dst.dim;
    dl.dtype = dst.dtype;
    dl.ranges = {dst.ranges[comm.rank]};
    dl.ptr = dst.ptr;
    dl.dev = dst.dev;
    dl.mask = dst.mask;
    Comm self;
    self.device = device;
    dist_copy(Scalar{1, 0}, sl, f0, s0, dl, f1, true, self);
    return true;
}

bool comm_all_equal(const Comm &comm, unsigned long long v) {
    if (comm.nprocs <= 1) return true;
    if (comm.nccl) {
        // one all-reduce (max) of (v, ~v): every rank learns max(v) and ~min(v)
        set_device(comm.device);
        hipStream_t s = get_stream(comm.device);
        unsigned long long h[2] = {v, ~v};
        Scratch buf(sizeof(h), comm.device);
        SBX_HIP_CHECK(hipMemcpyAsync(buf.ptr, h, sizeof(h), hipMemcpyHostToDevice, s));
        nccl_check(ncclAllReduce(buf.ptr, buf.ptr, 2, ncclUint64, ncclMax, (ncclComm_t)comm.nccl, s),
                   "ncclAllReduce");
        SBX_HIP_CHECK(hipMemcpyAsync(h, buf.ptr, sizeof(h), hipMemcpyDeviceToHost, s));
        SBX_HIP_CHECK(hipStreamSynchronize(s));
        return h[0] == ~h[1];
    }
    if (!comm.host_fn) throw Error("the communicator has no transport");
    // every rank sends its value to every other rank through the caller's all-to-all
    std::vector<unsigned long long> sn(comm.nprocs, sizeof(v)), sd(comm.nprocs, 0),
        rn(comm.nprocs, sizeof(v)), rd(comm.nprocs), all(comm.nprocs, v);
    sn[comm.rank] = rn[comm.rank] = 0;
    for (int q = 0; q < comm.nprocs; ++q) rd[q] = q * sizeof(v);
    const int rc = comm.host_fn(&v, sn.data(), sd.data(), all.data(), rn.data(), rd.data(),
                                comm.host_user);
    if (rc != 0) throw Error("the host all-to-all callback failed (" + std::to_string(rc) + ")");
    for (unsigned long long x : all)
        if (x != v) return false;
    return true;
}

void comm_barrier(const Comm &comm) {
    if (comm.nprocs <= 1) return;
    if (comm.nccl) {
        // a one-element all-reduce on the communicator's device, waited for on the host
        set_device(comm.device);
        hipStream_t s = get_stream(comm.device);
        Scratch one(sizeof(int), comm.device);
        SBX_HIP_CHECK(hipMemsetAsync(one.ptr, 0, sizeof(int), s));
        nccl_check(ncclAllReduce(one.ptr, one.ptr, 1, ncclInt, ncclSum, (ncclComm_t)comm.nccl, s),
                   "ncclAllReduce");
        SBX_HIP_CHECK(hipStreamSynchronize(s));
    } else if (comm.host_fn) {
        // one byte to and from every peer through the caller's all-to-all
        std::vector<unsigned long long> n(comm.nprocs, 1), d(comm.nprocs);
        for (int q = 0; q < comm.nprocs; ++q) d[q] = q;
        n[comm.rank] = 0;
        std::vector<char> sbuf(comm.nprocs, 0), rbuf(comm.nprocs, 0);
        const int rc = comm.host_fn(sbuf.data(), n.data(), d.data(), rbuf.data(), n.data(),
                                    d.data(), comm.host_user);
        if (rc != 0) throw Error("the host all-to-all callback failed (" + std::to_string(rc) + ")");
    } else {
        throw Error("the communicator has no transport");
    }
}

} // namespace sbx
