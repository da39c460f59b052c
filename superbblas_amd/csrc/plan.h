// Host planner: periodic range algebra, partitions and distributed tensor descriptors.
//
// Restated from the reference's behaviour (not its code):
//  * periodic intersections            dist.h:345-558
//  * translate/shift ranges            dist.h:568-653
//  * make_hole                         dist.h:3744-3825
//  * basic_partitioning,
//    partitioning_distributed_procs    dist.h:3264-3509
// All coordinates are handled internally in SlowToFast order; FastToSlow inputs are reversed
// at the API boundary (the reference does the same, e.g. tensor.h:718-727, 1282-1293).
#pragma once

#include <atomic>

#include "sbx_internal.h"

#include <functional>
#include <map>
#include <string>
#include <vector>

namespace sbx {

struct BsrOp;

using Coor = std::vector<int>;

struct Range {
    Coor from, size;
};

inline long volume(const Coor &c) {
    long v = 1;
    for (int x : c) v *= x;
    return v;
}

/// coor mod dim, also for negative values (dist.h:330-333)
inline int normalize_coor(long c, int dim) {
    if (dim == 0) return 0;
    long r = c % dim;
    return (int)(r < 0 ? r + dim : r);
}

/// Strides of a dense array of dims `size` in SlowToFast order (tensor.h:282-297)
inline std::vector<long> strides_slow_to_fast(const Coor &size) {
    std::vector<long> s(size.size());
    long acc = 1;
    for (int i = (int)size.size() - 1; i >= 0; --i) {
        s[i] = acc;
        acc *= size[i];
    }
    return s;
}

/// All ranges resulting from intersecting two ranges on a periodic lattice (dist.h:370-497)
std::vector<Range> intersection(const Range &a, const Range &b, const Coor &dim);
/// Intersect a list of ranges with a range
std::vector<Range> intersection(const std::vector<Range> &as, const Range &b, const Coor &dim);

/// Map a range of tensor A (labels la) to tensor B (labels lb) (translate_range, dist.h:612-634):
/// cB = fromB + (cA - fromA) for common labels, fromB for labels only in B
Range translate(const Range &r, const std::string &la, const Coor &fromA, const Coor &dimA,
                const std::string &lb, const Coor &fromB, const Coor &dimB);

/// Subranges of `r` after removing `hole` (dist.h:3744-3825)
std::vector<Range> make_hole(const Range &r, const Range &hole, const Coor &dim);

/// partitioning_distributed_procs (dist.h:3318-3383)
Coor partitioning_distributed_procs(const std::string &order, const Coor &dim,
                                    const std::string &dist_labels, unsigned nprocs);
/// basic_partitioning with labels (dist.h:3393-3460)
std::vector<Range> basic_partitioning(const char *order, const Coor &dim, const Coor &procs,
                                      const char *dist_labels, int nprocs, int ncomponents);
/// basic_partitioning with extension (dist.h:3475-3509)
std::vector<Range> basic_partitioning_ext(const Coor &dim, const Coor &procs, int nprocs,
                                          bool replicate, const Coor &ext_power);

/// Position of each label of `to` in `from` (-1 if absent) (tensor.h:417-440)
std::vector<int> find_permutation(const std::string &from, const std::string &to);

/// Communicator: nprocs == 1 means a single process (SelfComm, dist.h:142-149)
/// Host all-to-all callback of a host-staged communicator (sbx_alltoallv_fn in sbx.h)
typedef int (*HostAlltoallv)(const void *sendbuf, const unsigned long long *sendbytes,
                             const unsigned long long *senddispls, void *recvbuf,
                             const unsigned long long *recvbytes,
                             const unsigned long long *recvdispls, void *user);

/// Pinned host staging buffers of a host-staged communicator (grown on demand, reused)
struct HostStage {
    void *send = nullptr, *recv = nullptr;
    std::size_t send_cap = 0, recv_cap = 0;
    ~HostStage();
};

struct Comm {
    int nprocs = 1;
    int rank = 0;
    int device = -1;
    void *nccl = nullptr;            // ncclComm_t (RCCL transport: device buffers over xGMI)
    HostAlltoallv host_fn = nullptr; // host-staged transport (e.g. MPI_Alltoallv, gloo)
    void *host_user = nullptr;
    HostStage *stage = nullptr;      // owned by the sbx_comm handle
};

/// A distributed tensor as seen by one process.
///  - `ranges[r]` are the (global, periodic) ranges held by the components of rank r;
///  - `ptr`/`dev` are the local data of this rank's components, dense arrays of
///    `ranges[rank][i].size` elements in label order `labels` (SlowToFast);
///  - dev < 0 means host memory.
struct DistTensor {
    std::string labels;
    Coor dim;
    int dtype = SBX_CDOUBLE;
    std::vector<std::vector<Range>> ranges;
    std::vector<void *> ptr;
    std::vector<int> dev;
    std::vector<const float *> mask; ///< per local component (empty: no masks), copy() only
    int nd() const { return (int)labels.size(); }
    const float *mask_of(int i) const { return mask.empty() ? nullptr : mask[i]; }
};

/// A single-component view used by the local kernels
struct Local {
    void *ptr;
    int dev;
    Coor size; // extents of the box (the view)
    std::string labels;
    int dtype;
    Coor dims; // extents of the dense array the box lies in (empty: the box is the array)
};

//
// Distributed operations (dist.cpp)
//

/// Every rank of `comm` reaches this point before any leaves it (MPI_Barrier)
void comm_barrier(const Comm &comm);
/// Whether every rank passed the same `v` (the answer is the same on every rank)
bool comm_all_equal(const Comm &comm, unsigned long long v);

//
// SB_DEBUG self-checks (debug.cpp; runtime_features.h:24-37)
//
/// SB_DEBUG (read once; the tune key debug.level overrides it)
int debug_level();
extern std::atomic<int> g_debug_level;
/// tune key debug.corrupt_copy (tests of the checks only): > 0 drops that local piece (1-based) of
/// every distributed copy, a deliberately wrong plan
extern std::atomic<int> g_debug_corrupt;
/// Hash of call arguments (check_consistency's Hash, dist.h:513-606)
struct Hasher {
    unsigned long long h = 1469598103934665603ull;
    void add_bytes(const void *p, std::size_t n);
    void add(long v) { add_bytes(&v, sizeof(v)); }
    void add(const Coor &c);
    void add(const std::string &s);
    void add(const Scalar &s);
    void add(const struct DistTensor &t);
};
/// SB_DEBUG >= 1, several ranks: throws on EVERY rank unless every rank hashed the same
/// arguments (check_consistency, dist.h:702-736, which compares with rank 0's hash only and so
/// lets the agreeing ranks run on into an exchange the others never join)
void check_consistency(const Hasher &h, const char *what, const Comm &comm);
/// SB_DEBUG >= 2: run the copy on index-valued size_t mock tensors (same partitions, masks,
/// devices, communicator) and check every destination element exactly (ns_copy_test,
/// dist.h:1919-2116); throws "test_copy_check does not pass!" on a mismatch
void copy_mock_test(const struct DistTensor &src, const Coor &from0, const Coor &size0,
                    const struct DistTensor &dst, const Coor &from1, bool add, const Comm &comm);

/// The contraction's cross-rank sum of partial outputs as one RCCL collective (the
/// reference Adds them with a copy, dist.h:3183-3186, 1364-1404): when every rank holds one
/// partial component (the same range) containing the box [f0, f0 + s0) as a contiguous run, and
/// the destination box is owned by one rank (ncclReduce to it) or whole on every rank
/// (ncclAllReduce), RCCL sums the partials (complex as pairs of reals) into scratch and the
/// owners Add the sum into `dst` by a local copy.  All ranks decide alike from the global
/// partitions.  Returns false, having done nothing, when the shapes do not fit (or the tune key
/// dist.reduce is 0): the caller then Adds through dist_copy (point-to-point sends).
bool dist_reduce_collective(const DistTensor &part, const Coor &f0, const Coor &s0,
                            const DistTensor &dst, const Coor &f1, const Comm &comm);
extern int g_dist_reduce;
extern std::atomic<long long> g_dist_reduce_calls;
/// tune key dist.force_peer: 1 takes the several-GPUs-per-rank path (pack on the origin device,
/// hipMemcpyPeerAsync, unpack on the destination device) for every piece between two components
/// of a rank and for every component away from the communicator's device, even when the devices
/// are the same one -- so that path runs on a 1-GPU box; read-back dist.peer_copies counts the
/// peer copies issued
extern int g_dist_force_peer;
extern std::atomic<long long> g_dist_peer_copies;

/// copy: dst[from1 + P(c - from0)] (=|+=) alpha * src[c] for c in [from0, from0+size0).
/// With `deferred` and other ranks in the exchange, the call returns once the local pieces are
/// issued and the exchange is started (RCCL: packed and sent / received on the side stream;
/// host-staged: packed); *deferred then finishes it (unpack on the library stream after the
/// exchange) -- the reference's Request (dist.h:54-61, 2386-2437).  *deferred stays empty when
/// nothing is left to do.
void dist_copy(const Scalar &alpha, const DistTensor &src, const Coor &from0, const Coor &size0,
               const DistTensor &dst, const Coor &from1, bool add, const Comm &comm,
               std::function<void()> *deferred = nullptr);

/// Host-only argument checks, run before any device work (the reference validates first:
/// tensor.h:495-507 check_isomorphic, tensor.h:623-646 check_dimensions)
void check_copy_args(const std::string &l0, const Coor &from0, const Coor &size0,
                     const Coor &dim0, const std::string &l1, const Coor &from1,
                     const Coor &dim1);
void check_contraction_args(const std::string &l0, const Coor &size0, const std::string &l1,
                            const Coor &size1, const std::string &lr, const Coor &sizer, int t0,
                            int t1, int tr);

/// Element counts of the exchange dist_copy would do on `rank`: send[q] / recv[q] elements to /
/// from rank q (q != rank) and `local` elements moved within the rank (no GPU work)
void copy_plan_counts(const DistTensor &src, const Coor &from0, const Coor &size0,
                      const DistTensor &dst, const Coor &from1, bool add, int rank,
                      std::vector<long> &send, std::vector<long> &recv, long &local);

/// contraction: vr = alpha * contract(v0, v1) + beta * vr over the boxes [from, from+size)
void dist_contraction(const Scalar &alpha, const DistTensor &v0, const Coor &from0,
                      const Coor &size0, bool conj0, const DistTensor &v1, const Coor &from1,
                      const Coor &size1, bool conj1, const Scalar &beta, const DistTensor &vr,
                      const Coor &fromr, const Coor &sizer, const Comm &comm);

/// Local contraction of three dense single-component arrays on one device (GEMM mapping of
/// tensor.h:1475-1598, generalised to arbitrary strides)
void local_contraction(const Scalar &alpha, const Local &x, bool conjx, const Local &y,
                       bool conjy, const Scalar &beta, const Local &r);

//
// Dense batched solvers (dense.cpp, reference dense.h)
//
void dense_cholesky(const DistTensor &v, const std::string &orows, const std::string &ocols,
                    const Comm &comm);
void dense_inversion(const DistTensor &v, const std::string &orows, const std::string &ocols,
                     const Comm &comm);
void dense_solve(bool gesm, const Scalar &alpha, const DistTensor &c, const std::string &orows,
                 const std::string &ocols, const DistTensor &x, const DistTensor &y,
                 const Comm &comm);

//
// Tensor storage, the S3T format (storage.cpp, reference storage.h); storage dims SlowToFast
//
struct StorageCtx;
StorageCtx *storage_create(int dtype, const Coor &dim, const char *filename, const char *meta,
                           int meta_len, int checksum, const Comm &comm);
void storage_read_header(const char *filename, int &dtype, std::string &meta, Coor &dim);
StorageCtx *storage_open(int nd, int dtype, const char *filename, bool allow_writing,
                         const Comm &comm);
void storage_append_blocks(StorageCtx &s, const std::vector<Range> &p0, const std::string &o0,
                           const Coor &from0, const Coor &size0, const Coor &dim0,
                           const std::string &o1, const Coor &from1, const Comm &comm);
void storage_save(StorageCtx &s, const Scalar &alpha, const DistTensor &v, const Coor &from0,
                  const Coor &size0, const std::string &o1, const Coor &from1, const Comm &comm);
void storage_load(StorageCtx &s, const Scalar &alpha, const std::string &o0, const Coor &from0,
                  const Coor &size0, const DistTensor &v, const Coor &from1, const Comm &comm);
std::vector<Range> storage_get_blocks(const StorageCtx &s, const std::string &o0,
                                      const std::string &o1, const Coor &from1,
                                      const Coor &size1);
/// do_write: write the pending checksums; otherwise verify them (check_or_write_checksums)
void storage_checksums(StorageCtx &s, const Comm &comm, bool do_write);
void storage_flush(StorageCtx &s);
void storage_preallocate(StorageCtx &s, std::size_t size);
/// write the pending checksums and free the context
void storage_close(StorageCtx *s, const Comm &comm);

} // namespace sbx
