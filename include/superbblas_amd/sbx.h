/*
 * sbx.h -- C ABI of superbblas_amd, the MI355X-native implementation of superbblas's
 * distributed tensor-contraction hot path.
 *
 * This is the drop-in boundary.  The reference (eromero-vlc/superbblas) exposes a header-only
 * C++ template API (include/superbblas.h); `include/superbblas.h` in this repository keeps those
 * exact template signatures and flattens the compile-time ranks into the runtime descriptors
 * below.  Every entry point returns SBX_OK (0) on success or a negative status; the message of
 * the last failure is available from sbx_last_error() (the C++ layer rethrows it as
 * std::runtime_error, matching the reference's error behaviour, platform.h:226-243).
 *
 * Conventions shared by all entry points
 *  - Coordinates and sizes are `int` (reference `IndexType`, tensor.h:47-52).
 *  - A partition array for a tensor of rank N is `nprocs*ncomponents` items of {from[N],size[N]},
 *    i.e. the memory image of `std::vector<PartitionItem<N>>` (dist.h:39-45, 3251-3261).
 *  - Labels are strings of one character per dimension (tensor.h:265-276).
 *  - `co` is SBX_SLOW_TO_FAST or SBX_FAST_TO_SLOW (tensor.h:56-60).
 *  - Scalars (alpha, beta) are passed as two doubles {re, im}; the imaginary part is ignored
 *    for real types.
 *  - Tensor data pointers are caller-owned device (or host) pointers; the library never frees
 *    them (blas.h:268-269).  All GPU work is enqueued on the library stream of each device
 *    (platform.h:448-467); call sbx_sync() before reading results on the host.
 *  - `comm` is NULL for a single process (reference SelfComm, dist.h:142-149) or a communicator
 *    created by sbx_comm_create (replaces MPI_Comm; RCCL over xGMI underneath).
 *  - `session` must be 0 (cache.h:269).  Masks are not supported (pass NULL).
 */
#ifndef SUPERBBLAS_AMD_SBX_H
#define SUPERBBLAS_AMD_SBX_H

#ifdef __cplusplus
extern "C" {
#endif

#define SBX_OK 0
#define SBX_ERROR (-1)

/* Scalar types (reference supported_type, blas.h:57-65 / performance.h:29-48) */
enum sbx_dtype { SBX_FLOAT = 0, SBX_DOUBLE = 1, SBX_CFLOAT = 2, SBX_CDOUBLE = 3, SBX_INT = 4, SBX_SIZE_T = 5 };
/* CoorOrder (tensor.h:56-60) */
enum sbx_coor_order { SBX_SLOW_TO_FAST = 0, SBX_FAST_TO_SLOW = 1 };
/* CopyAdd (tensor.h:62-66) */
enum sbx_copy_add { SBX_COPY = 0, SBX_ADD = 1 };
/* MatrixLayout (bsr.h:28-31) */
enum sbx_matrix_layout { SBX_ROW_MAJOR = 0, SBX_COLUMN_MAJOR = 1 };
/* platform (platform.h:105-109); CUDA does not exist here, HIP == GPU */
enum sbx_platform { SBX_CPU = 0, SBX_GPU = 1 };

/* Context{plat, device} (platform.h:757-773) */
typedef struct sbx_context {
    int plat;
    int device;
} sbx_context;

typedef struct sbx_comm_s *sbx_comm; /* replaces MPI_Comm (dist.h:120-149) */
typedef struct sbx_bsr_s *sbx_bsr;   /* replaces BSR_handle* (bsr.h:34-52) */
typedef struct sbx_storage_s *sbx_storage; /* replaces Storage_handle (storage.h:2127) */

/* ---- errors / runtime (platform.h:757-841, blas.h:965-988, alloc.h:398-443) ---- */

/* Message of the last failed call on this thread */
const char *sbx_last_error(void);
/* Library version {major, minor} (version.h:4-5) */
int sbx_version(int *major, int *minor);
/* getGpuDevicesCount (platform.h:818-825) */
int sbx_get_gpu_devices_count(int *n);
/* sync(Context) (blas.h:965-974) */
int sbx_sync(sbx_context ctx);
/* The stream all work of `device` is enqueued on (getGpuAllocStream, platform.h:448-467) */
int sbx_stream_get(int device, void **stream);
/* Enqueue the work of `device` on a caller-owned hipStream_t (NULL = the null stream) */
int sbx_stream_set(int device, void *stream);
/* Go back to the library's own (non-blocking) stream of `device` */
int sbx_stream_reset(int device);
/* clearCaches (alloc.h:437-443): release cached plans and scratch memory */
int sbx_clear_caches(void);
/* clearHandles (platform.h:828-838): destroy library streams and communicator handles */
int sbx_clear_handles(void);
/* allocate / deallocate (alloc.h:398-430) on a context */
int sbx_allocate(unsigned long long bytes, sbx_context ctx, void **ptr);
int sbx_deallocate(void *ptr, sbx_context ctx);

/* ---- memory (getCustomAllocator / getCustomDeallocator platform.h:129-139,
   allocate_from_cache alloc.h:428-435, reportCacheUsage / checkForMemoryLeaks
   performance.h:436-518) ---- */
typedef void *(*sbx_alloc_fn)(unsigned long long bytes, int device, void *user);
typedef void (*sbx_free_fn)(void *ptr, int device, void *user);
/* Device memory the library allocates (sbx_allocate on GPU contexts and its scratch cache) comes
   from `alloc` / goes back to `dealloc` (both NULL: hipMalloc / hipFree).  Cached blocks of the
   previous allocator are released first. */
int sbx_set_custom_allocator(sbx_alloc_fn alloc, sbx_free_fn dealloc, void *user);
/* A buffer of the library's scratch cache, ordered on the library stream of the device */
int sbx_allocate_from_cache(unsigned long long bytes, sbx_context ctx, void **ptr);
int sbx_release_to_cache(void *ptr, sbx_context ctx);
/* Bytes of `device` held by the scratch cache: idle blocks and blocks in use */
int sbx_cache_usage(int device, unsigned long long *cached, unsigned long long *live);

/* ---- kernel timers (reportTimings / resetTimings, performance.h:356-518) ----
   When enabled, every GPU kernel family ("gemm", "gemm_splitk_reduce", "copy", "bsr") is
   bracketed by HIP events on the stream it is launched on; totals are summed on query. */
int sbx_timings_enable(int on);
int sbx_timings_reset(void);
/* time only these kernel families ("gemm,copy"; NULL or "" = all): each timed launch adds two
   event records to its stream */
int sbx_timings_filter(const char *names);
/* total milliseconds and launch count of one kernel family (synchronizes its events) */
int sbx_timings_get(const char *name, double *ms, long long *calls);
/* "name calls total_ms" per line into buf (truncated to len-1 chars) */
int sbx_timings_report(char *buf, int len);

/* ---- tuning hook (no reference counterpart) ----
   Override a kernel-shape choice of the library for tuning / comparison runs.  The defaults are
   the measured winners; read a key with sbx_tune_get before changing it to
   restore it afterwards.  Keys: "gemm.m3", "gemm.splits", "gemm.max_bytes", "gemm.t48",
   "gemm.share_ab", "gemm.loaders", "gemm.dma_spread", "gemm.skinny", "copy.nt", "copy.budget", "copy.run", "copy.max_elems", "copy.pair",
   "copy.order", "copy.trans", "copy.btrans", "bsr.variant", "bsr.row_max_cols", "bsr.split_max_cols",
   "bsr.split_cw", "bsr.split_jb", "bsr.split_ilv", "bsr.kron_mfma", "bsr.kron_mfma_min_cols",
   "bsr.kron_pack", "bsr.kron_xlds", "bsr.kron_ylds", "bsr.nt", "bsr.blk_pd", "dense.wave", "dist.reduce" (must be set alike on every rank: the ranks' reductions must
   match; SB_DEBUG >= 1 checks it), "dist.force_peer" (1: the several-GPUs-per-rank path -- pack, hipMemcpyPeerAsync, unpack -- for every piece between components of a rank even on one device), "alloc.max_cached", "debug.level" (overrides SB_DEBUG),
   "debug.corrupt_copy" (tests of the SB_DEBUG checks: drop that local piece of every copy); read-backs "bsr.last_kernel", "dist.peer_copies",
   "copy.last_pair", "dist.reduce_calls", "alloc.cross_stream_frees".  Unknown keys fail with an
   error. */
int sbx_tune_set(const char *key, long long value);
/* The box-copy kernel the library's planner picks for an N-d box copy (sizes and element strides
   of both sides, element types, Copy/Add, masked): *kind 0 masked, 1 contiguous, 2 direct
   gather, 3 LDS tile, 4 site-block transpose, 5 block transpose, -1 empty box; *blocks its grid.
   Host only (no GPU work): lets the planner be tested on machines without a GPU. */
int sbx_copy_kernel_plan(int nd, const long long *size, const long long *src_stride,
                         const long long *dst_stride, int t0, int t1, int add, int masked,
                         int *kind, long long *blocks);
int sbx_tune_get(const char *key, long long *value);

/* ---- communicator (replaces MPI; dist.h:1426-1773 send_receive) ---- */

/* Fill `id` (128 bytes) with a fresh RCCL unique id; call on one rank and broadcast it */
int sbx_comm_unique_id(unsigned char *id);
/* Create the communicator of `nprocs` ranks; `device` is this rank's GPU */
int sbx_comm_create(int nprocs, int rank, const unsigned char *id, int device, sbx_comm *comm);
/* Host all-to-all exchange: send sendbytes[q] bytes at sendbuf+senddispls[q] to rank q and
   receive recvbytes[q] bytes from rank q into recvbuf+recvdispls[q] (MPI_Alltoallv with byte
   counts); returns 0 on success.  Buffers are pinned host memory owned by the library. */
typedef int (*sbx_alltoallv_fn)(const void *sendbuf, const unsigned long long *sendbytes,
                                const unsigned long long *senddispls, void *recvbuf,
                                const unsigned long long *recvbytes,
                                const unsigned long long *recvdispls, void *user);
/* Communicator whose exchanges are staged through pinned host memory and `fn` (the reference's
   non-GPU-aware MPI path, dist.h:1426-1500: pack on the device, copy to the host, alltoallv,
   copy back, unpack).  Lets an MPI application keep its MPI_Comm (wrap MPI_Alltoallv) and lets
   several ranks share one GPU, which RCCL refuses. */
int sbx_comm_create_host(int nprocs, int rank, int device, sbx_alltoallv_fn fn, void *user,
                         sbx_comm *comm);
int sbx_comm_rank(sbx_comm comm, int *rank, int *nprocs);
/* What carries the exchanges: kind 0 = none (one rank), 1 = RCCL (count / user_rank from
   ncclCommCount / ncclCommUserRank, i.e. what RCCL itself sees), 2 = host-staged callback */
int sbx_comm_transport(sbx_comm comm, int *kind, int *count, int *user_rank);
int sbx_comm_destroy(sbx_comm comm);

/* ---- partitioning helpers (dist.h:3318-3509, 3744-3825) ---- */

/* partitioning_distributed_procs (dist.h:3318-3383): procs[nd] out */
int sbx_partitioning_distributed_procs(int nd, const char *order, const int *dim,
                                       const char *dist_labels, int nprocs, int *procs);
/* basic_partitioning(order, dim, procs, dist_labels, nprocs, ncomponents) (dist.h:3393-3460);
   out must hold max(nprocs, prod(procs))*ncomponents items of 2*nd ints */
int sbx_basic_partitioning(int nd, const char *order, const int *dim, const int *procs,
                           const char *dist_labels, int nprocs, int ncomponents, int *out);
/* basic_partitioning(dim, procs, nprocs, replicate, ext_power) (dist.h:3475-3509) */
int sbx_basic_partitioning_ext(int nd, const int *dim, const int *procs, int nprocs,
                               int replicate, const int *ext_power, int *out);
/* make_hole(from, size, hole_from, hole_size, dim) (dist.h:3802-3825); out holds up to maxout
   items of 2*nd ints (periodic wraps can split the result into more than nd boxes; 4*nd*2^nd is a
   safe bound), *nout receives the count */
int sbx_make_hole(int nd, const int *from, const int *size, const int *hole_from,
                  const int *hole_size, const int *dim, int maxout, int *out, int *nout);

/* ---- copy (dist.h:3583-3602 no-MPI / 3534-3558 MPI) ----
   v1[from1 + P(c - from0)] (=|+=) alpha * v0[c] for c in [from0, from0+size0) (periodic),
   P maps labels o0 -> o1; t0 -> t1 element conversion. */
int sbx_copy(int nd0, int nd1, const double *alpha, int t0, int t1,
             const int *p0, int ncomponents0, const char *o0, const int *from0, const int *size0,
             const int *dim0, const void *const *v0, const sbx_context *ctx0,
             const int *p1, int ncomponents1, const char *o1, const int *from1, const int *dim1,
             void *const *v1, const sbx_context *ctx1, sbx_comm comm, int co, int copyadd,
             int session);

/* copy with masks (the reference's mask0 / mask1 arguments, dist.h:3534-3602; MaskType =
   float, tensor.h:54): mask0[c] / mask1[c] are laid out like the data of component c;
   elements are copied (and, with SBX_COPY, the uncovered part of the region zeroed) only where
   the masks are nonzero.  As in the reference the two masks must select the same elements
   (tensor.h:1019-1027): the destination mask decides for pieces received from other ranks.
   mask0 may be null (no origin mask); mask1 is required when mask0 is given. */
int sbx_copy_masked(int nd0, int nd1, const double *alpha, int t0, int t1, const int *p0,
                    int ncomponents0, const char *o0, const int *from0, const int *size0,
                    const int *dim0, const void *const *v0, const float *const *mask0,
                    const sbx_context *ctx0, const int *p1, int ncomponents1, const char *o1,
                    const int *from1, const int *dim1, void *const *v1,
                    const float *const *mask1, const sbx_context *ctx1, sbx_comm comm, int co,
                    int copyadd, int session);

/* ---- deferred completion (the reference's Request, dist.h:54-61, 2386-2437) ----
   The _req entry points take the same arguments as their plain forms plus `request`.  When the
   operation exchanges data with other ranks, the call returns once the exchange is started --
   RCCL: packed and sent / received on the library's side stream, so later library-stream work
   (e.g. the product of another operator piece) overlaps the transfer; host-staged: packed --
   and *request receives a handle whose sbx_wait finishes it (unpack, and for bsr_krylov the
   local product and the output copies).  Otherwise the call completes and *request is NULL.
   As in the reference every rank must wait its requests, in the same order; the outputs are
   defined only after sbx_wait (then, as always, stream-ordered on the library stream). */
typedef struct sbx_request_s *sbx_request;
int sbx_wait(sbx_request request); /* NULL: no-op; the handle is freed */
int sbx_copy_req(int nd0, int nd1, const double *alpha, int t0, int t1, const int *p0,
                 int ncomponents0, const char *o0, const int *from0, const int *size0,
                 const int *dim0, const void *const *v0, const float *const *mask0,
                 const sbx_context *ctx0, const int *p1, int ncomponents1, const char *o1,
                 const int *from1, const int *dim1, void *const *v1, const float *const *mask1,
                 const sbx_context *ctx1, sbx_comm comm, int co, int copyadd, int session,
                 sbx_request *request);

/* Exchange plan of sbx_copy as seen by `rank` of `nprocs` (host only, no GPU work; the
   reference get_indices_to_send / get_indices_to_receive, dist.h:1789-1900, 2321-2324):
   send[q] / recv[q] = elements sent to / received from rank q, *local = elements moved within
   the rank.  For inspection and tests of the multi-process plan. */
int sbx_copy_plan(int nd0, int nd1, const int *p0, int ncomponents0, const char *o0,
                  const int *from0, const int *size0, const int *dim0, const int *p1,
                  int ncomponents1, const char *o1, const int *from1, const int *dim1, int nprocs,
                  int rank, int co, int copyadd, long long *send, long long *recv,
                  long long *local);

/* ---- contraction (dist.h:3701-3731 no-MPI / 3628-3662 MPI) ----
   vr = alpha * sum_{labels in o0 and o1, not in o_r} conj?(v0) conj?(v1) + beta * vr */
int sbx_contraction(int nd0, int nd1, int ndr, int t, const double *alpha,
                    const int *p0, const int *from0, const int *size0, const int *dim0,
                    int ncomponents0, const char *o0, int conj0, const void *const *v0,
                    const sbx_context *ctx0,
                    const int *p1, const int *from1, const int *size1, const int *dim1,
                    int ncomponents1, const char *o1, int conj1, const void *const *v1,
                    const sbx_context *ctx1, const double *beta,
                    const int *pr, const int *fromr, const int *sizer, const int *dimr,
                    int ncomponentsr, const char *o_r, void *const *vr, const sbx_context *ctxr,
                    sbx_comm comm, int co, int session);

/* ---- BSR operator (bsr.h:2440-2454 create_bsr, 2516-2543 bsr_krylov, 2495 destroy_bsr,
   2554-2580 bsr_get_preferred_layout) ----
   ii[c]: number of nonzero blocks of each block row of component c (not a prefix sum);
   jj[c]: nd ints per nonzero block, the domain coordinate of the block relative to the domain
   partition's `from` (a -1 first coordinate skips the block, ELL form). */
int sbx_create_bsr(int nd, int ni, int t, const int *pim, const int *dimi, const int *pdm,
                   const int *dimd, int ncomponents, const int *blockim, const int *blockdm,
                   int blockImFast, const int *const *ii, const int *const *jj,
                   const void *const *v, const sbx_context *ctx, sbx_comm comm, int co,
                   sbx_bsr *bsrh, int session);
/* create_kron_bsr (bsr.h:2476-2490 no MPI, 2322-2336 MPI): as sbx_create_bsr plus the
   Kronecker block dimensions kronim[ni] / krondm[nd] and, per component, kronv[c]: one
   ki x kd matrix (ki = volume(kronim), kd = volume(krondm); image index fastest if
   blockImFast) per nonzero position of a block row; every block row must have the same number
   of nonzero blocks and no -1 domain coordinates (get_kron_indices, bsr.h:1485-1537).
   kronv must stay allocated until sbx_destroy_bsr.  bsr_krylov then prefers row-major x / y
   with the Kronecker labels fastest: (D, d, C, kd) and (I, i, C, ki). */
int sbx_create_kron_bsr(int nd, int ni, int t, const int *pim, const int *dimi, const int *pdm,
                        const int *dimd, int ncomponents, const int *blockim, const int *blockdm,
                        const int *kronim, const int *krondm, int blockImFast,
                        const int *const *ii, const int *const *jj, const void *const *v,
                        const void *const *kronv, const sbx_context *ctx, sbx_comm comm, int co,
                        sbx_bsr *bsrh, int session);
int sbx_bsr_krylov(sbx_bsr bsrh, int nd, int ni, int nx, int ny, int t, const double *alpha,
                   const char *oim, const char *odm, const int *px, int ncomponents,
                   const char *ox, const int *fromx, const int *sizex, const int *dimx,
                   const void *const *vx, const double *beta, const int *py, const char *oy,
                   const int *fromy, const int *sizey, const int *dimy, char okr,
                   void *const *vy, const sbx_context *ctx, sbx_comm comm, int co, int session);
/* bsr_krylov with the reference's `just_local` (bsr.h:2352-2359: only this rank's part of the
   product, no exchange; the other ranks' components are ignored) and deferred completion (the
   halo exchange started, the local product queued at sbx_wait; see sbx_request above) */
int sbx_bsr_krylov_req(sbx_bsr bsrh, int nd, int ni, int nx, int ny, int t, const double *alpha,
                       const char *oim, const char *odm, const int *px, int ncomponents,
                       const char *ox, const int *fromx, const int *sizex, const int *dimx,
                       const void *const *vx, const double *beta, const int *py, const char *oy,
                       const int *fromy, const int *sizey, const int *dimy, char okr,
                       void *const *vy, const sbx_context *ctx, sbx_comm comm, int co,
                       int session, int just_local, sbx_request *request);
int sbx_bsr_get_preferred_layout(sbx_bsr bsrh, int ncomponents, const sbx_context *ctx,
                                 sbx_comm comm, int co, int *layout_x, int *layout_y);
int sbx_destroy_bsr(sbx_bsr bsrh);

/* ---- dense batched solvers (dense.h:1160-1290 no MPI, 1007-1157 MPI) ----
   The labels of `o` split into row labels `orows`, column labels `ocols` and batch labels (the
   rest); every batch entry is a square matrix (rows index = orows labels, last label fastest for
   SLOW_TO_FAST).  cholesky: A <- U with A = U^H U (upper triangle; the strict lower part is left
   untouched); inversion: A <- A^-1; trsm: y = alpha C^-1 x (x holds the column labels of the
   upper triangular C) or y = alpha x C^-1 (x holds its row labels); gesm: y = alpha C^-1 x for a
   general C (x holds the column labels).  A failed factorization returns an error carrying the
   LAPACK info ("Error in lapack routine: i"). */
int sbx_cholesky(int nd, int t, const int *p, const int *dim, int ncomponents, const char *o,
                 void *const *v, const char *orows, const char *ocols, const sbx_context *ctx,
                 sbx_comm comm, int co, int session);
int sbx_inversion(int nd, int t, const int *p, const int *dim, int ncomponents, const char *o,
                  void *const *v, const char *orows, const char *ocols, const sbx_context *ctx,
                  sbx_comm comm, int co, int session);
int sbx_trsm(int ndc, int ndx, int ndy, int t, const double *alpha, const int *pc, const int *dimc,
             int ncomponentsc, const char *oc, const void *const *vc, const char *orows,
             const char *ocols, const sbx_context *ctxc, const int *px, const int *dimx,
             int ncomponentsx, const char *ox, const void *const *vx, const sbx_context *ctxx,
             const int *py, const int *dimy, int ncomponentsy, const char *oy, void *const *vy,
             const sbx_context *ctxy, sbx_comm comm, int co, int session);
int sbx_gesm(int ndc, int ndx, int ndy, int t, const double *alpha, const int *pc, const int *dimc,
             int ncomponentsc, const char *oc, const void *const *vc, const char *orows,
             const char *ocols, const sbx_context *ctxc, const int *px, const int *dimx,
             int ncomponentsx, const char *ox, const void *const *vx, const sbx_context *ctxx,
             const int *py, const int *dimy, int ncomponentsy, const char *oy, void *const *vy,
             const sbx_context *ctxy, sbx_comm comm, int co, int session);

/* ---- tensor storage, the S3T file format (storage.h:19-54) ----
   Values types: SBX_FLOAT, SBX_DOUBLE, SBX_CFLOAT, SBX_CDOUBLE, SBX_INT (the file's
   values_datatype 0, 1, 2, 3, 5); checksum: 0 none, 1 global, 2 per block (checksum_type,
   storage.h:70).  Every rank of `comm` opens the same file; rank 0 writes the headers and
   checksums, all ranks write their own values.  comm may be NULL (one process). */
int sbx_storage_create(int nd, const int *dim, int co, const char *filename,
                       const char *metadata, int metadata_length, int checksum, int t,
                       sbx_comm comm, sbx_storage *sto);                  /* storage.h:2143, 2387 */
/* metadata is copied up to metadata_cap bytes; *metadata_length and *nd are the file's values;
   dim receives up to dim_cap dimensions (reversed for SBX_FAST_TO_SLOW) */
int sbx_storage_read_header(const char *filename, int co, int *t, char *metadata,
                            int metadata_cap, int *metadata_length, int *nd, int *dim,
                            int dim_cap);                                 /* storage.h:2161, 2405 */
int sbx_storage_open(int nd, int t, const char *filename, int allow_writing, sbx_comm comm,
                     sbx_storage *sto);                                   /* storage.h:2187, 2470 */
/* append the blocks p0 (num_blocks from/size pairs on a tensor with labels o0, dims dim0),
   restricted to [from0, from0+size0) and placed at from1 on the storage (labels o1); the simple
   form append_blocks(p, n, dim, ...) is o0 = o1 = trivial labels, from0 = from1 = 0 */
int sbx_storage_append_blocks(int nd0, int nd1, const int *p0, int num_blocks, const char *o0,
                              const int *from0, const int *size0, const int *dim0,
                              const char *o1, const int *from1, sbx_storage sto, sbx_comm comm,
                              int co);                                    /* storage.h:2230, 2510 */
int sbx_storage_save(int nd0, int nd1, const double *alpha, int t0, const int *p0,
                     int ncomponents0, const char *o0, const int *from0, const int *size0,
                     const int *dim0, const void *const *v0, const sbx_context *ctx0,
                     const char *o1, const int *from1, sbx_storage sto, sbx_comm comm, int co,
                     int session);                                        /* storage.h:2261, 2540 */
/* the values always replace the destination's, for Copy and Add alike (storage.h:1149-1150) */
int sbx_storage_load(int nd0, int nd1, const double *alpha, sbx_storage sto, const char *o0,
                     const int *from0, const int *size0, int t1, const int *p1, int ncomponents1,
                     const char *o1, const int *from1, const int *dim1, void *const *v1,
                     const sbx_context *ctx1, sbx_comm comm, int co, int copyadd,
                     int session);                                        /* storage.h:2292, 2572 */
/* stored blocks overlapping [from1, from1+size1) of a tensor with labels o1: up to cap from/size
   pairs (2*nd1 ints each) relative to from1; *nblocks is the total */
int sbx_storage_get_blocks(sbx_storage sto, int nd0, int nd1, const char *o0, const char *o1,
                           const int *from1, const int *size1, int co, int *blocks, int cap,
                           int *nblocks);                                 /* storage.h:2330, 2609 */
/* rank and values type of an open storage (the template checks of get_storage_context) */
int sbx_storage_info(sbx_storage sto, int *nd, int *t);
int sbx_storage_check(sbx_storage sto, sbx_comm comm);                    /* storage.h:2347, 2439 */
int sbx_storage_flush(sbx_storage sto);                                   /* storage.h:2434 */
int sbx_storage_preallocate(sbx_storage sto, unsigned long long size);    /* storage.h:2427 */
/* writes the pending checksums and releases the handle (also on error) */
int sbx_storage_close(sbx_storage sto, sbx_comm comm);                    /* storage.h:2361, 2451 */

/* ---- kernel-level entry points (the local hot path, for direct callers and benchmarks) ---- */

/* xgemm_batch_strided (blas.h:662-810; CPU blas_cpu_tmpl.hpp:376-478): BLAS column-major,
   transa/transb in {'N','T','C'} */
int sbx_xgemm_batch_strided(int t, char transa, char transb, int m, int n, int k,
                            const double *alpha, const void *a, int lda, long long stridea,
                            const void *b, int ldb, long long strideb, const double *beta,
                            void *c, int ldc, long long stridec, int batch, int device);

/* xgemm_batch_strided on a context (blas.h:662-810 GPU, blas_cpu_tmpl.hpp:376-478 CPU): a CPU
   context means host pointers, mirrored through device scratch for the product (complete on
   return); a GPU context is sbx_xgemm_batch_strided on its device */
int sbx_xgemm_batch_strided_ctx(int t, char transa, char transb, int m, int n, int k,
                                const double *alpha, const void *a, int lda, long long stridea,
                                const void *b, int ldb, long long strideb, const double *beta,
                                void *c, int ldc, long long stridec, int batch, sbx_context ctx);

/* ---- low-level memory of the superbblas::detail surface (include/superbblas_amd/detail.h) ----
   A CPU context means host memory (pageable or pinned).  Host destinations are complete on
   return; device work is enqueued on the library stream of the device. */
/* copy_n(v, xpu0, n, w, xpu1) (blas.h:170-231): bytes from src to dst (H2H, H2D, D2H, D2D, peer) */
int sbx_memcpy(void *dst, sbx_context dst_ctx, const void *src, sbx_context src_ctx,
               unsigned long long bytes);
/* zero_n (blas.h:436-490) */
int sbx_memset_zero(void *ptr, sbx_context ctx, unsigned long long bytes);
/* copy_n / copy_n_blocking with index vectors (copy_n.h:584-1050):
     w[(iw ? iw[d] : d*blocking) + r] (= | +=) alpha * v[(iv ? iv[d] : d*blocking) + r]
   for d < n, r < blocking, with the element conversion tv -> tw of copy(); index vectors (int)
   and data may live on the host or on one device each side */
int sbx_copy_n_blocking(const double *alpha, int tv, const void *v, sbx_context vctx,
                        long long blocking, const int *iv, sbx_context ivctx, long long n, int tw,
                        void *w, sbx_context wctx, const int *iw, sbx_context iwctx, int copyadd);
/* do_checksum (storage.h:701-731): the S3T format's CRC-32 (zlib polynomial) of `bytes` host
   bytes continuing from `prev`, or with blocksize > 0 the CRC of the CRCs of blocksize-byte
   chunks (prev must then be 0); host memory, computed on the host like the reference's */
int sbx_checksum(const void *p, unsigned long long bytes, unsigned long long blocksize,
                 unsigned prev, unsigned *out);
/* intersection(from0, size0, from1, size1, dim) of two periodic ranges (dist.h:461-486): up to
   maxout pieces of 2*nd ints {from, size}, first dimension fastest; *nout is the count */
int sbx_intersection(int nd, const int *from0, const int *size0, const int *from1,
                     const int *size1, const int *dim, int maxout, int *out, int *nout);

/* local_copy on one device (tensor.h:1055-1129): single component copy with labels */
int sbx_local_copy(int nd0, int nd1, const double *alpha, int t0, int t1, const char *o0,
                   const int *from0, const int *size0, const int *dim0, const void *v0,
                   const char *o1, const int *from1, const int *dim1, void *v1, int co,
                   int copyadd, int device);

#ifdef __cplusplus
}
#endif

#endif /* SUPERBBLAS_AMD_SBX_H */
