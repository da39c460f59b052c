"""superbblas_amd -- MI355X-native implementation of superbblas's distributed tensor
contraction hot path.

The product is the C-ABI shared library ``libsuperbblas_amd.so`` (HIP kernels for gfx950 +
C++ planner + RCCL communicator, declared in ``include/superbblas_amd/sbx.h``).  C++ callers use
the drop-in template header ``include/superbblas.h``; this module is the Python mirror of the
same operator interface (``copy``, ``contraction``, ``create_bsr``/``bsr_krylov``/``destroy_bsr``,
``basic_partitioning`` ...) over ``ctypes``, used by the tests and the benchmark.

Reference interface: eromero-vlc/superbblas include/superbblas/dist.h:3534-3742 (copy,
contraction), bsr.h:2269-2580 (BSR), dist.h:3264-3509 (partitioning), platform.h:757-841.

PyTorch is plumbing only (device memory and streams).  There is no CPU fallback: importing the
module fails loudly if the HIP library has not been built.
"""

from __future__ import annotations

import ctypes
import os
from typing import Iterable, List, Optional, Sequence, Tuple

import torch  # noqa: F401  (load torch's HIP runtime before the library)

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libsuperbblas_amd.so")

if not os.path.exists(_LIB_PATH):
    raise ImportError(
        "superbblas_amd: native library %s not found; run __graft_entry__.build() "
        "(or `make -C superbblas_amd/csrc`) first" % _LIB_PATH)

_lib = ctypes.CDLL(_LIB_PATH, mode=ctypes.RTLD_GLOBAL)
LIB_PATH = _LIB_PATH

# ---- enums (tensor.h:56-66, bsr.h:28-31, platform.h:105-109) ----
SlowToFast, FastToSlow = 0, 1
Copy, Add = 0, 1
RowMajor, ColumnMajor = 0, 1
CPU, GPU = 0, 1
FLOAT, DOUBLE, CFLOAT, CDOUBLE, INT, SIZE_T = range(6)

_DTYPES = {
    torch.float32: FLOAT,
    torch.float64: DOUBLE,
    torch.complex64: CFLOAT,
    torch.complex128: CDOUBLE,
    torch.int32: INT,
    torch.int64: SIZE_T,
    torch.uint64: SIZE_T,
}


class SuperbblasError(RuntimeError):
    """Raised when a library call fails (the reference throws std::runtime_error)."""


class _Ctx(ctypes.Structure):
    _fields_ = [("plat", ctypes.c_int), ("device", ctypes.c_int)]


_c_int_p = ctypes.POINTER(ctypes.c_int)
_c_double_p = ctypes.POINTER(ctypes.c_double)
_c_void_pp = ctypes.POINTER(ctypes.c_void_p)
_ctx_p = ctypes.POINTER(_Ctx)

_lib.sbx_last_error.restype = ctypes.c_char_p




# errors of requests that were dropped without wait() and finished at garbage collection: they
# are never silently lost -- a warning at once, then raised by the next Request.wait() or by
# check_dropped() (never by an unrelated call that succeeded)
import threading as _threading

_dropped_lock = _threading.Lock()
_dropped_request_errors: List[str] = []


def _check(rc: int):
    if rc != 0:
        raise SuperbblasError(_lib.sbx_last_error().decode())


def _raise_dropped():
    with _dropped_lock:
        msg = _dropped_request_errors.pop(0) if _dropped_request_errors else None
    if msg is not None:
        raise SuperbblasError("a Request dropped without wait() failed when it was finished at "
                              "garbage collection: " + msg)


def check_dropped():
    """Raise the failure of a Request that was dropped without wait() and failed when garbage
    collection finished it (oldest first); no-op when there is none."""
    _raise_dropped()


import array as _array

_VP = ctypes.c_void_p
_I = ctypes.c_int


class _Pack:
    """All integer arguments of one call in ONE int32 buffer (and the data pointers in one
    uint64 buffer): a single allocation instead of one ctypes array per argument, which is
    what dominates the host cost of a call from Python."""
    __slots__ = ("ints", "offs", "ptrs", "poffs")

    def __init__(self):
        self.ints = _array.array("i")
        self.offs = []
        self.ptrs = _array.array("Q")
        self.poffs = []

    def add(self, xs):
        self.offs.append(len(self.ints))
        self.ints.extend(xs)
        return len(self.offs) - 1

    def add_partition(self, p, nd):
        self.offs.append(len(self.ints))
        for frm, size in p:
            if len(frm) != nd or len(size) != nd:
                raise SuperbblasError("partition item with wrong rank")
            self.ints.extend(frm)
            self.ints.extend(size)
        return len(self.offs) - 1

    def add_ctxs(self, ts):
        self.offs.append(len(self.ints))
        for t in ts:
            if t.is_cuda:
                self.ints.append(GPU)
                self.ints.append(t.device.index or 0)
            else:
                self.ints.append(CPU)
                self.ints.append(-1)
        return len(self.offs) - 1

    def add_ptrs(self, ts):
        self.poffs.append(len(self.ptrs))
        for t in ts:
            self.ptrs.append(t.data_ptr())
        return len(self.poffs) - 1

    def addrs(self):
        if not self.ints:
            self.ints.append(0)
        if not self.ptrs:
            self.ptrs.append(0)
        bi = self.ints.buffer_info()[0]
        bp = self.ptrs.buffer_info()[0]
        return [bi + 4 * o for o in self.offs], [bp + 8 * o for o in self.poffs]


_lib.sbx_copy.argtypes = [_I, _I, _VP, _I, _I, _VP, _I, ctypes.c_char_p, _VP, _VP, _VP, _VP, _VP,
                          _VP, _I, ctypes.c_char_p, _VP, _VP, _VP, _VP, _VP, _I, _I, _I]
_lib.sbx_copy_masked.argtypes = [_I, _I, _VP, _I, _I, _VP, _I, ctypes.c_char_p, _VP, _VP, _VP,
                                 _VP, _VP, _VP, _VP, _I, ctypes.c_char_p, _VP, _VP, _VP, _VP, _VP,
                                 _VP, _I, _I, _I]
_lib.sbx_copy_req.argtypes = _lib.sbx_copy_masked.argtypes + [_VP]
_lib.sbx_wait.argtypes = [_VP]
_lib.sbx_comm_transport.argtypes = [_VP, _VP, _VP, _VP]


class Request:
    """Deferred completion of a distributed copy / bsr_krylov (the reference's Request,
    dist.h:54-61): the exchange is started; wait() finishes it.  Every rank waits its requests in
    the same order."""

    def __init__(self, handle):
        self._h = handle

    def wait(self):
        if self._h:
            h, self._h = self._h, None
            _check(_lib.sbx_wait(h))
        _raise_dropped()

    def __del__(self):
        # a dropped request is still completed, but at garbage-collection time rather than at a
        # point every rank agrees on: warn, and hand a failure to the next library call
        if not self._h:
            return
        import warnings
        warnings.warn("superbblas_amd: a Request was dropped without wait(); finishing its "
                      "exchange at garbage collection", ResourceWarning, stacklevel=2)
        h, self._h = self._h, None
        try:
            msg = _lib.sbx_last_error().decode() if _lib.sbx_wait(h) != 0 else None
        except Exception as e:  # pragma: no cover (interpreter shutdown)
            msg = str(e)
        if msg is not None:
            warnings.warn("superbblas_amd: the dropped Request failed: " + msg, RuntimeWarning,
                          stacklevel=2)
            with _dropped_lock:
                _dropped_request_errors.append(msg)


def wait(request: Optional["Request"]):
    if request is not None:
        request.wait()


_lib.sbx_contraction.argtypes = (
    [_I, _I, _I, _I, _VP] +
    [_VP, _VP, _VP, _VP, _I, ctypes.c_char_p, _I, _VP, _VP] * 2 + [_VP] +
    [_VP, _VP, _VP, _VP, _I, ctypes.c_char_p, _VP, _VP, _VP, _I, _I])


def _ints(xs: Sequence[int]):
    arr = (ctypes.c_int * max(1, len(xs)))(*[int(x) for x in xs])
    return arr


def _scalar(a) -> ctypes.Array:
    a = complex(a)
    return (ctypes.c_double * 2)(a.real, a.imag)


def _partition(p: Sequence[Tuple[Sequence[int], Sequence[int]]], nd: int):
    flat: List[int] = []
    for item in p:
        frm, size = item
        if len(frm) != nd or len(size) != nd:
            raise SuperbblasError("partition item with wrong rank")
        flat += list(frm) + list(size)
    return _ints(flat)


def _ctx_of(t: torch.Tensor) -> _Ctx:
    if t.is_cuda:
        return _Ctx(GPU, t.device.index if t.device.index is not None else 0)
    return _Ctx(CPU, -1)


def _ptrs(ts: Sequence[torch.Tensor]):
    return (ctypes.c_void_p * max(1, len(ts)))(*[t.data_ptr() for t in ts])


def _ctxs(ts: Sequence[torch.Tensor]):
    return (_Ctx * max(1, len(ts)))(*[_ctx_of(t) for t in ts])


def _dtype_of(ts: Sequence[torch.Tensor]) -> int:
    dts = {t.dtype for t in ts}
    if len(dts) != 1:
        raise SuperbblasError("all components of a tensor must have the same dtype")
    dt = dts.pop()
    if dt not in _DTYPES:
        raise SuperbblasError("unsupported dtype %s" % dt)
    return _DTYPES[dt]


_bound_streams = {}


def _bind_stream(ts: Iterable[torch.Tensor]):
    """Enqueue library work on torch's current stream of every device involved."""
    for t in ts:
        if t.is_cuda:
            d = t.device.index or 0
            s = torch.cuda.current_stream(d).cuda_stream
            if _bound_streams.get(d) != s:
                _check(_lib.sbx_stream_set(d, ctypes.c_void_p(s)))
                _bound_streams[d] = s


def _check_sizes(p, rank, ncomp, v, what):
    for i in range(ncomp):
        size = p[rank * ncomp + i][1]
        n = 1
        for s in size:
            n *= s
        if n and (v[i].numel() < n or not v[i].is_contiguous()):
            raise SuperbblasError("%s: component %d has %d elements, the partition needs %d "
                                  "(contiguous)" % (what, i, v[i].numel(), n))


# ---------------------------------------------------------------------------------------------
# runtime
# ---------------------------------------------------------------------------------------------

def version() -> Tuple[int, int]:
    ma, mi = ctypes.c_int(), ctypes.c_int()
    _check(_lib.sbx_version(ctypes.byref(ma), ctypes.byref(mi)))
    return ma.value, mi.value


def get_gpu_devices_count() -> int:
    """getGpuDevicesCount (platform.h:818-825)"""
    n = ctypes.c_int()
    _check(_lib.sbx_get_gpu_devices_count(ctypes.byref(n)))
    return n.value


def sync(device: int = 0):
    """sync(Context) (blas.h:965-974): wait for the library stream of `device`."""
    _check(_lib.sbx_sync(_Ctx(GPU, device)))


def stream(device: int = 0) -> int:
    """hipStream_t the library uses for `device`."""
    s = ctypes.c_void_p()
    _check(_lib.sbx_stream_get(device, ctypes.byref(s)))
    return s.value or 0


def set_stream(device: int, hip_stream: Optional[int]):
    """Enqueue the library's work for `device` on `hip_stream` (0 = the null stream); None
    restores the library's own stream."""
    if hip_stream is None:
        _check(_lib.sbx_stream_reset(device))
    else:
        _check(_lib.sbx_stream_set(device, ctypes.c_void_p(hip_stream)))


def timings_enable(on: bool = True):
    """Time every GPU kernel family with HIP events on its launch stream (reportTimings)."""
    _check(_lib.sbx_timings_enable(int(on)))


def timings_reset():
    _check(_lib.sbx_timings_reset())


def timings_filter(names: Optional[str] = None):
    """Time only these kernel families (comma-separated; None = all)."""
    _check(_lib.sbx_timings_filter(names.encode() if names else None))


def tune_set(key: str, value: int):
    """Override a kernel-shape choice for tuning runs (sbx_tune_set; 0 restores the default)."""
    _check(_lib.sbx_tune_set(key.encode(), ctypes.c_longlong(value)))


def tune_get(key: str) -> int:
    v = ctypes.c_longlong()
    _check(_lib.sbx_tune_get(key.encode(), ctypes.byref(v)))
    return v.value


def timings_get(name: str) -> Tuple[float, int]:
    """(total milliseconds, launches) of a kernel family: gemm, gemm_splitk_reduce, copy, bsr."""
    ms, calls = ctypes.c_double(), ctypes.c_longlong()
    _check(_lib.sbx_timings_get(name.encode(), ctypes.byref(ms), ctypes.byref(calls)))
    return ms.value, calls.value


def timings_report() -> str:
    buf = ctypes.create_string_buffer(8192)
    _check(_lib.sbx_timings_report(buf, len(buf)))
    return buf.value.decode()


def clear_caches():
    """clearCaches (alloc.h:437-443)"""
    _check(_lib.sbx_clear_caches())


_lib.sbx_cache_usage.argtypes = [_I, _VP, _VP]


def cache_usage(device: int = 0) -> Tuple[int, int]:
    """(idle bytes held by the scratch cache, bytes in use) of a device (performance.h:436-495)"""
    cached, live = ctypes.c_ulonglong(0), ctypes.c_ulonglong(0)
    _check(_lib.sbx_cache_usage(device, ctypes.byref(cached), ctypes.byref(live)))
    return cached.value, live.value


# ---------------------------------------------------------------------------------------------
# communicator (replaces MPI_Comm; RCCL underneath)
# ---------------------------------------------------------------------------------------------

_ULLP = ctypes.POINTER(ctypes.c_ulonglong)
_ALLTOALLV_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, _ULLP, _ULLP, ctypes.c_void_p,
                                 _ULLP, _ULLP, ctypes.c_void_p)
_lib.sbx_comm_create_host.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, _ALLTOALLV_FN,
                                      ctypes.c_void_p, ctypes.c_void_p]


class Comm:
    """A communicator over `nprocs` processes.  Default transport: RCCL over xGMI (one GPU per
    process).  `Comm.host_staged` builds the host-staged transport instead (pinned host buffers
    + a torch.distributed all-to-all, any backend), the reference's non-GPU-aware MPI path."""

    def __init__(self, nprocs: int, rank: int, unique_id: Optional[bytes], device: int,
                 _host_fn=None):
        self.nprocs, self.rank, self.device = nprocs, rank, device
        h = ctypes.c_void_p()
        self._fn = _host_fn
        if _host_fn is None:
            buf = (ctypes.c_ubyte * 128).from_buffer_copy(unique_id)
            _check(_lib.sbx_comm_create(nprocs, rank, buf, device, ctypes.byref(h)))
        else:
            _check(_lib.sbx_comm_create_host(nprocs, rank, device, _host_fn, None,
                                             ctypes.byref(h)))
        self._h = h

    @classmethod
    def host_staged(cls, device: int, group=None) -> "Comm":
        """Communicator of the current torch.distributed group whose exchanges go through
        pinned host memory and ``all_to_all_single`` on ``group`` (e.g. gloo).  Several ranks
        may share a GPU."""
        import numpy as _np
        import torch.distributed as dist
        rank, n = dist.get_rank(group), dist.get_world_size(group)

        def exchange(sbuf, sbytes, sdispl, rbuf, rbytes, rdispl, _user):
            try:
                sb_, sd_ = [sbytes[q] for q in range(n)], [sdispl[q] for q in range(n)]
                rb_, rd_ = [rbytes[q] for q in range(n)], [rdispl[q] for q in range(n)]
                send = _np.zeros(sum(sb_), _np.uint8)
                o = 0
                for q in range(n):
                    if sb_[q]:
                        ctypes.memmove(send.ctypes.data + o, sbuf + sd_[q], sb_[q])
                    o += sb_[q]
                recv = torch.empty(sum(rb_), dtype=torch.uint8)
                dist.all_to_all_single(recv, torch.from_numpy(send), rb_, sb_, group=group)
                o = 0
                for q in range(n):
                    if rb_[q]:
                        ctypes.memmove(rbuf + rd_[q], recv.data_ptr() + o, rb_[q])
                    o += rb_[q]
                return 0
            except Exception as e:  # never let an exception cross the C boundary
                import sys
                print("superbblas_amd host all-to-all failed: %r" % e, file=sys.stderr)
                return 1

        return cls(n, rank, None, device, _host_fn=_ALLTOALLV_FN(exchange))

    @staticmethod
    def unique_id() -> bytes:
        buf = (ctypes.c_ubyte * 128)()
        _check(_lib.sbx_comm_unique_id(buf))
        return bytes(buf)

    @classmethod
    def from_torch_distributed(cls, device: int) -> "Comm":
        """Create the communicator of the current torch.distributed group: rank 0 makes the
        RCCL unique id and broadcasts it through the process group (any backend)."""
        import torch.distributed as dist
        rank, n = dist.get_rank(), dist.get_world_size()
        obj = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls(n, rank, obj[0], device)

    @property
    def handle(self):
        return self._h

    def transport(self):
        """(kind, count, user_rank): kind "none" (one rank), "rccl" (count and user_rank as RCCL
        itself reports them: ncclCommCount / ncclCommUserRank) or "host" (host-staged)."""
        k, c, r = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(_lib.sbx_comm_transport(self._h, ctypes.byref(k), ctypes.byref(c),
                                       ctypes.byref(r)))
        return ({0: "none", 1: "rccl", 2: "host"}[k.value], c.value, r.value)

    def close(self):
        if self._h:
            _check(_lib.sbx_comm_destroy(self._h))
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _comm(comm: Optional[Comm]):
    return comm.handle if comm is not None else None


def _nprocs_rank(comm: Optional[Comm]):
    return (comm.nprocs, comm.rank) if comm is not None else (1, 0)


# ---------------------------------------------------------------------------------------------
# partitioning helpers (dist.h:3264-3509, 3744-3825)
# ---------------------------------------------------------------------------------------------

def partitioning_distributed_procs(order: str, dim: Sequence[int], dist_labels: str,
                                   nprocs: int) -> List[int]:
    nd = len(dim)
    out = _ints([0] * nd)
    _check(_lib.sbx_partitioning_distributed_procs(nd, order.encode(), _ints(dim),
                                                   dist_labels.encode(), nprocs, out))
    return list(out[:nd])


def basic_partitioning(order: Optional[str], dim: Sequence[int], procs: Sequence[int],
                       dist_labels: Optional[str], nprocs: int = -1, ncomponents: int = 1):
    """basic_partitioning(order, dim, procs, dist_labels, nprocs, ncomponents)"""
    nd = len(dim)
    vol = 1
    for p in procs:
        vol *= p
    n = (vol if nprocs < 0 else nprocs) * ncomponents
    out = _ints([0] * (n * 2 * nd))
    _check(_lib.sbx_basic_partitioning(nd, order.encode() if order else None, _ints(dim),
                                       _ints(procs), dist_labels.encode() if dist_labels else None,
                                       nprocs, ncomponents, out))
    return [(list(out[k * 2 * nd:k * 2 * nd + nd]), list(out[k * 2 * nd + nd:(k + 1) * 2 * nd]))
            for k in range(n)]


def basic_partitioning_ext(dim: Sequence[int], procs: Sequence[int], nprocs: int = -1,
                           replicate: bool = False, ext_power: Optional[Sequence[int]] = None):
    """basic_partitioning(dim, procs, nprocs, replicate, ext_power)"""
    nd = len(dim)
    vol = 1
    for p in procs:
        vol *= p
    n = vol if nprocs < 0 else nprocs
    out = _ints([0] * (n * 2 * nd))
    _check(_lib.sbx_basic_partitioning_ext(nd, _ints(dim), _ints(procs), nprocs, int(replicate),
                                           _ints(ext_power) if ext_power else None, out))
    return [(list(out[k * 2 * nd:k * 2 * nd + nd]), list(out[k * 2 * nd + nd:(k + 1) * 2 * nd]))
            for k in range(n)]


def make_hole(frm, size, hole_from, hole_size, dim):
    nd = len(dim)
    if not all(len(x) == nd for x in (frm, size, hole_from, hole_size)):
        raise SuperbblasError("make_hole: coordinates of different rank")
    maxout = 4 * max(nd, 1) * (1 << min(nd, 6))
    out = _ints([0] * (maxout * 2 * nd))
    nout = ctypes.c_int()
    _check(_lib.sbx_make_hole(nd, _ints(frm), _ints(size), _ints(hole_from), _ints(hole_size),
                              _ints(dim), maxout, out, ctypes.byref(nout)))
    return [(list(out[k * 2 * nd:k * 2 * nd + nd]), list(out[k * 2 * nd + nd:(k + 1) * 2 * nd]))
            for k in range(nout.value)]


# ---------------------------------------------------------------------------------------------
# copy / contraction (dist.h:3534-3742)
# ---------------------------------------------------------------------------------------------

def copy(alpha, p0, o0: str, from0, size0, dim0, v0: Sequence[torch.Tensor], p1, o1: str, from1,
         dim1, v1: Sequence[torch.Tensor], co: int = SlowToFast, copyadd: int = Copy,
         comm: Optional[Comm] = None, mask0: Optional[Sequence[torch.Tensor]] = None,
         mask1: Optional[Sequence[torch.Tensor]] = None, request: bool = False):
    """v1[from1 + P(c - from0)] (=|+=) alpha * v0[c]  for c in [from0, from0 + size0);
    with masks (float32 tensors shaped like the components, dist.h:3534-3602) only where the
    masks are nonzero.  request=True: returns a Request (the exchange of a distributed copy
    started, finished by its wait()) or None when the copy completed."""
    nprocs, rank = _nprocs_rank(comm)
    nd0, nd1 = len(o0), len(o1)
    nc0, nc1 = len(v0), len(v1)
    if len(p0) != nprocs * nc0 or len(p1) != nprocs * nc1:
        raise SuperbblasError("partition is incompatible with the communicator/components")
    _check_sizes(p0, rank, nc0, v0, "copy origin")
    _check_sizes(p1, rank, nc1, v1, "copy destination")
    t0, t1 = _dtype_of(v0), _dtype_of(v1)
    _bind_stream(v0)
    _bind_stream(v1)
    k = _Pack()
    k.add_partition(p0, nd0)
    k.add(from0)
    k.add(size0)
    k.add(dim0)
    k.add_ctxs(v0)
    k.add_partition(p1, nd1)
    k.add(from1)
    k.add(dim1)
    k.add_ctxs(v1)
    k.add_ptrs(v0)
    k.add_ptrs(v1)
    if mask0 is None and mask1 is None and not request:
        a, pp = k.addrs()
        _check(_lib.sbx_copy(nd0, nd1, _scalar(alpha), t0, t1, a[0], nc0, o0.encode(), a[1], a[2],
                             a[3], pp[0], a[4], a[5], nc1, o1.encode(), a[6], a[7], pp[1], a[8],
                             _comm(comm), co, copyadd, 0))
        return
    for m, v in ((mask0, v0), (mask1, v1)):
        if m is not None and (len(m) != len(v) or any(
                x.dtype != torch.float32 or x.numel() != y.numel() for x, y in zip(m, v))):
            raise SuperbblasError("masks must be float32 tensors shaped like the components")
    k.add_ptrs(mask0 or [])
    k.add_ptrs(mask1 or [])
    a, pp = k.addrs()
    h = ctypes.c_void_p()
    _check(_lib.sbx_copy_req(nd0, nd1, _scalar(alpha), t0, t1, a[0], nc0, o0.encode(), a[1],
                             a[2], a[3], pp[0], pp[2] if mask0 is not None else None, a[4],
                             a[5], nc1, o1.encode(), a[6], a[7], pp[1],
                             pp[3] if mask1 is not None else None, a[8], _comm(comm), co,
                             copyadd, 0, ctypes.byref(h) if request else None))
    if request:
        return Request(h.value) if h.value else None


def copy_plan(p0, o0: str, from0, size0, dim0, ncomponents0: int, p1, o1: str, from1, dim1,
              ncomponents1: int, nprocs: int, rank: int, co: int = SlowToFast,
              copyadd: int = Copy):
    """Host-side exchange plan of `copy` as rank `rank` of `nprocs` would run it (no GPU work):
    returns (send[q], recv[q], local) element counts."""
    nd0, nd1 = len(o0), len(o1)
    if len(p0) != nprocs * ncomponents0 or len(p1) != nprocs * ncomponents1:
        raise SuperbblasError("partition is incompatible with nprocs/components")
    send = (ctypes.c_longlong * nprocs)()
    recv = (ctypes.c_longlong * nprocs)()
    local = ctypes.c_longlong()
    _check(_lib.sbx_copy_plan(nd0, nd1, _partition(p0, nd0), ncomponents0, o0.encode(),
                              _ints(from0), _ints(size0), _ints(dim0), _partition(p1, nd1),
                              ncomponents1, o1.encode(), _ints(from1), _ints(dim1), nprocs, rank,
                              co, copyadd, send, recv, ctypes.byref(local)))
    return list(send), list(recv), local.value


def contraction(alpha, p0, from0, size0, dim0, o0: str, conj0: bool, v0, p1, from1, size1, dim1,
                o1: str, conj1: bool, v1, beta, pr, fromr, sizer, dimr, o_r: str, vr,
                co: int = SlowToFast, comm: Optional[Comm] = None):
    """vr = alpha * sum over the labels in o0 and o1 but not in o_r of v0 * v1 + beta * vr."""
    nprocs, rank = _nprocs_rank(comm)
    nd0, nd1, ndr = len(o0), len(o1), len(o_r)
    nc0, nc1, ncr = len(v0), len(v1), len(vr)
    if len(p0) != nprocs * nc0 or len(p1) != nprocs * nc1 or len(pr) != nprocs * ncr:
        raise SuperbblasError("partition is incompatible with the communicator")
    _check_sizes(p0, rank, nc0, v0, "contraction v0")
    _check_sizes(p1, rank, nc1, v1, "contraction v1")
    _check_sizes(pr, rank, ncr, vr, "contraction vr")
    t = _dtype_of(v0)
    if _dtype_of(v1) != t or _dtype_of(vr) != t:
        raise SuperbblasError("contraction: all tensors must have the same dtype")
    _bind_stream(v0)
    _bind_stream(v1)
    _bind_stream(vr)
    k = _Pack()
    for p, nd, f, sz, dm, v in ((p0, nd0, from0, size0, dim0, v0), (p1, nd1, from1, size1, dim1, v1),
                                (pr, ndr, fromr, sizer, dimr, vr)):
        k.add_partition(p, nd)
        k.add(f)
        k.add(sz)
        k.add(dm)
        k.add_ctxs(v)
        k.add_ptrs(v)
    a, pp = k.addrs()
    _check(_lib.sbx_contraction(
        nd0, nd1, ndr, t, _scalar(alpha),
        a[0], a[1], a[2], a[3], nc0, o0.encode(), int(conj0), pp[0], a[4],
        a[5], a[6], a[7], a[8], nc1, o1.encode(), int(conj1), pp[1], a[9], _scalar(beta),
        a[10], a[11], a[12], a[13], ncr, o_r.encode(), pp[2], a[14], _comm(comm), co, 0))


def local_copy(alpha, o0: str, from0, size0, dim0, v0: torch.Tensor, o1: str, from1, dim1,
               v1: torch.Tensor, co: int = SlowToFast, copyadd: int = Copy):
    """Single-component copy on one device (tensor.h:1055-1129)."""
    _bind_stream([v0, v1])
    _check(_lib.sbx_local_copy(len(o0), len(o1), _scalar(alpha), _DTYPES[v0.dtype],
                               _DTYPES[v1.dtype], o0.encode(), _ints(from0), _ints(size0),
                               _ints(dim0), ctypes.c_void_p(v0.data_ptr()), o1.encode(),
                               _ints(from1), _ints(dim1), ctypes.c_void_p(v1.data_ptr()), co,
                               copyadd, v1.device.index or 0))


def xgemm_batch_strided(transa: str, transb: str, m: int, n: int, k: int, alpha, a, lda: int,
                        stridea: int, b, ldb: int, strideb: int, beta, c, ldc: int, stridec: int,
                        batch: int):
    """BLAS column-major strided batched GEMM (blas.h:662-810) on MFMA."""
    _bind_stream([a, b, c])
    _check(_lib.sbx_xgemm_batch_strided(
        _DTYPES[c.dtype], ctypes.c_char(transa.encode()), ctypes.c_char(transb.encode()), m, n, k,
        _scalar(alpha), ctypes.c_void_p(a.data_ptr()), lda, ctypes.c_longlong(stridea),
        ctypes.c_void_p(b.data_ptr()), ldb, ctypes.c_longlong(strideb), _scalar(beta),
        ctypes.c_void_p(c.data_ptr()), ldc, ctypes.c_longlong(stridec), batch,
        c.device.index or 0))


# ---------------------------------------------------------------------------------------------
# BSR operator (bsr.h:2269-2580)
# ---------------------------------------------------------------------------------------------

class BSR:
    """Handle of a block-sparse operator (BSR_handle, bsr.h:34-52).  Keeps references to the
    nonzero values (they must stay alive until destroy, bsr.h:2284)."""

    def __init__(self, handle, nd, ni, dtype, co, keep):
        self._h, self.nd, self.ni, self.dtype, self.co, self._keep = handle, nd, ni, dtype, co, keep

    @property
    def handle(self):
        return self._h

    def destroy(self):
        if self._h:
            _check(_lib.sbx_destroy_bsr(self._h))
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def create_bsr(pim, dimi, pdm, dimd, blockim, blockdm, block_im_fast: bool,
               ii: Sequence[torch.Tensor], jj: Sequence[torch.Tensor],
               v: Sequence[torch.Tensor], co: int = SlowToFast,
               comm: Optional[Comm] = None) -> BSR:
    """create_bsr<Nd,Ni,T> (bsr.h:2440-2454).  ii[c]: int32 nonzero blocks per block row;
    jj[c]: int32 [nnz, Nd] domain coordinates; v[c]: nonzero blocks."""
    nd, ni = len(dimd), len(dimi)
    nc = len(v)
    h = ctypes.c_void_p()
    t = _dtype_of(v)
    iip = (ctypes.c_void_p * nc)(*[x.data_ptr() for x in ii])
    jjp = (ctypes.c_void_p * nc)(*[x.data_ptr() for x in jj])
    _bind_stream(list(v))
    _check(_lib.sbx_create_bsr(nd, ni, t, _partition(pim, ni), _ints(dimi), _partition(pdm, nd),
                               _ints(dimd), nc, _ints(blockim), _ints(blockdm), int(block_im_fast),
                               iip, jjp, _ptrs(v), _ctxs(v), _comm(comm), co, ctypes.byref(h), 0))
    return BSR(h, nd, ni, t, co, (list(ii), list(jj), list(v)))


def create_kron_bsr(pim, dimi, pdm, dimd, blockim, blockdm, kronim, krondm, block_im_fast: bool,
                    ii: Sequence[torch.Tensor], jj: Sequence[torch.Tensor],
                    v: Sequence[torch.Tensor], kronv: Sequence[torch.Tensor],
                    co: int = SlowToFast, comm: Optional[Comm] = None) -> BSR:
    """create_kron_bsr<Nd,Ni,T> (bsr.h:2476-2490): create_bsr plus, per component, kronv[c] =
    one volume(kronim) x volume(krondm) matrix per nonzero position of a block row."""
    nd, ni = len(dimd), len(dimi)
    nc = len(v)
    h = ctypes.c_void_p()
    t = _dtype_of(list(v) + list(kronv))
    iip = (ctypes.c_void_p * nc)(*[x.data_ptr() for x in ii])
    jjp = (ctypes.c_void_p * nc)(*[x.data_ptr() for x in jj])
    _bind_stream(list(v))
    _check(_lib.sbx_create_kron_bsr(nd, ni, t, _partition(pim, ni), _ints(dimi),
                                    _partition(pdm, nd), _ints(dimd), nc, _ints(blockim),
                                    _ints(blockdm), _ints(kronim), _ints(krondm),
                                    int(block_im_fast), iip, jjp, _ptrs(v), _ptrs(kronv),
                                    _ctxs(v), _comm(comm), co, ctypes.byref(h), 0))
    return BSR(h, nd, ni, t, co, (list(ii), list(jj), list(v), list(kronv)))


def bsr_krylov(alpha, bsr: BSR, oim: str, odm: str, px, ox: str, fromx, sizex, dimx, vx, beta,
               py, oy: str, fromy, sizey, dimy, okr: Optional[str], vy, co: int = SlowToFast,
               comm: Optional[Comm] = None, request: bool = False, just_local: bool = False):
    """y = alpha * A x (+ beta y) (bsr.h:2516-2543; MPI form 2352-2383).  just_local: only this
    rank's part, no exchange.  request=True: returns a Request when the halo exchange is left in
    flight (the local product runs at its wait()), else None."""
    nx, ny = len(ox), len(oy)
    nc = len(vx)
    t = _dtype_of(list(vx) + list(vy))
    _bind_stream(list(vx) + list(vy))
    h = ctypes.c_void_p()
    _check(_lib.sbx_bsr_krylov_req(
        bsr.handle, bsr.nd, bsr.ni, nx, ny, t, _scalar(alpha), oim.encode(), odm.encode(),
        _partition(px, nx), nc, ox.encode(), _ints(fromx), _ints(sizex), _ints(dimx), _ptrs(vx),
        _scalar(beta), _partition(py, ny), oy.encode(), _ints(fromy), _ints(sizey), _ints(dimy),
        ctypes.c_char((okr or "\0").encode()), _ptrs(vy), _ctxs(vx), _comm(comm), co, 0,
        int(just_local), ctypes.byref(h) if request else None))
    if request:
        return Request(h.value) if h.value else None


def _inplace_dense(fn, p, dim, o: str, v, orows: str, ocols: str, co, comm):
    nd = len(o)
    nc = len(v)
    t = _dtype_of(v)
    _bind_stream(list(v))
    _check(fn(nd, t, _partition(p, nd), _ints(dim), nc, o.encode(), _ptrs(v), orows.encode(),
              ocols.encode(), _ctxs(v), _comm(comm), co, 0))


def cholesky(p, dim, o: str, v: Sequence[torch.Tensor], orows: str, ocols: str,
             co: int = SlowToFast, comm: Optional[Comm] = None):
    """cholesky<N,T> (dense.h:1160-1175): every batch matrix (rows orows x columns ocols) is
    replaced by U with A = U^H U (upper triangle; the strict lower part is left as is)."""
    _inplace_dense(_lib.sbx_cholesky, p, dim, o, v, orows, ocols, co, comm)


def inversion(p, dim, o: str, v: Sequence[torch.Tensor], orows: str, ocols: str,
              co: int = SlowToFast, comm: Optional[Comm] = None):
    """inversion<N,T> (dense.h:1274-1287): every batch matrix is replaced by its inverse."""
    _inplace_dense(_lib.sbx_inversion, p, dim, o, v, orows, ocols, co, comm)


def _solve_dense(fn, alpha, pc, dimc, oc, vc, orows, ocols, px, dimx, ox, vx, py, dimy, oy, vy,
                 co, comm):
    t = _dtype_of(list(vc) + list(vx) + list(vy))
    _bind_stream(list(vc) + list(vx) + list(vy))
    _check(fn(len(oc), len(ox), len(oy), t, _scalar(alpha), _partition(pc, len(oc)), _ints(dimc),
              len(vc), oc.encode(), _ptrs(vc), orows.encode(), ocols.encode(), _ctxs(vc),
              _partition(px, len(ox)), _ints(dimx), len(vx), ox.encode(), _ptrs(vx), _ctxs(vx),
              _partition(py, len(oy)), _ints(dimy), len(vy), oy.encode(), _ptrs(vy), _ctxs(vy),
              _comm(comm), co, 0))


def trsm(alpha, pc, dimc, oc: str, vc, orows: str, ocols: str, px, dimx, ox: str, vx, py, dimy,
         oy: str, vy, co: int = SlowToFast, comm: Optional[Comm] = None):
    """trsm<Nc,Nx,Ny,T> (dense.h:1195-1222): y = alpha C^-1 x (x holds C's column labels) or
    y = alpha x C^-1 (x holds its row labels), C upper triangular (a Cholesky factor)."""
    _solve_dense(_lib.sbx_trsm, alpha, pc, dimc, oc, vc, orows, ocols, px, dimx, ox, vx, py,
                 dimy, oy, vy, co, comm)


def gesm(alpha, pc, dimc, oc: str, vc, orows: str, ocols: str, px, dimx, ox: str, vx, py, dimy,
         oy: str, vy, co: int = SlowToFast, comm: Optional[Comm] = None):
    """gesm<Nc,Nx,Ny,T> (dense.h:1239-1266): y = alpha C^-1 x for general C (LU with partial
    pivoting), x holding C's column labels."""
    _solve_dense(_lib.sbx_gesm, alpha, pc, dimc, oc, vc, orows, ocols, px, dimx, ox, vx, py,
                 dimy, oy, vy, co, comm)


def bsr_get_preferred_layout(bsr: BSR, ncomponents: int = 1, co: int = SlowToFast,
                             comm: Optional[Comm] = None):
    lx, ly = _ints([0] * ncomponents), _ints([0] * ncomponents)
    ctxs = (_Ctx * ncomponents)(*[_Ctx(GPU, 0)] * ncomponents)
    _check(_lib.sbx_bsr_get_preferred_layout(bsr.handle, ncomponents, ctxs, _comm(comm), co, lx,
                                             ly))
    return list(lx[:ncomponents]), list(ly[:ncomponents])


# ---------------------------------------------------------------------------------------------
# tensor storage, the S3T file format (storage.h:2374-2617)
# ---------------------------------------------------------------------------------------------

NoChecksum, GlobalChecksum, BlockChecksum = 0, 1, 2
_STORAGE_TYPES = {torch.float32: FLOAT, torch.float64: DOUBLE, torch.complex64: CFLOAT,
                  torch.complex128: CDOUBLE, torch.int32: INT}
_STORAGE_TORCH = {v: k for k, v in _STORAGE_TYPES.items()}


class Storage:
    """Handle of an S3T tensor storage (Storage_handle, storage.h:2127)."""

    def __init__(self, handle, nd, dtype):
        self._h, self.nd, self.dtype = handle, nd, dtype

    @property
    def handle(self):
        if not self._h:
            raise SuperbblasError("storage: the handle is closed")
        return self._h

    @property
    def torch_dtype(self):
        return _STORAGE_TORCH[self.dtype]

    def close(self, comm: Optional[Comm] = None):
        if self._h:
            h, self._h = self._h, None
            _check(_lib.sbx_storage_close(h, _comm(comm)))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _storage_type(dtype) -> int:
    if isinstance(dtype, int):
        return dtype
    if dtype not in _STORAGE_TYPES:
        raise SuperbblasError("storage: unsupported type %s" % dtype)
    return _STORAGE_TYPES[dtype]


def create_storage(dim, co: int, filename: str, metadata: bytes = b"",
                   checksum: int = NoChecksum, dtype=torch.complex128,
                   comm: Optional[Comm] = None) -> Storage:
    """create_storage<Nd,T> (storage.h:2386-2395): a new file (its content, if any, is lost)."""
    h = ctypes.c_void_p()
    t = _storage_type(dtype)
    meta = bytes(metadata)
    _check(_lib.sbx_storage_create(len(dim), _ints(dim), co, os.fsencode(filename), meta,
                                   len(meta), checksum, t, _comm(comm), ctypes.byref(h)))
    return Storage(h, len(dim), t)


def read_storage_header(filename: str, co: int = SlowToFast):
    """read_storage_header (storage.h:2405-2421): (values type, metadata bytes, dims)."""
    t, ml, nd = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    _check(_lib.sbx_storage_read_header(os.fsencode(filename), co, ctypes.byref(t), None, 0,
                                        ctypes.byref(ml), ctypes.byref(nd), None, 0))
    meta = ctypes.create_string_buffer(max(1, ml.value))
    dim = _ints([0] * nd.value)
    _check(_lib.sbx_storage_read_header(os.fsencode(filename), co, ctypes.byref(t), meta,
                                        ml.value, ctypes.byref(ml), ctypes.byref(nd), dim,
                                        nd.value))
    return t.value, meta.raw[:ml.value], list(dim[:nd.value])


def open_storage(filename: str, allow_writing: bool = False, nd: Optional[int] = None,
                 dtype=None, comm: Optional[Comm] = None) -> Storage:
    """open_storage<Nd,T> (storage.h:2469-2476); nd/dtype default to the file's own."""
    if nd is None or dtype is None:
        t0, _, d0 = read_storage_header(filename)
        nd = len(d0) if nd is None else nd
        dtype = t0 if dtype is None else dtype
    h = ctypes.c_void_p()
    t = _storage_type(dtype)
    _check(_lib.sbx_storage_open(nd, t, os.fsencode(filename), int(allow_writing), _comm(comm),
                                 ctypes.byref(h)))
    return Storage(h, nd, t)


def append_blocks(sto: Storage, p0, dim0, o0: Optional[str] = None, from0=None, size0=None,
                  o1: Optional[str] = None, from1=None, co: int = SlowToFast,
                  comm: Optional[Comm] = None):
    """append_blocks (storage.h:2484-2521): declare the blocks p0 (from/size pairs) stored; the
    short form (o0/o1 omitted) takes them in the storage's own coordinates."""
    nd0 = len(dim0)
    if o0 is None:
        o0 = "".join(chr(ord("a") + i) for i in range(nd0))
    if o1 is None:
        o1 = "".join(chr(ord("a") + i) for i in range(sto.nd))
    from0 = [0] * nd0 if from0 is None else from0
    size0 = list(dim0) if size0 is None else size0
    from1 = [0] * sto.nd if from1 is None else from1
    _check(_lib.sbx_storage_append_blocks(nd0, sto.nd, _partition(p0, nd0), len(p0), o0.encode(),
                                          _ints(from0), _ints(size0), _ints(dim0), o1.encode(),
                                          _ints(from1), sto.handle, _comm(comm), co))


def save(alpha, p0, o0: str, from0, size0, dim0, v0: Sequence[torch.Tensor], o1: str, from1,
         sto: Storage, co: int = SlowToFast, comm: Optional[Comm] = None):
    """save<Nd0,Nd1,T,Q> (storage.h:2539-2554): write alpha * v0[from0:from0+size0] into the
    stored blocks at from1 (labels o1); values outside the stored blocks are dropped."""
    nprocs, rank = _nprocs_rank(comm)
    nd0 = len(o0)
    nc0 = len(v0)
    if len(p0) != nprocs * nc0:
        raise SuperbblasError("partition is incompatible with the communicator/components")
    _check_sizes(p0, rank, nc0, v0, "save origin")
    t0 = _dtype_of(v0)
    _bind_stream(v0)
    _check(_lib.sbx_storage_save(nd0, sto.nd, _scalar(alpha), t0, _partition(p0, nd0), nc0,
                                 o0.encode(), _ints(from0), _ints(size0), _ints(dim0), _ptrs(v0),
                                 _ctxs(v0), o1.encode(), _ints(from1), sto.handle, _comm(comm),
                                 co, 0))


def load(alpha, sto: Storage, o0: str, from0, size0, p1, o1: str, from1, dim1,
         v1: Sequence[torch.Tensor], co: int = SlowToFast, copyadd: int = Copy,
         comm: Optional[Comm] = None):
    """load<Nd0,Nd1,T,Q> (storage.h:2571-2595): v1[from1 + P(c - from0)] = alpha * sto[c] for
    the stored c in [from0, from0+size0); the rest of v1 is untouched (Add copies as well, as
    the reference's local_load does)."""
    nprocs, rank = _nprocs_rank(comm)
    nd1 = len(o1)
    nc1 = len(v1)
    if len(p1) != nprocs * nc1:
        raise SuperbblasError("partition is incompatible with the communicator/components")
    _check_sizes(p1, rank, nc1, v1, "load destination")
    t1 = _dtype_of(v1)
    _bind_stream(v1)
    _check(_lib.sbx_storage_load(sto.nd, nd1, _scalar(alpha), sto.handle, o0.encode(),
                                 _ints(from0), _ints(size0), t1, _partition(p1, nd1), nc1,
                                 o1.encode(), _ints(from1), _ints(dim1), _ptrs(v1), _ctxs(v1),
                                 _comm(comm), co, copyadd, 0))


def get_blocks(sto: Storage, o0: str, o1: str, from1, size1, co: int = SlowToFast):
    """get_blocks<Nd0,Nd1,T> (storage.h:2608-2617): the stored boxes overlapping
    [from1, from1+size1) of a tensor with labels o1, as (from, size) relative to from1."""
    nd1 = len(o1)
    n = ctypes.c_int()
    _check(_lib.sbx_storage_get_blocks(sto.handle, sto.nd, nd1, o0.encode(), o1.encode(),
                                       _ints(from1), _ints(size1), co, None, 0, ctypes.byref(n)))
    out = _ints([0] * (2 * nd1 * n.value))
    _check(_lib.sbx_storage_get_blocks(sto.handle, sto.nd, nd1, o0.encode(), o1.encode(),
                                       _ints(from1), _ints(size1), co, out, n.value,
                                       ctypes.byref(n)))
    flat = list(out[:2 * nd1 * n.value])
    return [(flat[i * 2 * nd1:i * 2 * nd1 + nd1], flat[i * 2 * nd1 + nd1:(i + 1) * 2 * nd1])
            for i in range(n.value)]


def check_storage(sto: Storage, comm: Optional[Comm] = None):
    """check_storage (storage.h:2439-2446): verify the checksums; raises on a mismatch."""
    _check(_lib.sbx_storage_check(sto.handle, _comm(comm)))


def flush_storage(sto: Storage):
    """flush_storage (storage.h:2434)."""
    _check(_lib.sbx_storage_flush(sto.handle))


def preallocate_storage(sto: Storage, size: int):
    """preallocate_storage (storage.h:2427-2429): extend the file to `size` bytes."""
    _check(_lib.sbx_storage_preallocate(sto.handle, ctypes.c_ulonglong(size)))


def close_storage(sto: Storage, comm: Optional[Comm] = None):
    """close_storage (storage.h:2451-2460): write the pending checksums and release."""
    sto.close(comm)


__all__ = [
    "SlowToFast", "FastToSlow", "Copy", "Add", "RowMajor", "ColumnMajor", "SuperbblasError",
    "Comm", "copy", "copy_plan", "contraction", "local_copy", "xgemm_batch_strided", "create_bsr",
    "create_kron_bsr", "cholesky", "inversion", "trsm", "gesm",
    "bsr_krylov", "bsr_get_preferred_layout", "Request", "wait", "basic_partitioning", "basic_partitioning_ext",
    "partitioning_distributed_procs", "make_hole", "sync", "stream", "set_stream",
    "clear_caches", "timings_enable", "timings_reset", "timings_get", "timings_report",
    "get_gpu_devices_count", "version", "LIB_PATH", "Storage", "NoChecksum", "GlobalChecksum",
    "BlockChecksum", "create_storage", "read_storage_header", "open_storage", "append_blocks",
    "save", "load", "get_blocks", "check_storage", "flush_storage", "preallocate_storage",
    "close_storage",
]
