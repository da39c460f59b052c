#!/usr/bin/env python3
"""Benchmark: lattice contraction GFLOP/s (+ permute GB/s) -- BASELINE.json metric.

Workload (N = 1, default): BASELINE.json configs[1], the 16^4 lattice spin x color contraction
  v0 `tnsxyzc` {16,64,4,16,16,16,3} x v1 `tNSxyzc` -> vr `tNSns` {16,64,4,64,4},
  complex<double>, through superbblas_amd.contraction (the drop-in C-ABI).  One step = one
  contraction call (= one strided batched complex GEMM m = n = 256, k = 12288, batch 16 on MFMA,
  1.031e11 flop).  Inputs are resident in HBM before the timed region.
N > 1 (one process per GPU, RCCL; --config 4a, the default): configs[3], STRONG scaling -- one
  32^4, n = 64 problem (1.649e12 flop per step) split over an xyzt grid 2x1x1x1 / 2x2x1x1 /
  2x2x2x1; xyz is summed, so every rank runs its local batched GEMM and the partial tNSns outputs
  are reduced into rank 0's output through the library's remap communicator (RCCL over xGMI),
  pipelined over t chunks behind the GEMMs.  value = global flops / max-over-ranks time; rank 0
  then runs the same global problem alone (strong_scaling_vs_1gpu).  --config 4b: v1 split over
  t only, redistributed by an all-to-all inside the contraction.
Side measurements (extra fields): N = 1 -- the dist.cpp permute xyztsc -> tnsxyzc (64 slices),
  the 16^4 3x3-block BSR SpMM at n = 1 / 12 / 64 (config 3), the configs[4] chain on one GPU's
  share, the opt-in 3M complex form; N > 1 -- the configs[4] chain over the ranks, the 4b
  redistribution.
cpu_baseline: the real reference (oracle/_ref/ref_bench[_mkl]: header-only superbblas compiled
  here, linked with the image's OpenBLAS or MKL) timed on this box's host cores at configs[1]'s
  exact shape; the oracle restatement when the reference build is absent.
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 matrix (dense), MI355X_MICROARCH.md / BASELINE.md
PEAK_HBM_GBPS = 8000.0    # HBM3E spec


def vol(d):
    n = 1
    for x in d:
        n *= x
    return n


def fill(t, seed):
    g = torch.Generator(device=t.device)
    g.manual_seed(seed)
    r = torch.rand(t.numel(), 2, generator=g, device=t.device, dtype=torch.float64) * 2 - 1
    t.copy_(torch.view_as_complex(r))


_M32 = 0xffffffff


def _mix32(x):
    """32-bit integer finaliser (xor-shift-multiply, 'lowbias32') on int64 tensors holding values
    < 2^32; products wrap in int64, only their low 32 bits are kept."""
    x = x ^ (x >> 16)
    x = (x * 0x7feb352d) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846ca68b) & _M32
    return x ^ (x >> 16)


def global_values(g, seed):
    """val(g): a counter-based complex value in [-1, 1)^2 of the global SlowToFast index g (int64
    tensor).  The same g gives the same value on every rank, GPU and partition."""
    s = (seed * 0x9e3779b9) & _M32
    h = _mix32((g & _M32) ^ _mix32(((g >> 32) + s) & _M32))
    re = _mix32(h ^ 0x5bd1e995)
    im = _mix32(h ^ 0x27d4eb2f)
    sc = 2.0 / 4294967296.0
    return torch.complex(re.double() * sc - 1, im.double() * sc - 1)


def global_fill(t, gdim, frm, size, seed):
    """Fill t, this rank's component `size` at `frm` (periodic) of the global tensor `gdim`
    (SlowToFast), with val(global index): every partition of the tensor -- any number of ranks,
    or one GPU holding it whole -- holds slices of one and the same global tensor (SURVEY §8(c)
    5.1, distribution-invariant inputs).  Chunked over the slowest dimension."""
    nd = len(gdim)
    gstr = [1] * nd
    for d in range(nd - 2, -1, -1):
        gstr[d] = gstr[d + 1] * gdim[d + 1]
    dev = t.device
    off = torch.zeros(1, dtype=torch.int64, device=dev)
    for d in range(1, nd):
        idx = ((frm[d] + torch.arange(size[d], device=dev)) % gdim[d]) * gstr[d]
        off = (off[:, None] + idx[None, :]).reshape(-1)
    chunk = off.numel()
    assert t.numel() == chunk * size[0], (t.numel(), size)
    for i in range(size[0]):
        g = off + ((frm[0] + i) % gdim[0]) * gstr[0]
        t[i * chunk:(i + 1) * chunk] = global_values(g, seed).to(t.dtype)


def rel_err(a, b):
    """Normwise relative difference ||a - b|| / ||b|| (complex, any dtype)."""
    a, b = a.to(torch.complex128), b.to(torch.complex128)
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b)).item()


def host_cpu():
    """Host cores this process may use (its affinity mask, capped by OMP_NUM_THREADS when the box
    sets one), the machine's logical CPU count and the CPU model."""
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    threads = min(avail, int(omp)) if omp and omp.isdigit() and int(omp) > 0 else avail
    model = "unknown"
    cores = set()
    try:
        with open("/proc/cpuinfo") as f:
            phys = core = None
            for line in f:
                if line.startswith("model name") and model == "unknown":
                    model = line.split(":", 1)[1].strip()
                elif line.startswith("physical id"):
                    phys = line.split(":", 1)[1].strip()
                elif line.startswith("core id"):
                    core = line.split(":", 1)[1].strip()
                    cores.add((phys, core))
    except OSError:  # pragma: no cover
        pass
    return {"threads": threads, "affinity_cpus": avail, "nproc": os.cpu_count(), "model": model,
            "physical_cores": len(cores) or None}


REF_EXES = (("openblas", "ref_bench"), ("mkl", "ref_bench_mkl"))


def run_ref(args, threads, blas):
    """One run of the reference's CPU path (oracle/_ref, the real superbblas headers compiled here)
    with `threads` OpenMP threads; returns its JSON line or None."""
    exe = os.path.join(ROOT, "oracle", "_ref", dict(REF_EXES)[blas])
    if not os.path.exists(exe):
        return None
    env = dict(os.environ, OMP_NUM_THREADS=str(threads), OPENBLAS_NUM_THREADS="1",
               MKL_NUM_THREADS="1")
    try:
        out = subprocess.run([exe] + [str(a) for a in args], env=env, timeout=300,
                             capture_output=True, text=True, check=True).stdout
        return json.loads(out.strip().splitlines()[-1])
    except Exception as e:  # pragma: no cover
        print("cpu baseline: %s %s failed: %s" % (blas, args, e), file=sys.stderr)
        return None


def best_ref(args, thread_counts, key):
    """The reference's best configuration over the BLAS libraries of the image and thread counts
    (higher `key` is better); returns (best run, {"blas/threads": value})."""
    best, tried = None, {}
    for blas, _ in REF_EXES:
        for t in thread_counts:
            r = run_ref(args, t, blas)
            if r is None:
                continue
            tried["%s/%d" % (blas, t)] = round(r[key], 3)
            if best is None or r[key] > best[key]:
                best = dict(r, blas=blas)
    return best, tried


def cpu_baseline():
    """The reference's CPU contraction at configs[1]'s exact shape (16^4, n = 64, complex<double>;
    OpenMP over t with one zgemm per t, blas_cpu_tmpl.hpp:468-476) on this box's host cores,
    with the faster of the image's two BLAS libraries; the oracle restatement when the reference
    build is absent."""
    cpu = host_cpu()
    best, tried = best_ref(["contraction", 16, 64, 2], [cpu["threads"]], "gflops")
    if best is not None:
        out = {"value": round(best["gflops"], 2), "unit": "GFLOP/s", "cores": best["threads"],
               "kind": "reference",
               "sample": "superbblas::contraction tnsxyzc x tNSxyzc -> tNSns, 16^4, n=64, "
                         "complex<double>, 2 timed reps after 1 warm-up (OpenMP over t, one "
                         "zgemm per t; BLAS %s)" % best["blas"],
               "blas_tried_GFLOPs": tried, "cpu_model": cpu["model"], "nproc": cpu["nproc"],
               "physical_cores": cpu["physical_cores"], "affinity_cpus": cpu["affinity_cpus"],
               # the headline is the job's CPU share: the GPU box grants 16 host threads per GPU
               # (its OMP_NUM_THREADS); the whole host is not measured, only estimated below
               "threads_policy": "OMP_NUM_THREADS of the box (its CPU share per GPU)"}
        one = run_ref(["contraction", 16, 64, 1], 1, best["blas"])
        if one is not None:
            out["value_1thread"] = round(one["gflops"], 2)
            if cpu["physical_cores"]:
                # an upper bound (perfect scaling over every physical core), NOT a measurement
                out["whole_host_linear_estimate"] = round(one["gflops"] * cpu["physical_cores"], 1)
        return out
    # restatement (oracle/oracle.c) on a small sample
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from _common import oracle_gemm, random_valued
    m = n = 64
    k, b = 1536, 8
    a = random_valued(m * k * b, np.complex128, 1)
    bb = random_valued(n * k * b, np.complex128, 2)
    c = np.zeros(m * n * b, np.complex128)
    t = time.perf_counter()
    oracle_gemm("T", "N", m, n, k, 1.0, a, k, m * k, bb, k, n * k, 0.0, c, m, m * n, b)
    t = time.perf_counter() - t
    return {"value": round(8.0 * m * n * k * b / t / 1e9, 2), "unit": "GFLOP/s",
            "cores": cpu["threads"], "kind": "port",
            "sample": "oracle xgemm_batch_strided 'T','N' 64x64x1536 batch 8",
            "cpu_model": cpu["model"], "nproc": cpu["nproc"]}


def cpu_side_baselines():
    """The reference's CPU path for the side measurements (permute config 2p; BSR config 3 at
    n = 1, 12, 64), timed beside the GPU numbers (rank 0, N = 1).  The BSR builtin loop issues
    one tiny zgemm (zgemv at n = 1) per nonzero block (bsr.h:535-650): both BLAS libraries of the
    image lose time to per-call overhead and get SLOWER with more threads at n = 12 (OpenBLAS
    serialises concurrent calls on its buffer lock), so every (BLAS, threads in {1, all}) pair is
    timed and the best is reported."""
    cpu = host_cpu()
    threads = sorted({1, cpu["threads"]})
    out = {"cpu_reference_threads": cpu["threads"], "cpu_model": cpu["model"]}
    best, tried = best_ref(["permute", 16, 64, 1], [cpu["threads"]], "gbps")
    if best is not None:
        out["permute_cpu_reference_GBps"] = round(best["gbps"], 3)
    for ncols in (1, 12, 64):
        best, tried = best_ref(["bsr", 16, ncols, 2], threads, "gbps")
        if best is not None:
            out["bsr_n%d_cpu_reference_GBps" % ncols] = round(best["gbps"], 3)
            out["bsr_n%d_cpu_reference_best" % ncols] = "%s/%d threads" % (best["blas"],
                                                                           best["threads"])
            out["bsr_n%d_cpu_reference_tried_GBps" % ncols] = tried
    return out


def pmc_traffic(*kernel_substrs):
    """HBM bytes per launch of a kernel from the latest committed PMC pass (profiles/rNN_pmc.json,
    made by tools/pmc_summary.py from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this
    bench).  PMC counters cannot be read inside a timed run, so they come from that pass."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")))
    if not files:
        return None, None
    with open(files[-1]) as f:
        ks = json.load(f)["kernels"]
    for k, v in ks.items():
        if all(sub in k for sub in kernel_substrs):
            return v["hbm_bytes"], os.path.relpath(files[-1], ROOT) + ": " + k
    return None, None


# lattice grids of configs[3] (x, y, z, t split factors)
GRIDS = {1: [1, 1, 1, 1], 2: [2, 1, 1, 1], 4: [2, 2, 1, 1], 8: [2, 2, 2, 1]}
SEED_V0, SEED_V1 = 1, 2
# N > 1 answers against the same global problem on one GPU (complex<double>; the chain is
# complex<float>)
SCALE_TOL, CHAIN_TOL = 1e-10, 1e-5


_T_START = time.perf_counter()


def progress(msg):
    """A progress line on stderr (ranks > 1: every rank), so long multi-rank runs show where
    they are"""
    if int(os.environ.get("WORLD_SIZE", "1")) > 1 or os.environ.get("SBX_BENCH_PROGRESS"):
        print("bench[rank %s +%.1fs]: %s" % (os.environ.get("RANK", "0"),
                                             time.perf_counter() - _T_START, msg),
              file=sys.stderr, flush=True)


def launch_ranks(n, argv):
    """Run this script on n ranks under torch.distributed.run (one process per GPU, rendezvous on
    127.0.0.1) as a child process; rank 0 prints the JSON line to the inherited stdout.  Returns
    the launcher's exit code."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + list(argv)
    sys.stdout.flush()
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", choices=["1", "4a", "4b"], default=None,
                    help="1: configs[1] (16^4 on one GPU, the default at N = 1); 4a: configs[3], "
                         "the 32^4 problem over an xyz grid (the default at N > 1); 4b: the same "
                         "with the second operand over t only (redistributed)")
    ap.add_argument("--L", type=int, default=None)
    # --ncols: the same (--n is ambiguous after torch.distributed.run, which reads abbreviations)
    ap.add_argument("--n", "--ncols", dest="n", type=int, default=64)
    ap.add_argument("--chain-L", dest="chain_L", type=int, default=16,
                    help="configs[4] chain: spatial extent per rank (x, y, z)")
    ap.add_argument("--chain-T", dest="chain_T", type=int, default=64,
                    help="configs[4] chain: time extent")
    ap.add_argument("--no-side", action="store_true", help="skip the side measurements")
    ap.add_argument("--skip", default="",
                    help="comma-separated side measurements to skip (permute, bsr, chain, 3m, "
                         "chain_dist, redistribution, dense, skinny)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline")
    ap.add_argument("--no-1gpu", action="store_true",
                    help="N > 1: skip the same global problem on rank 0's GPU alone")
    ap.add_argument("--share-gpu", choices=["host", "rccl", "nccl"], nargs="?", const="host",
                    default=None,
                    help="rehearsal of the N>1 path on a box with fewer GPUs than ranks: ranks "
                         "share GPUs; 'host': host-staged exchanges over gloo, 'rccl': RCCL "
                         "with one host id per rank (socket transport) under a gloo process "
                         "group, 'nccl': the same RCCL transport under the real start-up "
                         "(init_process_group('nccl', device_id=...)) -- not a bench")
    args = ap.parse_args()

    # --gpus N is the number of ranks: without a launcher, start one (a child process, before
    # anything touches the GPU; never exec) and relay its exit code; under a launcher, its world
    # size must be N (the reference's `mpirun -np N` convention, tests/Makefile:77-84)
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus not in GRIDS:
        print("bench: --gpus %d: the lattice grids are for 1, 2, 4 or 8 GPUs (%s)"
              % (args.gpus, GRIDS), file=sys.stderr)
        sys.exit(2)
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if env_world is not None and int(env_world) != args.gpus:
        print("bench: the launcher started WORLD_SIZE=%s ranks but --gpus %d was asked"
              % (env_world, args.gpus), file=sys.stderr)
        sys.exit(2)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.share_gpu in ("rccl", "nccl"):
        os.environ["NCCL_HOSTID"] = "sbx-bench-rank-%d" % rank
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        os.environ.setdefault("NCCL_IB_DISABLE", "1")
    if args.share_gpu:
        local_rank %= torch.cuda.device_count()
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    import superbblas_amd as sb

    comm = None
    if world > 1:
        import torch.distributed as dist
        if args.share_gpu in ("host", "rccl"):
            dist.init_process_group("gloo")
            comm = (sb.Comm.host_staged(local_rank) if args.share_gpu == "host"
                    else sb.Comm.from_torch_distributed(local_rank))
        else:  # the real start-up (also --share-gpu nccl)
            dist.init_process_group("nccl", device_id=dev)
            comm = sb.Comm.from_torch_distributed(local_rank)

    progress("communicator ready")
    transport = {"kind": "none", "count": 1}
    if comm is not None:
        kind, count, urank = comm.transport()
        transport = {"kind": kind, "count": count}
        if count != world or urank != rank:
            raise SystemExit("bench: the communicator sees %d ranks (this one %d) but the launcher "
                             "started %d (this one %d)" % (count, urank, world, rank))

    config = args.config or ("1" if world == 1 else "4a")
    if config == "1" and world > 1:
        raise SystemExit("configs[1] is the single-GPU workload; use --config 4a/4b at N > 1")
    grid = GRIDS.get(world)
    if grid is None:
        raise SystemExit("unsupported --gpus %d" % world)
    L = args.L or (16 if config == "1" else 32)
    n = args.n
    # one global problem (strong scaling), split over the lattice grid
    gdim0 = [L, n, 4, L, L, L, 3]  # tnsxyzc
    gdimr = [L, n, 4, n, 4]  # tNSns
    procs = [grid[3], 1, 1, grid[0], grid[1], grid[2], 1]
    p0 = sb.basic_partitioning("tnsxyzc", gdim0, procs, "xyzt", world, 1)
    p1 = p0 if config != "4b" else sb.basic_partitioning("tNSxyzc", gdim0,
                                                         [world, 1, 1, 1, 1, 1, 1], "t", world, 1)
    pr = [([0] * 5, gdimr)] + [([0] * 5, [0] * 5)] * (world - 1)  # output on rank 0
    v0 = torch.empty(vol(p0[rank][1]), dtype=torch.complex128, device=dev)
    v1 = torch.empty(vol(p1[rank][1]), dtype=torch.complex128, device=dev)
    vr = torch.zeros(vol(gdimr) if rank == 0 else 1, dtype=torch.complex128, device=dev)
    # slices of two global tensors (the same values at any N, and in single_gpu_time)
    global_fill(v0, gdim0, p0[rank][0], p0[rank][1], SEED_V0)
    global_fill(v1, gdim0, p1[rank][0], p1[rank][1], SEED_V1)
    z7, z5 = [0] * 7, [0] * 5

    def step():
        sb.contraction(1.0, p0, z7, gdim0, gdim0, "tnsxyzc", False, [v0], p1, z7, gdim0, gdim0,
                       "tNSxyzc", False, [v1], 0.0, pr, z5, gdimr, gdimr, "tNSns", [vr],
                       comm=comm)

    def barrier():
        if world > 1:
            torch.distributed.barrier()

    # side measurements first: they also bring the GPU clocks up before the contraction is timed
    # (the first ~10 GEMM launches on an idle GPU run ~12 % slower)
    side = {}
    skip = set(x for x in args.skip.split(",") if x)
    if args.no_side:
        skip |= {"permute", "bsr", "wilson", "chain", "3m", "chain_dist", "redistribution", "dense",
                 "skinny"}
    if world == 1 and "permute" not in skip:
        side.update(permute_bench(sb, dev, 16, 64))
    if world == 1 and "bsr" not in skip:
        side.update(bsr_bench(sb, dev, 16))
    if world == 1 and "wilson" not in skip:
        try:
            side.update(wilson_bench(sb, dev, 16))
        except Exception as e:  # a side measurement never takes the bench down
            side["wilson_error"] = str(e)[:200]
    if world == 1 and "dense" not in skip:
        try:
            side.update(dense_bench(sb, dev))
        except Exception as e:  # a side measurement never takes the bench down
            side["dense_error"] = str(e)[:200]
    if world == 1 and "skinny" not in skip:
        try:
            side.update(skinny_gemm_bench(sb, dev))
        except Exception as e:  # a side measurement never takes the bench down
            side["skinny_error"] = str(e)[:200]
    if world == 1 and "chain" not in skip:
        try:
            side.update(chain_bench(sb, dev))
        except Exception as e:  # a side measurement never takes the bench down
            side["chain_error"] = str(e)[:200]
    # N > 1 results kept on rank 0 for the check against one GPU (scale_check_*)
    results = {}
    if world > 1 and "chain_dist" not in skip:
        progress("chain_dist")
        try:
            side.update(chain_dist_bench(sb, dev, comm, world, rank, grid[:3], barrier,
                                         Ls=args.chain_L, Lt=args.chain_T, check=not args.no_1gpu))
        except Exception as e:  # a side measurement never takes the bench down
            side["chain_dist_error"] = str(e)[:200]
    if world > 1 and config == "4a" and "redistribution" not in skip:
        # configs[3] "4b" beside the 4a headline: v1 over t only, (a) its all-to-all
        # redistribution alone, (b) the contraction that pipelines it behind the GEMMs
        progress("redistribution")
        try:
            side.update(redistribution_bench(sb, dev, comm, world, rank, gdim0, p0, v0, v1, pr,
                                             vr, barrier))
            if rank == 0:
                results["contraction_redistributed"] = vr.clone()
        except Exception as e:  # a side measurement never takes the bench down
            side["redistribution_error"] = str(e)[:200]
    flops_step = flops_of(L, n)
    if world == 1 and "3m" not in skip:
        # the same contraction with complex products in the opt-in 3-multiplication form: a
        # comparison point (not the headline: only a normwise error bound), and ~20 ms of MFMA
        # load right before the timed region
        side.update(form3m_bench(sb, step, flops_step))
    progress("warm-up")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # GEMM launches per step (one untimed step with the library's per-launch timers)
    sb.timings_enable(True)
    sb.timings_filter("gemm_total")
    sb.timings_reset()
    step()
    torch.cuda.synchronize()
    calls_per_step = sb.timings_get("gemm_total")[1]
    sb.timings_enable(False)
    barrier()
    torch.cuda.synchronize()
    # kernel time on the library's (= torch's current) stream by HIP events.  N = 1, where a step
    # is one GEMM launch and its split-K reduce: one event pair around the K timed steps, so the
    # average launch duration is the stream time per step (GEMM + reduce + the launch gaps
    # between them).  Otherwise (N > 1: a step's GEMM is cut in T chunks beside the exchanges)
    # one event pair around every GEMM launch with its reduce ("gemm_total") over K more steps
    # right after the timed ones: those two event records per launch cost ~9 us of stream time
    # each (marker packets between the kernels), so no timed step carries them.
    per_launch = world > 1 or calls_per_step != 1
    ev_start = torch.cuda.Event(enable_timing=True)
    ev_end = torch.cuda.Event(enable_timing=True)
    ev_start.record()
    # the shader clock the timed GEMMs ran at: workgroup 0 of every LDS-DMA GEMM launch sums its
    # s_memtime (shader clock) and s_memrealtime (100 MHz) spans (three vector atomics by one
    # thread per launch), so a slower box can be told apart from a slower kernel
    sb.tune_set("gemm.clock", 1)
    progress("timed steps")
    t0 = time.perf_counter()
    for i in range(args.steps):
        step()
    ev_end.record()
    torch.cuda.synchronize()
    barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cpu" if args.share_gpu in ("host", "rccl") else dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    clk_cycles, clk_ticks = sb.tune_get("gemm.clock_cycles"), sb.tune_get("gemm.clock_ticks")
    clk_launches = sb.tune_get("gemm.clock_launches")
    sb.tune_set("gemm.clock", 0)
    if per_launch:
        progress("per-launch GEMM timing")
        sb.timings_enable(True)
        sb.timings_filter("gemm_total")
        sb.timings_reset()
        for i in range(args.steps):
            step()
        torch.cuda.synchronize()
        barrier()
        gemm_ms, gemm_calls = sb.timings_get("gemm_total")
        sb.timings_enable(False)
    else:
        gemm_ms, gemm_calls = ev_start.elapsed_time(ev_end), args.steps
    sb.timings_filter(None)
    shader_ghz = round(clk_cycles / clk_ticks * 0.1, 4) if clk_ticks > 0 else None
    # one GEMM = the MFMA kernel launch + its split-K reduce (the reduce is part of the GEMM)
    kernel_s = gemm_ms / max(gemm_calls, 1) / 1e3

    value = flops_step * args.steps / elapsed / 1e9  # whole-job: global flops / max-rank time
    # this rank's flops per GEMM launch (a step's GEMM is cut in T chunks when a cross-rank
    # reduction is pipelined behind it) / the launch's average duration
    local_flops = flops_step * vol(p0[rank][1]) / vol(gdim0)
    flops_launch = local_flops * args.steps / max(gemm_calls, 1)
    # executed MFMA flops: the 4-multiplication form (default) issues 4 real multiply-adds per
    # complex MAC (8 flops); the opt-in 3-multiplication form 3 (6 flops)
    m3 = sb.tune_get("gemm.m3") > 0
    exec_per_alg = 6.0 / 8.0 if m3 else 1.0
    algorithmic = flops_launch / kernel_s / 1e12
    achieved = algorithmic * exec_per_alg

    # strong scaling: the same global problem on rank 0's GPU alone (outside the timed region),
    # whose output is also the answer every N > 1 result is checked against
    scaling_fields = {}
    if world > 1 and not args.no_1gpu:
        barrier()
        if rank == 0:
            results[config] = vr.clone()
            progress("same problem on one GPU")
            try:
                t1, ref = single_gpu_time(sb, dev, gdim0, gdimr)
                scaling_fields = {"value_1gpu_same_problem": round(flops_step / t1 / 1e9, 2),
                                  "ms_per_step_1gpu": round(t1 * 1e3, 4),
                                  "strong_scaling_vs_1gpu": round(t1 / (elapsed / args.steps), 3)}
                if side.get("contraction_redistributed_ms"):
                    # configs[3] 4b: the contraction whose second operand is redistributed by an
                    # all-to-all, against the same global problem on one GPU
                    scaling_fields["strong_scaling_vs_1gpu_4b"] = round(
                        t1 * 1e3 / side["contraction_redistributed_ms"], 3)
                for name, r in results.items():
                    scaling_fields["scale_check_rel_err_" + name] = rel_err(r, ref)
                del ref
            except Exception as e:  # pragma: no cover
                scaling_fields = {"single_gpu_error": str(e)[:200]}
            results.clear()
        barrier()
    if world > 1 and rank == 0:
        errs = {k: v for k, v in list(scaling_fields.items()) + list(side.items())
                if k.startswith("scale_check_rel_err")}
        bad = [k for k, v in errs.items()
               if not v <= (CHAIN_TOL if k.endswith("_chain") else SCALE_TOL)]
        scaling_fields["scale_check_ok"] = bool(errs) and not bad
        if bad:
            print("bench: N>1 results differ from the 1-GPU answer: %s"
                  % {k: errs[k] for k in bad}, file=sys.stderr)

    base = None
    if rank == 0 and world == 1 and not args.no_cpu:
        base = cpu_baseline()
        if not {"permute", "bsr"} <= skip:
            side.update(cpu_side_baselines())

    traffic, traffic_src = pmc_traffic("dma_kernel<", "128, 128, 16, 4, 4")
    if world > 1:
        # the committed PMC pass is of the single-GPU configs[1] GEMM; a rank's configs[3] GEMM
        # has another shape (k, batch), so its traffic is not known from it
        traffic, traffic_src = None, ("no PMC pass of the per-rank configs[3] GEMM shape (%s)"
                                      % traffic_src)
    if rank == 0:
        if config == "1":
            workload = ("configs[1]: 16^4 lattice spin x color contraction tnsxyzc x tNSxyzc -> "
                        "tNSns, n=64, complex<double>")
        else:
            workload = ("configs[3] %s: %d^4 lattice contraction tnsxyzc x tNSxyzc -> tNSns, n=%d, "
                        "complex<double>, one global problem, v0 split x%d y%d z%d t%d, v1 %s, "
                        "output on rank 0 (partial outputs reduced over %s)"
                        % (config, L, n, grid[0], grid[1], grid[2], grid[3],
                           "the same" if config == "4a" else "split over t (redistributed to "
                           "v0's partition by an all-to-all)",
                           "RCCL" if args.share_gpu != "host" else
                           "host staging"))
        line = {
            "metric": "lattice contraction GFLOP/s + permute GB/s, 16^4 spin×color, 1/2/4/8 GPUs",
            "value": round(value, 2),
            "unit": "GFLOP/s",
            "n_gpus": world,
            # what the exchanges actually ran on: RCCL's own rank count (ncclCommCount)
            "world_size_seen_by_rccl": transport["count"] if transport["kind"] == "rccl" else None,
            "comm_transport": transport["kind"],
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            # the N > 1 lines strong-scale configs[3]; N = 1 is the single-GPU configs[1] point
            # of the series (there is no scaling at N = 1)
            "scaling": "strong",
            "scaling_note": ("one global 32^4 problem split over the ranks" if world > 1 else
                             "single GPU: configs[1]; the N > 1 lines are strong scaling of "
                             "configs[3]"),
            "vs_baseline": None,
            "dtype": "complex<f64>",
            "data": "synthetic (complex in [-1,1)^2, a counter-based hash of each element's global "
                    "index: identical global tensors at every N)",
            "config": {"workload": workload, "L": L, "n": n,
                       "gemm": "T,N m=n=%d k=%d batch=%d per rank" % (
                           4 * n, vol(p0[rank][1][3:]), p0[rank][1][0]),
                       "parallelism": ("xyzt grid %s" % "x".join(map(str, grid))
                                       if world > 1 else "single GPU")},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 3),
                         "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                         "frac": round(achieved / PEAK_FP64_TFLOPS, 4),
                         "traffic": traffic, "traffic_unit": "bytes per launch",
                         "traffic_source": traffic_src,
                         "algorithmic_bytes": 16.0 * (vol(p0[rank][1]) + vol(p1[rank][1]) +
                                                      vol(gdimr)),
                         "per": ("one GEMM launch of rank 0 (achieved, traffic and "
                                 "algorithmic_bytes are per rank)" if world > 1 else
                                 "one GEMM launch"),
                         "kernel": "gemm_dma_kernel<complex<double>, 128x128x%d, %d waves> (FP64 "
                                   "MFMA 16x16x4, complex %s) + split-K reduce, %d launches, %.4f "
                                   "ms avg (HIP events on its launch stream, %s)" % (
                                       8 if m3 else 16, 8 if m3 else 16, "3M" if m3 else "4M",
                                       gemm_calls, kernel_s * 1e3,
                                       "a pair around every launch, K steps right after the "
                                       "timed ones" if per_launch else
                                       "one pair around the timed steps: GEMM + reduce + launch "
                                       "gaps per step"),
                         "flops_per_launch": flops_launch,
                         "executed_flops_per_launch": flops_launch * exec_per_alg,
                         "algorithmic_TFLOPs": round(algorithmic, 3),
                         "complex_product": ("3-multiplication form (6 executed real flops per "
                                             "complex MAC; value and algorithmic_TFLOPs count 8)"
                                             if m3 else "4-multiplication form (BLAS rounding)"),
                         "gemm_with_reduce_ms_avg": round(gemm_ms / max(gemm_calls, 1), 4),
                         "shader_clock_GHz": shader_ghz,
                         "shader_clock_source": ("s_memtime / s_memrealtime of workgroup 0 over "
                                                 "%d timed GEMM launches" % clk_launches)},
            "cpu_baseline": base,
        }
        line.update(scaling_fields)
        line.update(side)
        if args.share_gpu:
            line["rehearsal"] = ("ranks shared %d GPU(s) (%s exchanges): a test of the N>1 path, "
                                 "not a measurement" % (torch.cuda.device_count(),
                                                        args.share_gpu))
        print(json.dumps(line), flush=True)
    if comm is not None:
        comm.close()
        torch.distributed.destroy_process_group()


def single_gpu_time(sb, dev, gdim0, gdimr, reps=3):
    """The global contraction on this GPU alone (one component per tensor), on the same global
    inputs as the distributed run: the denominator of the strong-scaling figure, timed with HIP
    events on torch's current stream.  Returns (seconds per call, its output)."""
    a = torch.empty(vol(gdim0), dtype=torch.complex128, device=dev)
    b = torch.empty_like(a)
    z = [0] * len(gdim0)
    global_fill(a, gdim0, z, gdim0, SEED_V0)
    global_fill(b, gdim0, z, gdim0, SEED_V1)
    c = torch.empty(vol(gdimr), dtype=torch.complex128, device=dev)
    z7, z5 = [0] * 7, [0] * 5
    q0, qr = [(z7, gdim0)], [(z5, gdimr)]

    def run():
        sb.contraction(1.0, q0, z7, gdim0, gdim0, "tnsxyzc", False, [a], q0, z7, gdim0, gdim0,
                       "tNSxyzc", False, [b], 0.0, qr, z5, gdimr, gdimr, "tNSns", [c])
    run()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        run()
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / 1e3 / reps
    del a, b
    torch.cuda.empty_cache()
    return t, c


def redistribution_bench(sb, dev, comm, world, rank, gdim0, p0, v0, v1, pr, vr, barrier, reps=5):
    """configs[3] with redistribution (N > 1): v1 partitioned over t across the ranks (16/N t
    slices of the whole lattice each) is (a) copied into v0's xyz partition -- the MPI_Alltoallv
    of the reference's copy_request, here RCCL grouped send/recv -- and (b) contracted with v0
    as is, which makes the library redistribute it before the GEMMs (dist.h:3150-3159).
    Bytes moved per rank = the part of v1 that changes owner."""
    pt = sb.basic_partitioning("tNSxyzc", gdim0, [world, 1, 1, 1, 1, 1, 1], "t", world, 1)
    v1t = torch.empty(vol(pt[rank][1]), dtype=torch.complex128, device=dev)
    z7, z5 = [0] * 7, [0] * 5
    gdimr = [gdim0[0], gdim0[1], 4, gdim0[1], 4]
    # t-partitioned copy of v1 (itself an all-to-all), then the timed redistribution back
    sb.copy(1.0, p0, "tNSxyzc", z7, gdim0, gdim0, [v1], pt, "tNSxyzc", z7, gdim0, [v1t], comm=comm)
    tmp = torch.empty_like(v1)

    def redist():
        sb.copy(1.0, pt, "tNSxyzc", z7, gdim0, gdim0, [v1t], p0, "tNSxyzc", z7, gdim0, [tmp],
                comm=comm)

    def contract():
        sb.contraction(1.0, p0, z7, gdim0, gdim0, "tnsxyzc", False, [v0], pt, z7, gdim0, gdim0,
                       "tNSxyzc", False, [v1t], 0.0, pr, z5, gdimr, gdimr, "tNSns", [vr],
                       comm=comm)

    out = {}
    for name, fn in (("redistribute", redist), ("contraction_redistributed", contract)):
        fn()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        barrier()
        out[name + "_ms"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
    ok = bool(torch.equal(tmp, v1))
    # bytes this rank receives: its xyz block minus the t slices it already owned
    moved = 16.0 * vol(p0[rank][1]) * (world - 1) / world
    out["redistribute_GBps_per_rank"] = round(moved / out["redistribute_ms"] / 1e6, 1)
    out["redistribute_exact"] = ok
    del v1t, tmp
    return out


def flops_of(L, n):
    return 8.0 * L * (L ** 3 * 3) * (n * 4) ** 2  # 8 * volT * volA * volB * volC


def form3m_bench(sb, step, flops, reps=15):
    prev = sb.tune_get("gemm.m3")
    sb.tune_set("gemm.m3", 1)
    try:
        step()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            step()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / reps
    finally:
        sb.tune_set("gemm.m3", prev)
    return {"contraction_3M_ms": round(t, 4), "contraction_3M_TFLOPs": round(flops / t / 1e9, 2)}


def permute_bench(sb, dev, L, n, reps=3):
    """dist.cpp:237-266: copy xyztsc into every n-slice of tnsxyzc (complex<double>).
    Timed two ways: eager API calls (host-bound from Python: ~10 us per call) and the same 64
    calls captured once in a HIP graph and replayed (the launch-bound loop as a graph)."""
    d0 = [L, L, L, L, 4, 3]
    d1 = [L, n, 4, L, L, L, 3]
    a = torch.empty(vol(d0), dtype=torch.complex128, device=dev)
    fill(a, 7)
    b = torch.empty(vol(d1), dtype=torch.complex128, device=dev)
    p0, p1 = [([0] * 6, d0)], [([0] * 7, d1)]

    def run():
        for k in range(n):
            sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [a], p1, "tnsxyzc", [0, k, 0, 0, 0, 0, 0],
                    d1, [b])

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) / 1e3 / reps

    t_eager = timed(run)
    # eager from Python (ctypes marshalling per call; the C++ loop below is the reference's shape)
    res = {"permute_eager_python_GBps": round(32.0 * vol(d1) / t_eager / 1e9, 1)}
    try:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            run()
        t = timed(g.replay)
        res["permute_graph"] = True
    except Exception as ex:  # pragma: no cover
        print("permute: graph capture failed (%s); eager timing only" % ex, file=sys.stderr)
        t = t_eager
        res["permute_graph"] = False
    gbps = 32.0 * vol(d1) / t / 1e9
    res.update({"permute_GBps": round(gbps, 1), "permute_frac_hbm": round(gbps / PEAK_HBM_GBPS, 4),
                "permute_ms": round(t * 1e3, 3)})
    # the reference's second variant (tests/dist.cpp:268-300): complex<float> source copied and
    # converted into complex<double> slices; 8 + 16 bytes per element
    af = a.to(torch.complex64)

    def run_f():
        for k in range(n):
            sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [af], p1, "tnsxyzc", [0, k, 0, 0, 0, 0, 0],
                    d1, [b])
    try:
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2):
            run_f()
        t2 = timed(g2.replay)
    except Exception:  # pragma: no cover
        t2 = timed(run_f)
    res["permute_cf2cd_GBps"] = round(24.0 * vol(d1) / t2 / 1e9, 1)

    def graph_time(fn):
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                fn()
            return timed(g.replay)
        except Exception:  # pragma: no cover
            return timed(fn)
    # the reference's own element type (tests/dist.cpp:200, Scalar = complex<float>) and its
    # "overhead" figure: the permute loop against the same bytes copied contiguously into the 64
    # slices (its "dummy copying", dist.cpp:205-235)
    bf = torch.empty(vol(d1), dtype=torch.complex64, device=dev)

    def run_ff():
        for k in range(n):
            sb.copy(1.0, p0, "xyztsc", [0] * 6, d0, d0, [af], p1, "tnsxyzc", [0, k, 0, 0, 0, 0, 0],
                    d1, [bf])
    nel0 = vol(d0)

    def memcpy_f():
        for k in range(n):
            bf[k * nel0:(k + 1) * nel0].copy_(af)

    def memcpy_d():
        for k in range(n):
            b[k * nel0:(k + 1) * nel0].copy_(a)
    t3 = graph_time(run_ff)
    tmf, tmd = graph_time(memcpy_f), graph_time(memcpy_d)
    res.update({"permute_cf2cf_GBps": round(16.0 * vol(d1) / t3 / 1e9, 1),
                "permute_cf2cf_ms": round(t3 * 1e3, 3),
                "memcpy_slices_cf_GBps": round(16.0 * vol(d1) / tmf / 1e9, 1),
                "permute_cf2cf_overhead_vs_memcpy": round(t3 / tmf, 3),
                "memcpy_slices_cd_GBps": round(32.0 * vol(d1) / tmd / 1e9, 1),
                "permute_overhead_vs_memcpy": round(t / tmd, 3)})
    del bf
    # what the slice loop's bytes are: the 12.6 / 25.2 MB source is re-read by all 64 slices and
    # stays in the Infinity Cache (256 MB), so half of the algorithmic bytes never reach HBM; the
    # HBM figures are the write stream of the loop and the whole-tensor permute below
    res["permute_frac_note"] = ("permute_frac_hbm counts 32 B per element (read + write) against "
                                "8 TB/s, but the 25 MB source is re-read from the Infinity Cache "
                                "by every slice; HBM: permute_write_stream_frac_hbm and "
                                "permute_whole_frac_hbm")
    res["permute_write_stream_frac_hbm"] = round(16.0 * vol(d1) / t / 1e9 / PEAK_HBM_GBPS, 4)
    # the whole-tensor permute xyztnsc -> tnsxyzc (1.61 GB, every byte to and from HBM)
    dw = [L, L, L, L, n, 4, 3]
    w = torch.empty(vol(dw), dtype=torch.complex128, device=dev)
    w.view(torch.float64).zero_()

    def run_w():
        sb.copy(1.0, [([0] * 7, dw)], "xyztnsc", [0] * 7, dw, dw, [w], p1, "tnsxyzc", [0] * 7, d1,
                [b])
    tw = timed(run_w)
    del w
    res.update({"permute_whole_GBps": round(32.0 * vol(d1) / tw / 1e9, 1),
                "permute_whole_frac_hbm": round(32.0 * vol(d1) / tw / 1e9 / PEAK_HBM_GBPS, 4),
                "permute_whole_ms": round(tw * 1e3, 3)})
    # the same 64-slice loop called eagerly from C++ through the C ABI (tests/dist.cpp's loop;
    # no Python between calls): the host cost per sbx_copy with the plan / launch caches warm,
    # and the reference's overhead-vs-memcpy ratio of that loop, for both element types
    exe = os.path.join(ROOT, "tools", "capi_overhead")
    if os.path.exists(exe):
        for ty in ("cd", "cf"):
            try:
                r = subprocess.run([exe, "permute", str(L), str(n), "5", ty], timeout=120,
                                   capture_output=True, text=True, check=True).stdout
                r = json.loads(r.strip().splitlines()[-1])
                key = "permute_eager_cpp" if ty == "cd" else "permute_cf2cf_eager_cpp"
                res[key + "_GBps"] = r["GBps"]
                res[key + "_overhead_vs_memcpy"] = r["overhead_vs_memcpy"]
                if ty == "cd":
                    res["permute_eager_cpp_frac_hbm"] = round(r["GBps"] / PEAK_HBM_GBPS, 4)
                    res["capi_host_us_per_copy"] = r["host_us_per_copy"]
            except Exception as e:  # pragma: no cover
                res["permute_eager_cpp_error"] = str(e)[:200]
    return res


def chain_bench(sb, dev, Ls=16, Lt=64, ncols=12, reps=3):
    """configs[4] on one GPU's share (16^3 x 64 sites, = 32^3 x 64 over a 2x2x2 grid),
    complex<float>: (1) redistribute a propagator from `tnsxyzc` into the operator's domain
    layout `pxyztscn`, (2) apply the 9-point 12x12-block (spin 4 x color 3) BSR operator,
    (3) contract the result with its conjugate over the lattice and color into `TSnsN`.
    Stage times from HIP events; the ranks' exchanges are absent on one GPU."""
    s_, c_ = 4, 3
    dims = [Ls, Ls, Ls, Lt]
    V = Ls * Ls * Ls * Lt
    b = s_ * c_
    cf = torch.complex64
    # (1) source propagator tnsxyzc
    dsrc = [Lt, ncols, s_, Ls, Ls, Ls, c_]
    src = torch.empty(vol(dsrc), dtype=cf, device=dev)
    fill_f = torch.empty(vol(dsrc), dtype=torch.complex128, device=dev)
    fill(fill_f, 21)
    src.copy_(fill_f)
    del fill_f
    dx = [1, Ls, Ls, Ls, Lt, s_, c_, ncols]
    x = torch.empty(vol(dx), dtype=cf, device=dev)
    y = torch.empty_like(x)
    # (2) operator: site-major blocks, 9 neighbours (self, -+x, -+y, -+z, -+t)
    sites = np.array(np.unravel_index(np.arange(V), dims)).T
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for sg in (-1, 1):
            cc = sites.copy()
            cc[:, d] = (cc[:, d] + sg) % dims[d]
            jj[:, k, :4] = cc
            k += 1
    vals = torch.empty(V * 9 * b * b, dtype=cf, device=dev)
    vals.real.uniform_(-1, 1)
    vals.imag.uniform_(-1, 1)
    dim = dims + [s_, c_]
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, s_, c_]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False,
                       [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                       [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
    del jj, sites
    # (3) output of the contraction: T S n s N
    dr = [Lt, s_, ncols, s_, ncols]
    vr = torch.empty(vol(dr), dtype=cf, device=dev)
    p_src, p_x, p_r = [([0] * 7, dsrc)], [([0] * 8, dx)], [([0] * 5, dr)]

    def stage1():
        sb.copy(1.0, p_src, "tnsxyzc", [0] * 7, dsrc, dsrc, [src], p_x, "pxyztscn", [0] * 8, dx,
                [x])

    def stage2():
        sb.bsr_krylov(1.0, op, "XYZTSC", "xyztsc", p_x, "pxyztscn", [0] * 8, dx, dx, [x], 0.0,
                      p_x, "pXYZTSCn", [0] * 8, dx, dx, "p", [y])

    def stage3():
        sb.contraction(1.0, p_x, [0] * 8, dx, dx, "pXYZTSCn", True, [y], p_x, [0] * 8, dx, dx,
                       "pXYZTsCN", False, [y], 0.0, p_r, [0] * 5, dr, dr, "TSnsN", [vr])
    stages = (stage1, stage2, stage3)
    # steady state first: ~0.1 s of the chain (clocks ramp over the first launches)
    t_end = time.perf_counter() + 0.1
    while True:
        for f in stages:
            f()
        torch.cuda.synchronize()
        if time.perf_counter() >= t_end:
            break
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    times = [0.0, 0.0, 0.0]
    for _ in range(reps):
        ev[0].record()
        for i, f in enumerate(stages):
            f()
            ev[i + 1].record()
        torch.cuda.synchronize()
        for i in range(3):
            times[i] += ev[i].elapsed_time(ev[i + 1]) / reps
    # the whole chain back to back (stream-ordered, no events between stages: the host's calls
    # overlap the GPU's work), then each stage's kernels alone (library kernel timers, in a
    # second pass: their event pairs cost stream time between the kernels)
    nrep = 10
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(nrep):
        for f in stages:
            f()
    t1.record()
    torch.cuda.synchronize()
    chain_stream_ms = t0.elapsed_time(t1) / nrep
    sb.timings_enable(True)
    sb.timings_filter("copy,bsr,gemm_total")
    sb.timings_reset()
    for _ in range(nrep):
        for f in stages:
            f()
    torch.cuda.synchronize()
    kern = {k: sb.timings_get(k)[0] / nrep for k in ("copy", "bsr", "gemm_total")}
    sb.timings_enable(False)
    sb.timings_filter(None)
    op.destroy()
    # full-size property check of the chain's result: vr[T,S,n,s,N] = sum conj(y[..S..n]) y[..s..N]
    # is Hermitian under (S n) <-> (s N)
    h = vr.view(Lt, s_ * ncols, s_ * ncols)
    herm = (torch.linalg.vector_norm(h - h.conj().transpose(1, 2)) /
            torch.linalg.vector_norm(h)).item()
    by1 = 16.0 * vol(dsrc)
    by2 = 8.0 * (9 * b * b * V + 2 * b * V * ncols) + 4.0 * (10 * V + 1)
    fl2 = 8.0 * 9 * b * b * V * ncols
    fl3 = 8.0 * vol(dr) * Ls * Ls * Ls * c_
    return {"chain_workload": "configs[4] per-GPU share: 16^3x64 sites, n=12, spin 4 x color 3, "
                              "complex<float>; redistribute -> BSR 12x12 9-point -> contraction",
            "chain_ms": round(chain_stream_ms, 3),
            # per stage: events around each stage's Python call (host gaps included)
            "chain_ms_stage_events": [round(t, 3) for t in times],
            # per stage from its kernels' time (library timers)
            "chain_redistribute_ms": round(kern["copy"], 4),
            "chain_redistribute_GBps": round(by1 / (kern["copy"] / 1e3) / 1e9, 1),
            "chain_bsr_ms": round(kern["bsr"], 4),
            "chain_bsr_GBps": round(by2 / (kern["bsr"] / 1e3) / 1e9, 1),
            "chain_bsr_TFLOPs": round(fl2 / (kern["bsr"] / 1e3) / 1e12, 2),
            "chain_contraction_ms": round(kern["gemm_total"], 4),
            "chain_contraction_TFLOPs": round(fl3 / (kern["gemm_total"] / 1e3) / 1e12, 2),
            "chain_hermitian_rel_err": herm}


SEED_SRC, SEED_VALS = 21, 22


def lattice_jj(sites, gdim, dfrom):
    """Block columns of the 9-point operator (self, then -x, +x, -y, +y, -z, +z, -t, +t) of the
    given global sites, relative to the domain's first site `dfrom` (periodic)."""
    jj = np.zeros((len(sites), 9, 6), np.int32)
    jj[:, 0, :4] = (sites - dfrom) % gdim
    k = 1
    for d in range(4):
        for sg in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + sg) % gdim[d]
            jj[:, k, :4] = (c - dfrom) % gdim
            k += 1
    return jj


def chain_global(sb, dev, G, Lt, ncols):
    """configs[4]'s chain on the WHOLE lattice G on this GPU alone, from the same global inputs
    (SEED_SRC, SEED_VALS) as chain_dist_bench: the answer its N-rank result must equal."""
    s_, c_ = 4, 3
    b = s_ * c_
    cf = torch.complex64
    dim = G + [s_, c_]
    dsrc = [Lt, ncols, s_, G[0], G[1], G[2], c_]
    src = torch.empty(vol(dsrc), dtype=cf, device=dev)
    global_fill(src, dsrc, [0] * 7, dsrc, SEED_SRC)
    dx = [1] + G + [s_, c_, ncols]
    x = torch.empty(vol(dx), dtype=cf, device=dev)
    V = vol(G)
    sites = np.array(np.unravel_index(np.arange(V), G)).T
    jj = lattice_jj(sites, np.array(G), np.zeros(4, np.int64))
    del sites
    vals = torch.empty(V * 9 * b * b, dtype=cf, device=dev)
    global_fill(vals, G + [9, b * b], [0] * 6, G + [9, b * b], SEED_VALS)
    full = [([0] * 6, dim)]
    blk = [1, 1, 1, 1, s_, c_]
    op = sb.create_bsr(full, dim, full, dim, blk, blk, False,
                       [torch.full((V,), 9, dtype=torch.int32, device=dev)],
                       [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])
    del jj
    px, z8 = [([0] * 8, dx)], [0] * 8
    sb.copy(1.0, [([0] * 7, dsrc)], "tnsxyzc", [0] * 7, dsrc, dsrc, [src], px, "pxyztscn", z8, dx,
            [x])
    del src
    y = torch.empty_like(x)
    sb.bsr_krylov(1.0, op, "XYZTSC", "xyztsc", px, "pxyztscn", z8, dx, dx, [x], 0.0, px,
                  "pXYZTSCn", z8, dx, dx, "p", [y])
    op.destroy()
    del vals, x
    dr = [Lt, s_, ncols, s_, ncols]
    vr = torch.empty(vol(dr), dtype=cf, device=dev)
    sb.contraction(1.0, px, z8, dx, dx, "pXYZTSCn", True, [y], px, z8, dx, dx, "pXYZTsCN", False,
                   [y], 0.0, [([0] * 5, dr)], [0] * 5, dr, dr, "TSnsN", [vr])
    torch.cuda.synchronize()
    del y
    torch.cuda.empty_cache()
    return vr


def chain_dist_bench(sb, dev, comm, world, rank, grid, barrier, Ls=16, Lt=64, ncols=12, reps=3,
                     check=True):
    """configs[4] on N ranks (weak scaling, 16^3 x 64 sites per rank; N = 8: the 32^3 x 64
    lattice over a 2x2x2 grid), complex<float>: (1) redistribute the propagator from a t
    partition (source `tnsxyzc`, Lt/N t slices per rank) into the operator's xyz partition
    `pxyztscn` (all-to-all), (2) apply the 9-point 12x12-block operator, whose domain partition
    is the image partition plus a one-site halo in x, y, z (halo exchange inside bsr_krylov),
    (3) contract the result with its conjugate over x, y, z and color into `TSnsN` on rank 0
    (partial outputs reduced across the ranks).  Stage times are max-over-ranks wall times."""
    s_, c_ = 4, 3
    b = s_ * c_
    cf = torch.complex64
    G = [Ls * grid[0], Ls * grid[1], Ls * grid[2], Lt]
    dim = G + [s_, c_]
    dsrc = [Lt, ncols, s_, G[0], G[1], G[2], c_]
    psrc = sb.basic_partitioning("tnsxyzc", dsrc, [world, 1, 1, 1, 1, 1, 1], "t", world, 1)
    dx = [1] + G + [s_, c_, ncols]
    px = sb.basic_partitioning("pxyztscn", dx, [1] + grid + [1, 1, 1, 1], "xyz", world, 1)
    src = torch.empty(vol(psrc[rank][1]), dtype=cf, device=dev)
    global_fill(src, dsrc, psrc[rank][0], psrc[rank][1], SEED_SRC)
    x = torch.empty(vol(px[rank][1]), dtype=cf, device=dev)
    y = torch.empty_like(x)
    # operator: image = the rank's xyz block, domain = image + one-site halo in x, y, z
    pi = sb.basic_partitioning("xyztsc", dim, grid + [1, 1, 1], "xyz", world, 1)
    pd = []
    for f, sz in pi:
        f, sz = list(f), list(sz)
        for d in range(3):
            if sz[d] + 2 <= dim[d]:
                sz[d] += 2
                f[d] = (f[d] - 1) % dim[d]
            else:
                sz[d], f[d] = dim[d], 0
        pd.append((f, sz))
    f0, s0 = pi[rank]
    V = vol(s0[:4])
    sites = np.array(np.unravel_index(np.arange(V), s0[:4])).T + np.array(f0[:4])
    gdim = np.array(G)
    jj = lattice_jj(sites, gdim, np.array(pd[rank][0][:4]))
    # the block values of the rank's image sites: a box of the global [x, y, z, t, 9, 144] array
    vals = torch.empty(V * 9 * b * b, dtype=cf, device=dev)
    global_fill(vals, G + [9, b * b], list(f0[:4]) + [0, 0], list(s0[:4]) + [9, b * b],
                SEED_VALS)
    blk = [1, 1, 1, 1, s_, c_]
    iiv = torch.full((V,), 9, dtype=torch.int32, device=dev)
    progress("chain_dist: create_bsr")
    op = sb.create_bsr(pi, dim, pd, dim, blk, blk, False, [iiv],
                       [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals], comm=comm)
    # the same operator split as the reference's create_lattice_split (tests/bsr.cpp:402-545):
    # a core piece (blocks whose column is one of this rank's sites: domain = image, no
    # exchange) and a halo piece (the other blocks: domain = image + halo); the halo piece's
    # exchange runs on the side stream while the core piece's product runs (bsr_krylov request +
    # just_local), then the halo product is added
    nb = np.zeros((V, 9, 4), np.int64)
    nb[:, 0] = sites
    k = 1
    for d in range(4):
        for sg in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + sg) % gdim[d]
            nb[:, k] = c
            k += 1
    lo, sz = np.array(f0[:4]), np.array(s0[:4])
    inside = np.all((nb - lo) % gdim < sz, axis=2)
    jj_core = np.full((V, 9, 6), -1, np.int32)
    jj_core[:, :, :4] = np.where(inside[:, :, None], (nb - lo) % gdim, -1)
    jj_core[:, :, 4:] = np.where(inside[:, :, None], 0, -1)
    jj_halo = jj.copy()
    jj_halo[inside] = -1
    core = sb.create_bsr(pi, dim, pi, dim, blk, blk, False, [iiv],
                         [torch.from_numpy(jj_core.reshape(-1)).to(dev)], [vals], comm=comm)
    halo = sb.create_bsr(pi, dim, pd, dim, blk, blk, False, [iiv],
                         [torch.from_numpy(jj_halo.reshape(-1)).to(dev)], [vals], comm=comm)
    del jj, sites, nb, jj_core, jj_halo
    dr = [Lt, s_, ncols, s_, ncols]
    pr = [([0] * 5, dr)] + [([0] * 5, [0] * 5)] * (world - 1)
    vr = torch.empty(vol(dr) if rank == 0 else 1, dtype=cf, device=dev)
    z7, z8, z5 = [0] * 7, [0] * 8, [0] * 5

    def stage1():
        sb.copy(1.0, psrc, "tnsxyzc", z7, dsrc, dsrc, [src], px, "pxyztscn", z8, dx, [x],
                comm=comm)

    def stage2_whole():
        sb.bsr_krylov(1.0, op, "XYZTSC", "xyztsc", px, "pxyztscn", z8, dx, dx, [x], 0.0, px,
                      "pXYZTSCn", z8, dx, dx, "p", [y], comm=comm)

    def stage2():
        # halo piece first (exchange in flight, product deferred and added), core piece now
        r = sb.bsr_krylov(1.0, halo, "XYZTSC", "xyztsc", px, "pxyztscn", z8, dx, dx, [x], 1.0,
                          px, "pXYZTSCn", z8, dx, dx, "p", [y], comm=comm, request=True)
        sb.bsr_krylov(1.0, core, "XYZTSC", "xyztsc", px, "pxyztscn", z8, dx, dx, [x], 0.0, px,
                      "pXYZTSCn", z8, dx, dx, "p", [y], comm=comm, just_local=True)
        sb.wait(r)

    def stage3():
        sb.contraction(1.0, px, z8, dx, dx, "pXYZTSCn", True, [y], px, z8, dx, dx, "pXYZTsCN",
                       False, [y], 0.0, pr, z5, dr, dr, "TSnsN", [vr], comm=comm)
    # the split application must equal the whole operator's
    progress("chain_dist: redistribute")
    stage1()
    progress("chain_dist: bsr (whole)")
    stage2_whole()
    y_whole = y.clone()
    progress("chain_dist: bsr (split)")
    stage2()
    torch.cuda.synchronize()
    progress("chain_dist: timed")
    split_err = (torch.linalg.vector_norm(y - y_whole) / torch.linalg.vector_norm(y_whole)).item()
    del y_whole
    t_whole = 0.0
    for _ in range(reps):
        barrier()
        t0 = time.perf_counter()
        stage2_whole()
        torch.cuda.synchronize()
        barrier()
        t_whole += (time.perf_counter() - t0) / reps
    stages = (stage1, stage2, stage3)
    for fn in stages:
        fn()
    torch.cuda.synchronize()
    barrier()
    times = [0.0, 0.0, 0.0]
    t_all = time.perf_counter()
    for _ in range(reps):
        for i, fn in enumerate(stages):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            barrier()
            times[i] += (time.perf_counter() - t0) / reps
    t_all = (time.perf_counter() - t_all) / reps
    op.destroy()
    core.destroy()
    halo.destroy()
    out = {"chain_dist_workload": "configs[4]: %dx%dx%dx%d lattice over an xyz grid %s, n=%d, "
                                  "spin 4 x color 3, complex<float>" % (G[0], G[1], G[2], G[3],
                                                                        grid, ncols),
           "chain_dist_ms": t_all * 1e3,
           "chain_dist_bsr_unsplit_ms": t_whole * 1e3,
           "chain_dist_bsr_split_rel_diff": split_err}
    if check:
        # rank 0's TSnsN (after the timed repetitions: split operator, partials reduced over the
        # ranks) against the whole chain on one GPU from the same global inputs
        del x, y, src, vals
        torch.cuda.empty_cache()
        barrier()
        progress("chain_dist: whole chain on one GPU")
        if rank == 0:
            out["scale_check_rel_err_chain"] = rel_err(vr, chain_global(sb, dev, G, Lt, ncols))
        barrier()
    for i, name in enumerate(("redistribute", "bsr", "contraction")):
        out["chain_dist_%s_ms" % name] = times[i] * 1e3
    if world > 1 and dist_available():
        on_cpu = torch.distributed.get_backend() == "gloo"
        t = torch.tensor([out[k] for k in sorted(out) if k.endswith("_ms")], dtype=torch.float64,
                         device="cpu" if on_cpu else dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        for k, v in zip(sorted(k for k in out if k.endswith("_ms")), t.tolist()):
            out[k] = v
    for k in list(out):
        if k.endswith("_ms"):
            out[k] = round(out[k], 3)
    return out


def dist_available():
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def dense_bench(sb, dev, L=16, n=12, reps=5):
    """The dense batched solvers on one 12x12 complex<double> matrix per site of
    the 16^4 lattice (tools/studies/dense_bench.py): inversion and Cholesky, kernel time from the
    library's timers and the whole call (layout copies included); bytes = the matrices in and
    out once."""
    nb = L ** 4
    dim = [nb, n, n]
    full = [([0, 0, 0], dim)]
    g = torch.Generator(device=dev).manual_seed(7)
    a = torch.randn(nb, n, n, dtype=torch.complex128, device=dev, generator=g)
    a0 = (a @ a.conj().transpose(1, 2) + n * torch.eye(n, dtype=torch.complex128, device=dev)).reshape(-1)
    del a
    v = torch.empty_like(a0)
    out = {}
    for op in ("inversion", "cholesky"):
        def f():
            v.copy_(a0)
            getattr(sb, op)(full, dim, "tij", [v], "i", "j")
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        call = (time.perf_counter() - t0) / reps
        # kernel time in a second pass (the timers' event pairs add stream time between kernels)
        sb.timings_enable(True)
        sb.timings_filter("dense")
        sb.timings_reset()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        ms, calls = sb.timings_get("dense")
        sb.timings_enable(False)
        sb.timings_filter(None)
        kern = ms / max(calls, 1) / 1e3
        by = 2.0 * nb * n * n * 16
        out.update({"dense_%s_12x12_kernel_us" % op: round(kern * 1e6, 1),
                    "dense_%s_12x12_kernel_GBps" % op: round(by / kern / 1e9, 1),
                    "dense_%s_12x12_call_us" % op: round(call * 1e6, 1)})
    if sb.tune_get("dense.wave"):
        out["dense_kernel"] = ("inversion: inv_wave_kernel (Gauss-Jordan in registers, a 16-lane row per "
                               "matrix, DPP row broadcasts, in place); Cholesky: potrf_wave_kernel "
                               "(64 / n matrices per wave)")
    out["dense_workload"] = "16^4 matrices of 12x12 complex<double> (one per site), tij, rows i"
    return out


def skinny_gemm_bench(sb, dev, reps=10):
    """The reference's own xgemm_batch_strided sweep shapes (tests/dist.cpp test_gemm, at its
    default lattice: k = 49152 local sites x colors, batch 32, complex<double>): the Krylov inner
    product m = n = 12 ('C', 'N') and the update m = 49152, n = k = 12 ('N', 'N'), on
    gemm_frag_kernel; kernel time (GEMM + split-K reduce) from the library's timers, bytes = the
    operands and the output once."""
    out = {}
    K, batch, s = 49152, 32, 12
    for kind, (m, n, k, ta) in (("inner", (s, s, K, "C")), ("update", (K, s, s, "N"))):
        g = torch.Generator(device=dev).manual_seed(11)
        a = torch.randn(batch * m * k, dtype=torch.complex128, device=dev, generator=g)
        b = torch.randn(batch * k * n, dtype=torch.complex128, device=dev, generator=g)
        c = torch.zeros(batch * m * n, dtype=torch.complex128, device=dev)
        lda = k if ta != "N" else m

        def f():
            sb.xgemm_batch_strided(ta, "N", m, n, k, 1.0, a, lda, m * k, b, k, k * n, 0.0, c, m,
                                   m * n, batch)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        sb.timings_enable(True)
        sb.timings_filter("gemm_total")
        sb.timings_reset()
        for _ in range(reps):
            f()
        torch.cuda.synchronize()
        ms, calls = sb.timings_get("gemm_total")
        sb.timings_enable(False)
        sb.timings_filter(None)
        t = ms / max(calls, 1) / 1e3
        by = 16.0 * batch * (m * k + k * n + m * n)
        out.update({"gemm_%s12_us" % kind: round(t * 1e6, 1),
                    "gemm_%s12_TFLOPs" % kind: round(8.0 * m * n * k * batch / t / 1e12, 2),
                    "gemm_%s12_frac_hbm" % kind: round(by / t / 8e12, 3)})
        del a, b, c
    out["gemm_skinny_workload"] = ("tests/dist.cpp xgemm_batch_strided shapes, complex<double>, "
                                   "batch 32: inner product m = n = 12, k = 49152 (C,N); update "
                                   "m = 49152, n = k = 12 (N,N); gemm_frag_kernel")
    return out


def wilson_bench(sb, dev, L, ncols=12, reps=5):
    """config 3's secondary shapes on the 16^4 lattice, complex<double>, n = 12: the 12x12
    (spin 4 x color 3) block operator (bsr_mfma_dma_kernel) and the same Wilson-like operator in
    Kronecker form (3x3 color blocks x 4x4 spin matrices, bsr_kron_mfma_kernel).  Kernel time
    from the library's HIP-event timers; algorithmic bytes: values, x and y once, the columns."""
    dims = [L, L, L, L]
    V = L ** 4
    sites = np.array(np.unravel_index(np.arange(V), dims)).T
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for sg in (-1, 1):
            cc = sites.copy()
            cc[:, d] = (cc[:, d] + sg) % L
            jj[:, k, :4] = cc
            k += 1
    ii = torch.full((V,), 9, dtype=torch.int32, device=dev)
    jjt = torch.from_numpy(jj.reshape(-1)).to(dev)
    out = {}

    def timed(run):
        # steady state: ~0.1 s of the kernel first (clocks ramp over the first launches)
        t_end = time.perf_counter() + 0.1
        while time.perf_counter() < t_end:
            run()
            torch.cuda.synchronize()
        sb.timings_enable(True)
        sb.timings_filter("bsr")
        sb.timings_reset()
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        ms, calls = sb.timings_get("bsr")
        sb.timings_enable(False)
        sb.timings_filter(None)
        return ms / max(calls, 1) / 1e3

    # 12x12 blocks, x pXYZTSCn -> y pxyztscn
    dim = dims + [4, 3]
    full = [([0] * 6, dim)]
    vals = torch.empty(V * 9 * 144, dtype=torch.complex128, device=dev)
    fill(vals, 31)
    op = sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 4, 3], [1, 1, 1, 1, 4, 3], False, [ii],
                       [jjt], [vals])
    dimx = [1] + dims + [4, 3, ncols]
    x = torch.empty(V * 12 * ncols, dtype=torch.complex128, device=dev)
    fill(x, 32)
    y = torch.empty_like(x)
    px = [([0] * 8, dimx)]
    t = timed(lambda: sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx,
                                    dimx, [x], 0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y]))
    by = 16.0 * (9 * 144 * V + 2 * 12 * V * ncols) + 4.0 * (10 * V + 1)
    out.update({"bsr12_n12_kernel": "bsr_mfma_dma_kernel (12x12 blocks on FP64 MFMA, blocks by "
                                    "LDS-DMA one ahead)",
                "bsr12_n12_kernel_ms": round(t * 1e3, 4),
                "bsr12_n12_kernel_GBps": round(by / t / 1e9, 1),
                "bsr12_n12_kernel_frac_hbm": round(by / t / 1e9 / PEAK_HBM_GBPS, 4),
                "bsr12_n12_algorithmic_bytes": by})
    op.destroy()
    del vals
    # Kronecker form: 3x3 color blocks, Wilson spin matrices (1 -+ gamma_mu, chiral basis)
    i_ = 1j
    g = [np.array([[0, 0, 0, i_], [0, 0, i_, 0], [0, -i_, 0, 0], [-i_, 0, 0, 0]]),
         np.array([[0, 0, 0, -1], [0, 0, 1, 0], [0, 1, 0, 0], [-1, 0, 0, 0]]),
         np.array([[0, 0, i_, 0], [0, 0, 0, -i_], [-i_, 0, 0, 0], [0, i_, 0, 0]]),
         np.array([[0, 0, 1, 0], [0, 0, 0, 1], [1, 0, 0, 0], [0, 1, 0, 0]])]
    ks = [np.eye(4)]
    for gm in g:
        ks += [np.eye(4) - gm, np.eye(4) + gm]
    kron = torch.from_numpy(np.array(ks, np.complex128).reshape(-1)).to(dev)
    dim = dims + [4, 3]
    full = [([0] * 6, dim)]
    cvals = torch.empty(V * 81, dtype=torch.complex128, device=dev)
    fill(cvals, 33)
    blk, kr = [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 4, 1]
    op = sb.create_kron_bsr(full, dim, full, dim, blk, blk, kr, kr, False, [ii], [jjt], [cvals],
                            [kron])
    dimx = [1] + dims + [3, ncols, 4]
    px = [([0] * 8, dimx)]
    t = timed(lambda: sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTCnS", [0] * 8, dimx,
                                    dimx, [x], 0.0, px, "pxyztcns", [0] * 8, dimx, dimx, "p", [y]))
    by = 16.0 * (81 * V + 2 * 12 * V * ncols) + 4.0 * 9 * V
    form = sb.tune_get("bsr.last_kernel")
    out.update({"kron_n12_kernel": ("bsr_kron_spin_kernel (spin first on the VALU, a lane per (row, "
                                    "column) pair, zero spin entries skipped, rows in the XCD order)"
                                    if form == 9 else
                                    ("bsr_kron_mfma_packed_kernel (a wave's 16 column slots over "
                                     "several rows; " if form == 6 else "bsr_kron_mfma_kernel (") +
                                    "color on the VALU, spin on v_mfma_f64_4x4x4_4b)"),
                "kron_n12_kernel_ms": round(t * 1e3, 4),
                "kron_n12_kernel_GBps": round(by / t / 1e9, 1),
                "kron_n12_kernel_frac_hbm": round(by / t / 1e9 / PEAK_HBM_GBPS, 4),
                "kron_n12_algorithmic_bytes": by})
    op.destroy()
    return out


def bsr_operator(sb, dev, L):
    """config 3's operator: 16^4 periodic 9-point stencil, 3x3 blocks, complex<double>."""
    dim = [L, L, L, L, 1, 3]
    V = L ** 4
    sites = np.array(np.unravel_index(np.arange(V), (L, L, L, L))).T
    jj = np.zeros((V, 9, 6), np.int32)
    jj[:, 0, :4] = sites
    k = 1
    for d in range(4):
        for s in (-1, 1):
            c = sites.copy()
            c[:, d] = (c[:, d] + s) % L
            jj[:, k, :4] = c
            k += 1
    ii = np.full(V, 9, np.int32)
    vals = torch.empty(V * 9 * 9, dtype=torch.complex128, device=dev)
    fill(vals, 9)
    full = [([0] * 6, dim)]
    return sb.create_bsr(full, dim, full, dim, [1, 1, 1, 1, 1, 3], [1, 1, 1, 1, 1, 3], False,
                         [torch.from_numpy(ii).to(dev)],
                         [torch.from_numpy(jj.reshape(-1)).to(dev)], [vals])


def bsr_setup(sb, dev, L, ncols, op=None):
    """(op, x, y, run) for one config-3 product y = A x with ncols rhs (run() launches it)."""
    op = op or bsr_operator(sb, dev, L)
    dimx = [1, L, L, L, L, 1, 3, ncols]
    x = torch.empty(vol(dimx), dtype=torch.complex128, device=dev)
    fill(x, 10)
    y = torch.empty_like(x)
    px = [([0] * 8, dimx)]

    def run():
        sb.bsr_krylov(1.0, op, "xyztsc", "XYZTSC", px, "pXYZTSCn", [0] * 8, dimx, dimx, [x],
                      0.0, px, "pxyztscn", [0] * 8, dimx, dimx, "p", [y])
    return op, x, y, run


def bsr_bench(sb, dev, L, ncols_list=(1, 12, 64), reps=5):
    """config 3: 16^4 periodic 9-point stencil, 3x3 blocks, complex<double>, n = 1 / 12 / 64 rhs.
    Kernel time from the library's HIP-event timers on the launch stream; algorithmic bytes
    16 (81 V + 2 3 V n) + 4 (9 V + V + 1) per application."""
    V = L ** 4
    op = bsr_operator(sb, dev, L)
    out = {}
    for ncols in ncols_list:
        _, x, y, run = bsr_setup(sb, dev, L, ncols, op)
        # first launch loads the code object; then ~0.1 s of the kernel to steady clocks
        t_end = time.perf_counter() + 0.1
        while True:
            run()
            torch.cuda.synchronize()
            if time.perf_counter() >= t_end:
                break
        sb.timings_enable(True)
        sb.timings_filter("bsr")
        sb.timings_reset()
        for _ in range(reps):
            run()
        torch.cuda.synchronize()
        bms, bcalls = sb.timings_get("bsr")
        sb.timings_enable(False)
        sb.timings_filter(None)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            run()
        e.record()
        torch.cuda.synchronize()
        t = s.elapsed_time(e) / 1e3 / reps
        flops = 8.0 * 81 * V * ncols
        bytes_ = 16.0 * (81 * V + 2 * 3 * V * ncols) + 4.0 * (9 * V + V + 1)
        tk = bms / max(bcalls, 1) / 1e3
        p = "bsr_n%d_" % ncols
        out[p + "kernel"] = {
            1: "bsr_ell9_row_kernel (one thread per nonzero block, values by LDS-DMA)",
            2: "bsr_ell9_split_kernel (a thread per block row x 3 nonzero blocks x rhs lane, "
               "partial products summed through LDS, XCD halves interleaved)",
            3: "bsr_ell9_kernel (row chunks, values by LDS-DMA, XCD halves interleaved)"}.get(sb.tune_get("bsr.last_kernel"), "other")
        out.update({p + "GFLOPs": round(flops / t / 1e9, 1), p + "GBps": round(bytes_ / t / 1e9, 1),
                    p + "ms": round(t * 1e3, 4), p + "kernel_ms": round(tk * 1e3, 4),
                    p + "kernel_GBps": round(bytes_ / tk / 1e9, 1),
                    p + "kernel_frac_hbm": round(bytes_ / tk / 1e9 / PEAK_HBM_GBPS, 4),
                    p + "algorithmic_bytes": bytes_})
        del x, y
    op.destroy()
    return out


if __name__ == "__main__":
    main()
