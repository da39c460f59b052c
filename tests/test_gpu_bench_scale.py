"""bench.py --gpus N proves its answer: every N > 1 line carries scale_check_rel_err_* fields,
the distributed configs[3] contraction (4a), its redistributing form (4b) and the configs[4]
chain each compared with the same global problem run on one GPU from the same global inputs.

On a 1-GPU test box the two ranks share the GPU and exchange through RCCL's socket transport
(bench.py --share-gpu rccl, one RCCL host id per rank); the library code is the xGMI path's."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("config", ["4a", "4b"])
def test_bench_n2_scale_check(gpu, config):
    env = dict(os.environ, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--config", config, "--L", "8", "--ncols", "16", "--chain-L", "4", "--chain-T", "8",
           "--share-gpu", "rccl"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-6000:])
    line = json.loads([s for s in r.stdout.splitlines() if s.startswith("{")][-1])
    errs = {k: v for k, v in line.items() if k.startswith("scale_check_rel_err")}
    want = {"scale_check_rel_err_" + config, "scale_check_rel_err_chain"}
    if config == "4a":
        want.add("scale_check_rel_err_contraction_redistributed")
    assert set(errs) == want, line
    for k, v in errs.items():
        assert v <= (1e-5 if k.endswith("_chain") else 1e-10), (k, v)
    assert line["scale_check_ok"] is True
    assert line["chain_dist_bsr_split_rel_diff"] < 1e-5


def _bench_no_launcher(n, extra, timeout=420, share="rccl"):
    """bench.py --gpus n run WITHOUT a launcher: it must start the n ranks itself"""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--share-gpu",
           share] + extra
    # the ranks' progress lines (stderr) go to a file under gpurun_out/ when it exists, so a long
    # multi-rank run keeps showing signs of life
    outdir = os.path.join(ROOT, "gpurun_out")
    os.makedirs(outdir, exist_ok=True)
    log = os.path.join(outdir, "bench_n%d.log" % n)
    with open(log, "w") as f:
        r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=f, text=True,
                           timeout=timeout)
    with open(log) as f:
        err = f.read()
    assert r.returncode == 0, (r.stdout[-3000:], err[-6000:])
    lines = [s for s in r.stdout.splitlines() if s.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [2, 4, 8])
def test_bench_gpus_n_launches_ranks(gpu, n):
    """`bench.py --gpus N` with no launcher runs N ranks (configs[3]'s grids 2x1x1x1, 2x2x1x1,
    2x2x2x1 at a reduced lattice), RCCL reports N ranks, and the 4a, 4b-redistributed and chain
    answers match the same global problem on one GPU"""
    line = _bench_no_launcher(n, ["--steps", "2", "--warmup", "1", "--L", "8", "--ncols", "8",
                                  "--chain-L", "4", "--chain-T", "8"])
    assert line["n_gpus"] == n
    assert line["world_size_seen_by_rccl"] == n and line["comm_transport"] == "rccl"
    assert line["config"]["parallelism"] == "xyzt grid " + {2: "2x1x1x1", 4: "2x2x1x1",
                                                           8: "2x2x2x1"}[n]
    errs = {k: v for k, v in line.items() if k.startswith("scale_check_rel_err")}
    assert set(errs) == {"scale_check_rel_err_4a", "scale_check_rel_err_contraction_redistributed",
                         "scale_check_rel_err_chain"}, line
    for k, v in errs.items():
        assert v <= (1e-5 if k.endswith("_chain") else 1e-10), (k, v)
    assert line["scale_check_ok"] is True


@pytest.mark.parametrize("n", [2, 4])
def test_bench_real_startup_nccl_pg(gpu, n):
    """the start-up of the driver's multi-GPU run itself: init_process_group("nccl",
    device_id=dev) plus the library's own RCCL communicator (two per process); only RCCL's
    host ids differ (--share-gpu nccl), so the ranks can share the test box's GPU"""
    line = _bench_no_launcher(n, ["--steps", "2", "--warmup", "1", "--L", "8", "--ncols", "8",
                                  "--chain-L", "4", "--chain-T", "8"], share="nccl")
    assert line["n_gpus"] == n
    assert line["world_size_seen_by_rccl"] == n and line["comm_transport"] == "rccl"
    errs = {k: v for k, v in line.items() if k.startswith("scale_check_rel_err")}
    assert len(errs) == 3 and line["scale_check_ok"] is True, line


def test_bench_scale_command_defaults(gpu):
    """the driver's SCALE command at its defaults -- `bench.py --gpus 8`, nothing else, here with
    the 8 ranks sharing the test box's GPU (--share-gpu nccl: the real init_process_group("nccl")
    start-up, one RCCL host id per rank): 20 timed steps of configs[3] (32^4, n = 64, the 2x2x2x1
    grid), the 4b redistribution and redistributing contraction, and configs[4]'s full 32^3 x 64
    chain, each checked against the same global problem on one GPU (45 s on the GPU box, peak
    146 GB of device memory: profiles/r06_scale8_share_nccl*)"""
    line = _bench_no_launcher(8, [], timeout=900, share="nccl")
    assert line["n_gpus"] == 8 and line["world_size_seen_by_rccl"] == 8
    assert line["steps"] == 20 and line["warmup"] == 10
    assert line["config"]["parallelism"] == "xyzt grid 2x2x2x1" and line["config"]["L"] == 32
    assert line["config"]["n"] == 64
    assert "32x32x32x64" in line["chain_dist_workload"]
    errs = {k: v for k, v in line.items() if k.startswith("scale_check_rel_err")}
    assert set(errs) == {"scale_check_rel_err_4a", "scale_check_rel_err_contraction_redistributed",
                         "scale_check_rel_err_chain"}, line
    for k, v in errs.items():
        assert v <= (1e-5 if k.endswith("_chain") else 1e-10), (k, v)
    assert line["scale_check_ok"] is True
    assert line["strong_scaling_vs_1gpu"] > 0 and line["strong_scaling_vs_1gpu_4b"] > 0
    assert line["redistribute_exact"] is True
