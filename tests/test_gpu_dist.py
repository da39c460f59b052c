"""Multi-process GPU parity: copy / contraction / BSR with the data really split across ranks
(tests/dist_worker.py, one process per rank, launched with torch.distributed.run).

The host-staged transport lets the ranks share the one GPU of a test box.  The RCCL transport runs
with a GPU per rank, or -- on a 1-GPU box -- with every rank declaring its own RCCL host id
(NCCL_HOSTID; RCCL refuses two ranks of one host on one device), so the ranks exchange through
RCCL's socket transport: the library's RCCL path (grouped ncclSend/ncclRecv on the library and
side streams, the T-chunk pipeline) runs for real, only the wire differs from xGMI.  The planner,
pack/unpack kernels, cross-rank reductions and halo exchange are the same code for both."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(nprocs, transport, cases=None, shared=False, pg=None):
    env = dict(os.environ, SBX_TEST_TRANSPORT=transport, OMP_NUM_THREADS="2")
    if pg:
        env["SBX_TEST_PG"] = pg
    if cases:
        env["SBX_TEST_CASES"] = cases
    if shared:
        env["SBX_RCCL_SHARED_GPU"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(nprocs), "--master-addr", "127.0.0.1", "--master-port",
           str(_free_port()), os.path.join(HERE, "dist_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=420)
    if r.returncode != 0 or "DIST OK" not in r.stdout:
        # keep the whole output of a failed multi-rank run (pytest shows only its tail)
        out = os.path.join(os.path.dirname(HERE), "gpurun_out")
        if os.path.isdir(out):
            with open(os.path.join(out, "dist_fail_%s_%d.log" % (transport, nprocs)), "w") as f:
                f.write(r.stdout + "\n---- stderr ----\n" + r.stderr)
    assert r.returncode == 0 and "DIST OK" in r.stdout, (r.stdout[-3000:], r.stderr[-6000:])


@pytest.mark.parametrize("nprocs", [2, 3])
def test_dist_host_staged(gpu, nprocs):
    _run(nprocs, "host")


def test_dist_host_staged_grid4(gpu):
    """4 ranks on a 2x2x1 lattice grid (bench configs[3] at N=4), golden contractions only"""
    _run(4, "host", cases="golden")


@pytest.mark.parametrize("nprocs", [2, 3, 4])
def test_dist_rccl(gpu, nprocs):
    import torch
    _run(nprocs, "rccl", shared=torch.cuda.device_count() < nprocs)


@pytest.mark.parametrize("nprocs", [4, 8])
def test_dist_rccl_golden_grid(gpu, nprocs):
    """configs[3]'s lattice grids at N = 4 (2x2x1) and N = 8 (2x2x2): the reference's golden
    random-valued contractions with v0 / v1 on the xyz grid (4a) or v1 over t (4b, redistributed)
    over RCCL, both reductions (collective / point-to-point), within 1e-10 per component"""
    import torch
    _run(nprocs, "rccl", cases="golden", shared=torch.cuda.device_count() < nprocs)


def test_dist_peer_host_staged(gpu):
    """two components per rank through the several-GPUs-per-rank path (dist.force_peer)"""
    _run(2, "host", cases="peer")


@pytest.mark.parametrize("nprocs", [2, 4])
def test_dist_rccl_nccl_pg_peer(gpu, nprocs):
    """bench.py's real N > 1 start-up -- init_process_group("nccl", device_id=...) and a second
    RCCL communicator for the library (Comm.from_torch_distributed) -- with the golden
    contractions, the reductions, and two components per rank through the peer path"""
    import torch
    _run(nprocs, "rccl", cases="golden,reduce,peer", shared=torch.cuda.device_count() < nprocs,
         pg="nccl")
