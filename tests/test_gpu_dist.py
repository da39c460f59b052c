"""Multi-process GPU parity: copy / contraction / BSR with the data really split across ranks
(tests/dist_worker.py, one process per rank, launched with torch.distributed.run).

The host-staged transport lets the ranks share the one GPU of a test box (RCCL refuses two ranks
on one device); the RCCL transport runs when there is a GPU per rank.  The planner, pack/unpack
kernels, cross-rank reductions and halo exchange are the same code for both transports."""
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


def _run(nprocs, transport):
    env = dict(os.environ, SBX_TEST_TRANSPORT=transport, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(nprocs), "--master-addr", "127.0.0.1", "--master-port",
           str(_free_port()), os.path.join(HERE, "dist_worker.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=420)
    assert r.returncode == 0 and "DIST OK" in r.stdout, (r.stdout[-3000:], r.stderr[-6000:])


@pytest.mark.parametrize("nprocs", [2, 3])
def test_dist_host_staged(gpu, nprocs):
    _run(nprocs, "host")


def test_dist_rccl(gpu):
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip("RCCL transport needs one GPU per rank (this box has %d)"
                    % torch.cuda.device_count())
    _run(2, "rccl")
