"""bench.py keeps the driver's command-line contract (no GPU needed: argument parsing only)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_cli_contract():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--help"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    for flag in ("--gpus", "--steps", "--warmup"):
        assert flag in r.stdout


def test_global_fill_partition_invariant():
    """bench.global_fill gives every partition (including periodic wraps) slices of one global
    tensor: the property the N > 1 scale checks rest on"""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    g = [3, 4, 5, 6]
    full = torch.empty(bench.vol(g), dtype=torch.complex128)
    bench.global_fill(full, g, [0] * 4, g, 1)
    f = full.view(*g)
    part = torch.empty(2 * 4 * 3 * 6, dtype=torch.complex128)
    bench.global_fill(part, g, [2, 0, 3, 0], [2, 4, 3, 6], 1)  # wraps in x and z
    assert torch.equal(part.view(2, 4, 3, 6), torch.cat([f[2:3], f[0:1]])[:, :, [3, 4, 0]])
    c64 = torch.empty(bench.vol(g), dtype=torch.complex64)
    bench.global_fill(c64, g, [0] * 4, g, 1)
    assert torch.equal(c64, full.to(torch.complex64))
    other = torch.empty_like(full)
    bench.global_fill(other, g, [0] * 4, g, 2)
    assert not torch.equal(other, full)
    assert full.real.abs().max() <= 1 and full.imag.abs().max() <= 1
    assert abs(full.real.mean().item()) < 0.1 and full.real.std().item() > 0.5


def test_bench_gpus_must_match_launcher():
    """Under a launcher, --gpus must equal its WORLD_SIZE (a silent N = 1 line otherwise);
    unsupported N fail before any rank starts.  No GPU is touched on these paths."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr, r.stderr
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "--gpus 3" in r.stderr, r.stderr


def test_bench_launch_command():
    """Without a launcher, --gpus N > 1 starts torch.distributed.run with N ranks as a child
    process on 127.0.0.1, passing the same arguments through."""
    import unittest.mock as um
    sys.path.insert(0, ROOT)
    import bench
    with um.patch.object(bench.subprocess, "run") as run:
        run.return_value.returncode = 7
        rc = bench.launch_ranks(8, ["--gpus", "8", "--steps", "3"])
    assert rc == 7
    cmd = run.call_args[0][0]
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")
