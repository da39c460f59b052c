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
