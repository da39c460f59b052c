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
