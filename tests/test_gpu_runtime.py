"""Runtime support on the GPU: the scratch cache's cap (the reference's LRU bound, cache.h:237-294,
SB_CACHEGB_GPU), frees away from the allocation stream, and the reference's SB_* environment
flags read by the library itself (runtime_features.h:15-158): SB_TRACK_TIME, SB_DEBUG."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _host_to_device_copy(sb, torch, gpu, n=1 << 18):
    """A copy from a host component: staged through device scratch (n complex<double>)"""
    d = [n]
    src = torch.arange(n, dtype=torch.float64).to(torch.complex128)
    dst = torch.zeros(n, dtype=torch.complex128, device=gpu)
    sb.copy(1.0, [([0], d)], "i", [0], d, d, [src], [([0], d)], "i", [0], d, [dst])
    torch.cuda.synchronize()
    assert torch.equal(dst.cpu(), src)


def test_cache_cap(gpu):
    import torch
    import superbblas_amd as sb
    prev = sb.tune_get("alloc.max_cached")
    try:
        sb.tune_set("alloc.max_cached", 0)
        _host_to_device_copy(sb, torch, gpu)
        cached, live = sb.cache_usage(gpu.index or 0)
        assert cached == 0 and live == 0
        sb.tune_set("alloc.max_cached", 1 << 30)
        _host_to_device_copy(sb, torch, gpu)
        cached, live = sb.cache_usage(gpu.index or 0)
        assert 16 << 18 <= cached <= 1 << 30 and live == 0
        # a cap below the idle bytes returns the least recently freed blocks at the next free
        sb.tune_set("alloc.max_cached", 1 << 10)
        _host_to_device_copy(sb, torch, gpu, n=16)
        cached, _ = sb.cache_usage(gpu.index or 0)
        assert cached <= 1 << 10
    finally:
        sb.tune_set("alloc.max_cached", -1)
    # the default cap: 10 % of the device's memory
    total = torch.cuda.get_device_properties(gpu).total_memory
    assert abs(sb.tune_get("alloc.max_cached") - total // 10) <= total // 100


def test_no_cross_stream_frees_in_single_process_paths(gpu):
    """Every scratch block of the single-process paths is freed on the stream it was allocated
    on (the multi-rank pipelines join their side stream before freeing)."""
    import torch
    import superbblas_amd as sb
    sb.tune_set("alloc.cross_stream_frees", 0)
    _host_to_device_copy(sb, torch, gpu)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        _host_to_device_copy(sb, torch, gpu)
    _host_to_device_copy(sb, torch, gpu)
    torch.cuda.synchronize()
    assert sb.tune_get("alloc.cross_stream_frees") == 0


def _run_py(code, env_extra):
    env = dict(os.environ)
    for k in ("SB_TRACK_TIME", "SB_DEBUG", "SB_CACHEGB_GPU"):
        env.pop(k, None)
    env.update(env_extra)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240,
                       env=env, cwd=ROOT)
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


_PRELUDE = """
import torch, superbblas_amd as sb
gpu = torch.device('cuda', 0)
n = 1 << 18
d = [n]
src = torch.arange(n, dtype=torch.float64).to(torch.complex128)
dst = torch.zeros(n, dtype=torch.complex128, device=gpu)
sb.copy(1.0, [([0], d)], 'i', [0], d, d, [src], [([0], d)], 'i', [0], d, [dst])
torch.cuda.synchronize()
assert torch.equal(dst.cpu(), src)
"""


def test_env_track_time(gpu):
    """SB_TRACK_TIME=1: the library's kernel timers run from the first call"""
    _run_py(_PRELUDE + "ms, calls = sb.timings_get('copy')\nassert calls >= 1 and ms > 0\n"
            "print('OK')\n", {"SB_TRACK_TIME": "1"})
    _run_py(_PRELUDE + "assert sb.timings_get('copy')[1] == 0\nprint('OK')\n", {})


def test_env_cache_gb(gpu):
    """SB_CACHEGB_GPU=0: no idle scratch is kept"""
    _run_py(_PRELUDE + "assert sb.cache_usage(0) == (0, 0)\n"
            "assert sb.tune_get('alloc.max_cached') == 0\nprint('OK')\n", {"SB_CACHEGB_GPU": "0"})
    _run_py(_PRELUDE + "assert sb.tune_get('alloc.max_cached') == 1 << 29\nprint('OK')\n",
            {"SB_CACHEGB_GPU": "0.5"})


def test_env_debug(gpu):
    """SB_DEBUG=1: syncs around copy and contraction; results unchanged"""
    _run_py(_PRELUDE + """
a = torch.randn(4, 6, dtype=torch.complex128, device=gpu)
b = torch.randn(5, 6, dtype=torch.complex128, device=gpu)
c = torch.zeros(4, 5, dtype=torch.complex128, device=gpu)
sb.contraction(1.0, [([0, 0], [4, 6])], [0, 0], [4, 6], [4, 6], 'ik', False, [a],
               [([0, 0], [5, 6])], [0, 0], [5, 6], [5, 6], 'jk', False, [b], 0.0,
               [([0, 0], [4, 5])], [0, 0], [4, 5], [4, 5], 'ij', [c])
torch.cuda.synchronize()
assert torch.allclose(c, a @ b.T, rtol=1e-12, atol=1e-12)
print('OK')
""", {"SB_DEBUG": "1"})


def test_scratch_reuse_across_streams(gpu):
    """Split-K scratch freed on the null stream (no event recorded: a durable stream) and reused at
    once from a caller's stream, and the other way round: the second call's GEMM (short, the same
    scratch size) must not write its partials before the first call's reduce has read them --
    results bit-identical to the same GEMMs run one at a time."""
    import torch
    import superbblas_amd as sb
    m, batch = 256, 16
    ks = (8192, 1024)  # both split over 4 pieces: one 67 MB scratch block each
    g = torch.Generator(device=gpu).manual_seed(3)
    a = [torch.randn(batch * m * k, dtype=torch.complex128, device=gpu, generator=g) for k in ks]
    b = [torch.randn(batch * k * m, dtype=torch.complex128, device=gpu, generator=g) for k in ks]

    def gemm(i, c):
        k = ks[i]
        sb.xgemm_batch_strided("T", "N", m, m, k, 1.0, a[i], k, m * k, b[i], k, k * m, 0.0, c, m,
                               m * m, batch)

    ref = [torch.zeros(batch * m * m, dtype=torch.complex128, device=gpu) for _ in range(2)]
    for i in range(2):
        gemm(i, ref[i])
        torch.cuda.synchronize()
    s = torch.cuda.Stream()
    for rep in range(3):
        for first_on_user_stream in (False, True):
            out = [torch.zeros_like(ref[0]) for _ in range(2)]
            torch.cuda.synchronize()
            if first_on_user_stream:
                with torch.cuda.stream(s):
                    gemm(0, out[0])
                gemm(1, out[1])
            else:
                gemm(0, out[0])
                with torch.cuda.stream(s):
                    gemm(1, out[1])
            torch.cuda.synchronize()
            for i in range(2):
                assert torch.equal(out[i], ref[i]), (rep, first_on_user_stream, i)
