"""The drop-in C++ header on the GPU: tests/cpp/dropin_test.cpp is an application written
against include/superbblas.h (superbblas's template API) and compiled with plain g++; it runs a
lattice contraction, a permuting copy into a slice, a BSR stencil product and an error path,
all compared exactly with host loops."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("track_time", ["", "1"])
def test_dropin_application(gpu, track_time):
    """Also run under SB_TRACK_TIME=1 (runtime_features.h:55-68): reportTimings then reports the
    kernels from the first call on, unchanged application code."""
    exe = os.path.join(HERE, "cpp", "dropin_test")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", os.path.join(HERE, "cpp"), "dropin_test"])
    env = dict(os.environ)
    env.pop("SB_TRACK_TIME", None)
    if track_time:
        env["SB_TRACK_TIME"] = track_time
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "DROPIN OK" in r.stdout, (r.stdout, r.stderr)
