"""The drop-in C++ header on the GPU: tests/cpp/dropin_test.cpp is an application written
against include/superbblas.h (superbblas's template API) and compiled with plain g++; it runs a
lattice contraction, a permuting copy into a slice, a BSR stencil product and an error path,
all compared exactly with host loops."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_dropin_application(gpu):
    exe = os.path.join(HERE, "cpp", "dropin_test")
    if not os.path.exists(exe):
        subprocess.check_call(["make", "-C", os.path.join(HERE, "cpp"), "dropin_test"])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "DROPIN OK" in r.stdout, (r.stdout, r.stderr)
