"""The reference's own test programs compile unchanged against the drop-in header
(include/superbblas.h with its superbblas::detail surface): superbblas's tests/bsr.cpp,
contract.cpp, dist.cpp, blas.cpp, dense.cpp, storage.cpp and storage_details.cpp,
syntax-checked with plain g++ from where they lie under /root/reference (skipped where the reference is absent, e.g. on the GPU box)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference/tests"


@pytest.mark.skipif(not os.path.isdir(REF), reason="the reference is not present here")
@pytest.mark.parametrize("name", ["bsr", "contract", "dist", "blas", "dense", "storage",
                                  "storage_details"])
@pytest.mark.parametrize("std", ["-std=c++14", "-std=c++17"])
def test_reference_caller_compiles(name, std):
    r = subprocess.run(["g++", std, "-fsyntax-only", "-fopenmp", "-I", os.path.join(ROOT, "include"),
                        os.path.join(REF, name + ".cpp")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]


def test_golden_events_cover_invocations():
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from _refcallers import INVOCATIONS, STORAGE_DETAILS, STORAGE_FILES, details_key, key
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "refcallers.json")))
    want = [key(*i) for i in INVOCATIONS]
    want += [details_key(f, a) for f in STORAGE_FILES for a in STORAGE_DETAILS]
    assert sorted(g) == sorted(want)
