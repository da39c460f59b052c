"""Regenerate tests/golden/refcallers.json: what the reference's own test programs print (timings
blanked) for the invocations of tests/_refcallers.py, run against the reference's own headers
(oracle/_ref/contract and oracle/_ref/test_*, built by `make -C oracle refcallers` from
/root/reference/tests; CPU, OpenBLAS).  Run in the build container, where /root/reference
exists:

    python3 tests/golden/make_refcallers_golden.py
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
from _refcallers import (INVOCATIONS, STORAGE_DETAILS, STORAGE_FILES, details_key,  # noqa: E402
                         events, key)


def main():
    subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "refcallers"])
    out = {}
    for name, args, env in INVOCATIONS:
        exe = os.path.join(ROOT, "oracle", "_ref", "contract" if name == "contract" else "test_" + name)
        e = dict(os.environ, OMP_NUM_THREADS="4", **env)
        # (storage.cpp writes tensor.s3t into its working directory)
        with tempfile.TemporaryDirectory() as wd:
            r = subprocess.run([exe] + args, capture_output=True, text=True, env=e, timeout=600,
                               cwd=wd)
        if r.returncode != 0:
            raise SystemExit("reference %s %s failed: rc %d\n%s" % (name, args, r.returncode, r.stderr))
        out[key(name, args, env)] = events(name, r.stdout)
        print(key(name, args, env), len(out[key(name, args, env)]), "events")
    # storage_details.cpp on the golden storage files: its whole output
    exe = os.path.join(ROOT, "oracle", "_ref", "test_storage_details")
    for fname in STORAGE_FILES:
        for args in STORAGE_DETAILS:
            r = subprocess.run([exe, os.path.join(HERE, fname)] + list(args), capture_output=True,
                               text=True, timeout=120)
            if r.returncode != 0:
                raise SystemExit("reference storage_details %s %s failed: rc %d\n%s"
                                 % (fname, args, r.returncode, r.stderr))
            out[details_key(fname, args)] = r.stdout
            print(details_key(fname, args), len(r.stdout.splitlines()), "lines")
    with open(os.path.join(HERE, "refcallers.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
