"""The reference's own test programs as callers of the drop-in build (shared by the golden
generator and the tests).

tests/refcallers/Makefile compiles superbblas's tests/bsr.cpp, contract.cpp, dist.cpp, blas.cpp,
dense.cpp, storage.cpp and storage_details.cpp, unchanged and from where they lie under /root/reference, against
include/superbblas.h and libsuperbblas_amd.so.  oracle/Makefile (`refcallers`) builds the same
sources against the reference's own headers (CPU, OpenBLAS).  The checks the programs carry
(bsr.cpp:287-352 exact product values at SB_DEBUG=1, contract.cpp:238-271 against a brute-force
contraction, blas.cpp:47-63 copy_n against host loops, storage.cpp:280-351 every value read back
from the file and its metadata, dimensions and type) print "Caught error: ..." or abort; so
what a run prints, with the timings blanked, is compared against what the reference prints for
the same invocation (tests/golden/refcallers.json, tests/golden/make_refcallers_golden.py).
"""
import re

# name, arguments, extra environment -- the invocations of tests/test_gpu_refcallers.py
INVOCATIONS = [
    ("bsr", ["--dim=4 4 4 4 2 3"], {"SB_DEBUG": "1"}),
    ("bsr", ["--dim=4 4 4 4 2 12"], {"SB_DEBUG": "1"}),
    ("bsr", ["--dim=4 4 4 4 3 3", "--components=2"], {"SB_DEBUG": "1"}),
    ("bsr", ["--dim=4 4 4 4 2 12", "--power=2"], {"SB_DEBUG": "1"}),
    ("bsr", ["--dim=6 4 4 6 5 3"], {"SB_DEBUG": "1"}),
    ("dense", ["--dim=4 4 4 4 2 12"], {"SB_DEBUG": "1"}),
    ("dense", ["--dim=2 2 2 2 2 3"], {"SB_DEBUG": "1"}),
    ("dist", ["--dim=8 8 8 8 8", "--reps=2"], {}),
    ("blas", ["--size=1000", "--rep=2"], {}),
    ("storage", [], {}),
] + [("contract", ["--test=%d" % t], {}) for t in
     # spread over both scalar types: 0..663551 real double, 663552.. complex<double>
     (0, 1, 2, 3, 17, 255, 4567, 12345, 55295, 89012, 200001, 345678, 500000, 663551,
      663552, 700001, 888888, 1000000, 1200000, 1327103)] + [
    ("contract", ["--test=%d" % t, "--components=2"], {}) for t in (5, 123457, 777777)]

NUM = re.compile(r"-?\d+(\.\d+)?(e[-+]?\d+)?")


def key(name, args, env):
    return " ".join([name] + args + ["%s=%s" % kv for kv in sorted(env.items())])


def events(name, out):
    """(section, normalised event line) pairs of a run's stdout; a section is "k|marker" for
    the k-th section marker line (">>> CPU tests ...", "- Blocking:", ...)"""
    ev = []
    section, nsec = "", 0
    for line in out.splitlines():
        s = line.strip()
        if s.startswith(">>>") or s.startswith("- "):
            nsec += 1
            section = "%d|%s" % (nsec, NUM.sub("#", s))
            continue
        keep = (s.startswith("Time in") or s.startswith("Caught error")
                or s.startswith("Everything went ok") or s.startswith("*)")
                or (name == "blas" and " in " in s and "GiB/s" in s))
        if not keep:
            continue
        if name == "blas":
            s = s.split("(")[0].strip()  # type and operation; the throughputs follow
        ev.append((section, NUM.sub("#", s)))
    return ev


# storage_details.cpp (the S3T inspection tool) on the golden storage files (tests/golden/*.s3t,
# written by the reference): name, arguments after the file
STORAGE_DETAILS = [("show", "--list-blocks"), ("show", "--only-metadata")]
STORAGE_FILES = ["sto_block.s3t", "sto_block_cf.s3t", "sto_f2s.s3t", "sto_general.s3t",
                 "sto_global.s3t", "sto_plain.s3t"]


def details_key(fname, args):
    return " ".join(["storage_details", fname] + list(args))
