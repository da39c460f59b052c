"""The drop-in header compiles as C++14 and C++17 with plain g++ (no HIP headers needed), and
the C ABI header compiles as C."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _compile(args, src, suffix):
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, "t" + suffix)
        with open(f, "w") as fh:
            fh.write(src)
        r = subprocess.run(args + ["-I", os.path.join(ROOT, "include"), "-fsyntax-only", f],
                           capture_output=True, text=True)
        assert r.returncode == 0, r.stderr


def test_dropin_header_compiles():
    src = '#include "superbblas.h"\nint main() { return 0; }\n'
    for std in ("-std=c++14", "-std=c++17"):
        _compile(["g++", std, "-Wall", "-Werror"], src, ".cpp")


def test_dropin_application_compiles():
    with open(os.path.join(ROOT, "tests", "cpp", "dropin_test.cpp")) as f:
        _compile(["g++", "-std=c++14", "-Wall"], f.read(), ".cpp")


def test_c_abi_header_compiles_as_c():
    _compile(["gcc", "-std=c99", "-Wall", "-Werror"],
             '#include "superbblas_amd/sbx.h"\nint main(void) { return sbx_version(0, 0); }\n',
             ".c")


def test_mpi_overloads_typecheck():
    """The SUPERBBLAS_USE_MPI section instantiates against a declarations-only <mpi.h>."""
    with open(os.path.join(ROOT, "tests", "cpp", "mpi_overloads.cpp")) as f:
        _compile(["g++", "-std=c++14", "-Wall", "-DSUPERBBLAS_USE_MPI", "-I",
                  os.path.join(ROOT, "tests", "cpp", "mpi_stub")], f.read(), ".cpp")
