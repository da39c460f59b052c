"""The C-ABI library (libsuperbblas_amd.so) loads on a host without a GPU and exports every entry
point include/superbblas_amd/sbx.h declares.  No compute call is made."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "superbblas_amd", "sbx.h")


def declared_symbols():
    with open(HEADER) as f:
        text = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    return sorted(set(re.findall(r"\b(sbx_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("sbx_copy", "sbx_contraction", "sbx_create_bsr", "sbx_create_kron_bsr", "sbx_bsr_krylov",
              "sbx_copy_masked", "sbx_cholesky", "sbx_trsm", "sbx_gesm", "sbx_inversion",
              "sbx_destroy_bsr", "sbx_comm_create", "sbx_xgemm_batch_strided", "sbx_storage_create",
              "sbx_storage_open", "sbx_storage_append_blocks", "sbx_storage_save",
              "sbx_storage_load", "sbx_storage_get_blocks", "sbx_storage_close"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    import superbblas_amd as sb
    lib = ctypes.CDLL(sb.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_version_and_error_path():
    import superbblas_amd as sb
    assert sb.version() >= (0, 1)
    # an invalid call fails loudly with the library's message (no GPU work involved)
    try:
        sb.make_hole([0, 0], [2, 2], [0], [1], [4, 4])
    except Exception as e:  # wrong rank of the hole: rejected by the wrapper or the library
        assert str(e)
    else:
        raise AssertionError("expected an error")


def test_copy_plan_single_process():
    import superbblas_amd as sb
    dim = [4, 6, 5]
    p = [([0, 0, 0], dim)]
    q = [([0, 0, 0], [5, 4, 6])]
    send, recv, local = sb.copy_plan(p, "xyz", [1, 2, 3], [3, 4, 5], dim, 1, q, "zxy", [0, 0, 0],
                                     [5, 4, 6], 1, 1, 0)
    assert send == [0] and recv == [0] and local == 3 * 4 * 5


def test_checksum_matches_zlib_crc32():
    """sbx_checksum (detail::do_checksum, storage.h:701-731) is the zlib CRC-32, continued from a
    previous value, and with a block size the CRC of the blocks' CRCs (host-only: no GPU call)"""
    import struct
    import zlib
    import superbblas_amd as sb
    lib = ctypes.CDLL(sb.LIB_PATH)
    data = b"Quixote was a great guy" * 37
    out = ctypes.c_uint(0)

    def cs(buf, bs=0, prev=0):
        rc = lib.sbx_checksum(buf, ctypes.c_ulonglong(len(buf)), ctypes.c_ulonglong(bs),
                              ctypes.c_uint(prev), ctypes.byref(out))
        assert rc == 0
        return out.value
    assert cs(data) == zlib.crc32(data)
    assert cs(data[10:], prev=zlib.crc32(data[:10])) == zlib.crc32(data)
    blocks = [data[i:i + 64] for i in range(0, len(data), 64)]
    want = zlib.crc32(b"".join(struct.pack("<I", zlib.crc32(b)) for b in blocks))
    assert cs(data, bs=64) == want


def test_library_has_no_undefined_internal_symbols():
    """every sbx:: function the library calls is defined in it (a shared library links with
    undefined symbols; a missing definition would only fail at load time on the GPU box)"""
    import subprocess
    import superbblas_amd as sb
    r = subprocess.run(["nm", "-C", "-u", sb.LIB_PATH], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    bad = [l for l in r.stdout.splitlines() if "sbx::" in l or " sbx_" in l]
    assert not bad, bad
