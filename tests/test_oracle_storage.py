"""Pin the S3T restatement (oracle/s3t.py) against the files the real reference wrote
(tests/golden/*.s3t, oracle/ref_golden.cpp storage_cases).  CPU only.

For every golden file: all checksums verify; every stored block holds exactly the values the
case saved (alpha * the "index" tensor, permuted, at a periodic offset, converted to the storage
type); the loaded tensor is the initial tensor overwritten by the stored blocks; and rebuilding
the file from its blocks gives the same bytes.  Corrupting a value byte must fail the check."""
import numpy as np
import pytest

from _golden import (NPT, gen, manifest, output, piece, storage_golden_path, storage_loaded,
                     storage_tensor)
from oracle import s3t

CASES = manifest("storage")


def _read(case):
    with open(storage_golden_path(case), "rb") as f:
        return f.read()


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_golden_file_parses(case):
    buf = _read(case)
    assert len(buf) == case["file_bytes"]
    st = s3t.parse(buf)  # raises on any checksum mismatch
    assert st["checksum"] == case["checksum"]
    assert st["meta"] == case["meta"].encode()
    assert st["dim"] == case["dim"]
    assert s3t.VTYPES[st["vtype"]] == NPT[case["q"]]
    S = storage_tensor(case)
    for blocks in st["chunks"]:
        for b in blocks:
            assert np.array_equal(b["values"], piece(S.ravel(), case["dim"], b["from"], b["size"]))
    blocks = [(b["from"], b["size"], b["values"]) for ch in st["chunks"] for b in ch]
    out = storage_loaded(case, blocks)
    ref = output(case, NPT[case["q"]])
    assert np.array_equal(out.view(np.uint8), ref.view(np.uint8))


@pytest.mark.parametrize("case", CASES, ids=lambda c: c["name"])
def test_golden_file_rebuilds(case):
    buf = _read(case)
    st = s3t.parse(buf)
    chunks = [[(b["from"], b["size"], b["values"]) for b in ch] for ch in st["chunks"]]
    again = s3t.build(st["vtype"], st["checksum"], st["dim"], st["meta"], chunks, st["blocksize"])
    assert again == buf


@pytest.mark.parametrize("case", [c for c in CASES if c["checksum"]], ids=lambda c: c["name"])
def test_golden_file_corruption_detected(case):
    buf = bytearray(_read(case))
    st = s3t.parse(bytes(buf))
    b = st["chunks"][0][0]
    buf[b["disp"] + 3] ^= 0x10
    with pytest.raises(s3t.ChecksumError):
        s3t.parse(bytes(buf))


GENERAL = manifest("storage_general")


def _general_storage():
    """Storage "xy" (6 x 4) of oracle/ref_golden.cpp storage_general_case as (stored mask,
    values): t = 1..24 on "yx" (4 x 6), y in [1, 4) saved at (x + 2, y)."""
    t = np.arange(1, 25, dtype=np.float64).reshape(4, 6)
    S = np.zeros((6, 4))
    for y in range(1, 4):
        for x in range(6):
            S[(x + 2) % 6, y] = t[y, x]
    stored = np.zeros((6, 4), bool)
    stored[:, 1:3] = True  # the first block: y in [1, 3), every x
    stored[[4, 5, 0], 3] = True  # the second, trimmed to y = 3
    return stored, S


@pytest.mark.parametrize("case", GENERAL, ids=lambda c: "general%d" % c["id"])
def test_golden_general_file(case):
    with open(storage_golden_path(case), "rb") as f:
        buf = f.read()
    st = s3t.parse(buf)
    assert [[(b["from"], b["size"]) for b in ch] for ch in st["chunks"]] == \
        [[([2, 1], [6, 2])], [([4, 3], [3, 1])]]
    stored, S = _general_storage()
    # a block spanning the whole x is laid out from x = 0 (GridHash::append_block normalises
    # its origin, storage.h:581-582), whatever its chunk header says
    b0, b1 = st["chunks"][0][0], st["chunks"][1][0]
    assert np.array_equal(b0["values"].reshape(6, 2), S[:, 1:3])
    assert np.array_equal(b1["values"], S[[4, 5, 0], 3])
    chunks = [[(b["from"], b["size"], b["values"]) for b in ch] for ch in st["chunks"]]
    assert s3t.build(st["vtype"], st["checksum"], st["dim"], st["meta"], chunks,
                     st["blocksize"]) == buf
    # the load: x in [5, 9), y in [1, 4) -> "yx" (3 x 5) at (0, 1), alpha 2, unstored untouched
    L = gen("int", 15, 2, np.float64).reshape(3, 5)
    for iy in range(3):
        for ix in range(4):
            x, y = (5 + ix) % 6, 1 + iy
            if stored[x, y]:
                L[iy, 1 + ix] = 2 * S[x, y]
    assert np.array_equal(L.ravel(), output(case, np.float64))
