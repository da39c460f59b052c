"""Storage host logic without a GPU: file creation, block appends (overlaps trimmed as the
reference does), headers, reopening, get_blocks and the error paths.  Saves and loads move data
through the GPU and are covered by tests/test_gpu_storage.py."""
import numpy as np
import pytest
import torch

from _golden import manifest, storage_golden_path
from oracle import s3t


def _blocks(st):
    return [[(b["from"], b["size"]) for b in ch] for ch in st["chunks"]]


@pytest.mark.parametrize("case", manifest("storage"), ids=lambda c: c["name"])
def test_append_blocks_like_reference(case, tmp_path):
    """The chunk and block layout of every golden file, rebuilt from its append_blocks calls."""
    import superbblas_amd as sb
    fts = case["co"] == "FastToSlow"
    R = (lambda c: list(c)[::-1]) if fts else list
    fn = str(tmp_path / "a.s3t")
    q = {"cdouble": torch.complex128, "float": torch.float32, "double": torch.float64,
         "cfloat": torch.complex64}[case["q"]]
    sto = sb.create_storage(R(case["dim"]), sb.FastToSlow if fts else sb.SlowToFast, fn,
                            case["meta"].encode(), sb.NoChecksum, q)
    for key in ("blocks1", "blocks2"):
        if case[key]:
            sb.append_blocks(sto, [(R(f), R(s)) for f, s in case[key]], R(case["dim"]),
                             co=sb.FastToSlow if fts else sb.SlowToFast)
    sto.close()
    with open(fn, "rb") as f:
        mine = s3t.parse(f.read())  # unsaved values read as zeros (the file is extended)
    with open(storage_golden_path(case), "rb") as f:
        ref = s3t.parse(f.read())
    assert _blocks(mine) == _blocks(ref)
    assert mine["header_size"] == ref["header_size"] and mine["meta"] == ref["meta"]


def test_header_open_get_blocks(tmp_path):
    import superbblas_amd as sb
    fn = str(tmp_path / "h.s3t")
    dim = [8, 6, 4]
    sto = sb.create_storage(dim, sb.SlowToFast, fn, b"abc\0def", sb.NoChecksum, torch.float32)
    # As the reference (storage.h:1725-1731 with GridHash::intersection, storage.h:611-646), an
    # append removes from the new block both every overlapping stored block and the overlap
    # expressed relative to that block's origin:
    sb.append_blocks(sto, [([6, 0, 0], [4, 6, 4])], dim)  # a in {6, 7, 0, 1} (wraps)
    sb.append_blocks(sto, [([0, 0, 0], [8, 6, 4])], dim)  # holes: a {6, 7, 0, 1} and a [0, 4)
    sb.append_blocks(sto, [([1, 1, 1], [2, 2, 2])], dim)  # holes: a {6, 7, 0, 1} and a {3}
    sto.close()
    t, meta, d = sb.read_storage_header(fn)
    assert (t, meta, d) == (sb.FLOAT, b"abc\0def", dim)
    assert sb.read_storage_header(fn, sb.FastToSlow)[2] == dim[::-1]
    with open(fn, "rb") as f:
        st = s3t.parse(f.read())
    assert _blocks(st) == [[([6, 0, 0], [4, 6, 4])], [([4, 0, 0], [2, 6, 4])],
                           [([2, 1, 1], [1, 2, 2])]]
    sto = sb.open_storage(fn, False)
    assert (sto.nd, sto.dtype) == (3, sb.FLOAT)
    sb.check_storage(sto)
    # every stored box overlapping a region, relative to from1, in the tensor's labels "cab"
    got = sb.get_blocks(sto, "abc", "cab", [0, 5, 0], [4, 4, 6])
    # region a in [5, 9) = {5, 6, 7, 0}: {6, 7, 0} from the first block, {5} from the second
    assert sorted(map(lambda x: (tuple(x[0]), tuple(x[1])), got)) == sorted([
        ((0, 1, 0), (4, 3, 6)), ((0, 0, 0), (4, 1, 6))])
    got = sb.get_blocks(sto, "abc", "abc", [2, 0, 0], [1, 6, 4])
    assert got == [([0, 1, 1], [1, 2, 2])]
    assert sb.get_blocks(sto, "abc", "abc", [0, 0, 0], [0, 6, 4]) == []
    sto.close()


def test_open_errors(tmp_path):
    import superbblas_amd as sb
    fn = str(tmp_path / "e.s3t")
    sto = sb.create_storage([3, 4], sb.SlowToFast, fn, b"", sb.GlobalChecksum, torch.complex64)
    sto.close()
    with pytest.raises(sb.SuperbblasError, match="datatype of the storage"):
        sb.open_storage(fn, False, 2, torch.complex128)
    with pytest.raises(sb.SuperbblasError, match="number of dimensions"):
        sb.open_storage(fn, False, 3, torch.complex64)
    with pytest.raises(sb.SuperbblasError, match="Error opening file"):
        sb.open_storage(str(tmp_path / "none.s3t"), False)
    bad = tmp_path / "bad.s3t"
    bad.write_bytes(b"\1" * 64)
    with pytest.raises(sb.SuperbblasError, match="magic number"):
        sb.read_storage_header(str(bad))
    sto = sb.open_storage(fn, False)
    with pytest.raises(sb.SuperbblasError, match="read-only"):
        sb.append_blocks(sto, [([0, 0], [3, 4])], [3, 4])
    sb.check_storage(sto)
    sto.close()
    # a flipped header byte breaks the global checksum
    buf = bytearray(open(fn, "rb").read())
    buf[8] ^= 0  # values type untouched
    buf[30] ^= 1  # metadata padding / dims region
    open(fn, "wb").write(bytes(buf))
    sto = sb.open_storage(fn, False)
    with pytest.raises(sb.SuperbblasError, match="Checksum failed"):
        sb.check_storage(sto)
    sto.close()


def test_big_endian_file(tmp_path):
    """A byte-swapped file (written on a big-endian host) reads the same (storage.h:1548-1556)."""
    import superbblas_amd as sb
    fn = str(tmp_path / "le.s3t")
    sto = sb.create_storage([2, 3], sb.SlowToFast, fn, b"m", sb.NoChecksum, torch.float64)
    sb.append_blocks(sto, [([0, 1], [2, 2])], [2, 3])
    sto.close()
    le = open(fn, "rb").read()
    st = s3t.parse(le)
    # swap every 4-byte int of the fixed header and every double after it
    be = bytearray(le)
    for i in range(0, 24, 4):
        be[i:i + 4] = be[i:i + 4][::-1]
    start = 24 + 8  # metadata "m" padded to 8
    for i in range(start, len(be), 8):
        be[i:i + 8] = be[i:i + 8][::-1]
    fb = str(tmp_path / "be.s3t")
    open(fb, "wb").write(bytes(be))
    assert sb.read_storage_header(fb) == (sb.DOUBLE, b"m", [2, 3])
    sto = sb.open_storage(fb, False)
    assert sb.get_blocks(sto, "ab", "ab", [0, 0], [2, 3]) == [([0, 1], [2, 2])]
    sto.close()
    assert _blocks(st) == [[([0, 1], [2, 2])]]
