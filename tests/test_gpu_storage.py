"""Tensor storage (S3T files) through the library on the GPU.

Golden cases replay oracle/ref_golden.cpp storage_cases: the file the library writes must be
byte-identical to the one the real reference wrote, and loading it back must give the
reference's tensor bit for bit.  Other cases check the files against the S3T restatement
(oracle/s3t.py: every checksum verified on parse) and the loads against numpy."""
import os

import numpy as np
import pytest

from _golden import (NPT, gen, manifest, output, piece, storage_golden_path, storage_tensor,
                     vol)
from oracle import s3t

pytestmark = pytest.mark.gpu


def _torch_dtype(npt):
    import torch
    return {np.complex128: torch.complex128, np.complex64: torch.complex64,
            np.float64: torch.float64, np.float32: torch.float32, np.int32: torch.int32}[npt]


def _scatter(glob, dim, p, gpu, host_odd=False):
    import torch
    return [torch.from_numpy(piece(glob, dim, f, s)).to(
        "cpu" if (host_odd and i % 2) else gpu) for i, (f, s) in enumerate(p)]


def _gather(comps, dim, p, dtype):
    from _golden import put_piece
    g = np.zeros(vol(dim), dtype)
    for (f, s), c in zip(p, comps):
        put_piece(g, dim, f, s, c.cpu().numpy())
    return g


def _rev(case):
    fts = case["co"] == "FastToSlow"
    R = (lambda c: list(c)[::-1]) if fts else (lambda c: list(c))
    RP = lambda p: [(R(f), R(s)) for f, s in p]  # noqa: E731
    RS = (lambda o: o[::-1]) if fts else (lambda o: o)
    return R, RP, RS


@pytest.mark.parametrize("case", manifest("storage"), ids=lambda c: c["name"])
def test_golden_storage(gpu, case, tmp_path):
    import torch
    import superbblas_amd as sb
    R, RP, RS = _rev(case)
    co = sb.FastToSlow if case["co"] == "FastToSlow" else sb.SlowToFast
    t, q = NPT[case["t"]], NPT[case["q"]]
    dim = case["dim"]
    nd = len(dim)
    os_ = "".join(chr(ord("a") + i) for i in range(nd))
    fn = str(tmp_path / case["file"])
    sto = sb.create_storage(R(dim), co, fn, case["meta"].encode(), case["checksum"],
                            _torch_dtype(q))
    sb.append_blocks(sto, RP(case["blocks1"]), R(dim), co=co)
    if case["blocks2"]:
        sb.append_blocks(sto, RP(case["blocks2"]), R(dim), co=co)
    g0 = gen("index", vol(case["dim0"]), 1, t)
    v0 = _scatter(g0, case["dim0"], case["p0"], gpu, host_odd=True)
    alpha = complex(*case["alpha"]) if np.dtype(t).kind == "c" else case["alpha"][0]
    sb.save(alpha, RP(case["p0"]), RS(case["o0"]), R(case["from0"]), R(case["size0"]),
            R(case["dim0"]), v0, RS(os_), R(case["from1"]), sto, co=co)
    sto.close()
    with open(fn, "rb") as f:
        mine = f.read()
    with open(storage_golden_path(case), "rb") as f:
        ref = f.read()
    assert mine == ref

    # header, open, checksums, load back
    vt, meta, d = sb.read_storage_header(fn, co)
    assert meta == case["meta"].encode() and d == R(dim)
    sto2 = sb.open_storage(fn, False, nd, _torch_dtype(q))
    sb.check_storage(sto2)
    ol = case["ol"]
    diml = [dim[os_.index(lab)] for lab in ol]
    gl = gen("int", vol(diml), 2, q)
    vl = _scatter(gl, diml, case["pl"], gpu, host_odd=True)
    sb.load(1.0, sto2, RS(os_), [0] * nd, R(dim), RP(case["pl"]), RS(ol), [0] * nd, R(diml), vl,
            co=co)
    torch.cuda.synchronize()
    out = _gather(vl, diml, case["pl"], q)
    assert np.array_equal(out.view(np.uint8), output(case, q).view(np.uint8))

    # get_blocks lists the stored boxes (relative to from1 = 0 here)
    stored = s3t.parse(ref)
    want = sorted((b["from"], b["size"]) for ch in stored["chunks"] for b in ch)
    got = sorted((list(f), list(s)) for f, s in sb.get_blocks(sto2, RS(os_), os_, [0] * nd, dim,
                                                            co=co))
    assert got == [(list(f), list(s)) for f, s in want]
    sto2.close()


def _roundtrip_file(tmp_path, dim, blocks, checksum, dtype, gpu, name="t.s3t"):
    """Create a storage with `blocks`, save the "index" tensor over the whole of it, close."""
    import torch
    import superbblas_amd as sb
    nd = len(dim)
    o = "".join(chr(ord("a") + i) for i in range(nd))
    fn = str(tmp_path / name)
    sto = sb.create_storage(dim, sb.SlowToFast, fn, b"meta", checksum, dtype)
    sb.append_blocks(sto, blocks, dim)
    g = torch.arange(vol(dim), dtype=torch.float64).to(dtype)
    sb.save(1.0, [([0] * nd, dim)], o, [0] * nd, dim, dim, [g.to(gpu)], o, [0] * nd, sto)
    sto.close()
    return fn, g.numpy()


@pytest.mark.parametrize("checksum", [0, 1, 2])
def test_storage_against_restatement(gpu, tmp_path, checksum):
    """A larger file (several blocks, two chunks, a periodic block) checked by the restatement:
    it parses, its checksums verify, and every block holds the saved values."""
    import torch
    dim = [6, 10, 7, 5]
    blocks = [([0, 0, 0, 0], [3, 10, 7, 5]), ([3, 2, 0, 0], [3, 6, 7, 5]),
              ([3, 8, 0, 0], [3, 4, 7, 5])]  # the last wraps around dimension 1
    fn, g = _roundtrip_file(tmp_path, dim, blocks, checksum, torch.complex128, gpu)
    with open(fn, "rb") as f:
        st = s3t.parse(f.read())
    assert st["checksum"] == checksum and st["dim"] == dim
    flat = [b for ch in st["chunks"] for b in ch]
    assert [(b["from"], b["size"]) for b in flat] == [(list(f), list(s)) for f, s in blocks]
    for b in flat:
        assert np.array_equal(b["values"], piece(g, dim, b["from"], b["size"]))


def test_storage_checksum_blocks(gpu, tmp_path):
    """A block above the 64 MiB checksum block size: the checksum is the CRC of per-64 MiB CRCs
    (storage.h:709-735), verified by the restatement; then corruption is detected."""
    import torch
    import superbblas_amd as sb
    dim = [9, 1024, 1024]  # 72 MiB of float64
    fn, _ = _roundtrip_file(tmp_path, dim, [([0, 0, 0], dim)], 2, torch.float64, gpu)
    with open(fn, "rb") as f:
        buf = bytearray(f.read())
    st = s3t.parse(bytes(buf))
    assert st["chunks"][0][0]["values"].nbytes > st["blocksize"]
    sto = sb.open_storage(fn, False)
    sb.check_storage(sto)
    sto.close()
    buf[st["chunks"][0][0]["disp"] + 70 * 1024 * 1024] ^= 1
    with open(fn, "wb") as f:
        f.write(buf)
    sto = sb.open_storage(fn, False)
    with pytest.raises(sb.SuperbblasError, match="Checksum failed"):
        sb.check_storage(sto)
    sto.close()


def test_storage_global_checksum_corruption(gpu, tmp_path):
    import torch
    import superbblas_amd as sb
    dim = [4, 5, 6]
    fn, _ = _roundtrip_file(tmp_path, dim, [([0, 0, 0], dim)], 1, torch.complex64, gpu)
    sto = sb.open_storage(fn, False)
    sb.check_storage(sto)
    sto.close()
    with open(fn, "r+b") as f:
        f.seek(400)
        c = f.read(1)
        f.seek(400)
        f.write(bytes([c[0] ^ 4]))
    sto = sb.open_storage(fn, False)
    with pytest.raises(sb.SuperbblasError, match="Checksum failed"):
        sb.check_storage(sto)
    sto.close()


def test_storage_block_header_corruption(gpu, tmp_path):
    """A corrupted chunk header fails already when opening (the running header CRC)."""
    import torch
    import superbblas_amd as sb
    dim = [4, 5, 6]
    fn, _ = _roundtrip_file(tmp_path, dim, [([0, 0, 0], [2, 5, 6]), ([2, 0, 0], [2, 5, 6])], 2,
                            torch.float32, gpu)
    with open(fn, "rb") as f:
        st = s3t.parse(f.read())
    # the first from coordinate of the second block, 2.0 -> 3.0 changes the header CRC
    off = st["header_size"] + 8 + 8 + 8 * 6
    with open(fn, "r+b") as f:
        f.seek(off)
        f.write(np.float64(3.0).tobytes())
    with pytest.raises(sb.SuperbblasError, match="Checksum failed"):
        sb.open_storage(fn, False)


def test_storage_subregion_load(gpu, tmp_path):
    """load a periodic sub-region into a permuted, offset, multi-component tensor; elements
    outside the region or not stored keep their values (numpy reference)."""
    import torch
    import superbblas_amd as sb
    dim = [5, 6, 4]
    blocks = [([0, 0, 0], [5, 3, 4]), ([0, 4, 0], [5, 2, 4])]  # rows 3 of "b" never stored
    fn, g = _roundtrip_file(tmp_path, dim, blocks, 0, torch.complex128, gpu)
    S = g.reshape(dim).copy()
    stored = np.zeros(dim, bool)
    stored[:, 0:3, :] = True
    stored[:, 4:6, :] = True
    from0, size0 = [3, 2, 1], [4, 5, 3]  # wraps in a and b
    o1, dim1 = "cxab", [4, 2, 6, 7]
    from1 = [2, 1, 5, 0]
    p1 = [([0, 0, 0, 0], [4, 2, 3, 7]), ([0, 0, 3, 0], [4, 2, 3, 7])]
    init = gen("int", vol(dim1), 3, np.complex128)
    v1 = _scatter(init, dim1, p1, gpu, host_odd=True)
    sto = sb.open_storage(fn, False)
    sb.load(2.0, sto, "abc", from0, size0, p1, o1, from1, dim1, v1)
    torch.cuda.synchronize()
    sto.close()
    ref = init.reshape(dim1).copy()
    for ia in range(size0[0]):
        for ib in range(size0[1]):
            for ic in range(size0[2]):
                a, b, c = (from0[0] + ia) % 5, (from0[1] + ib) % 6, (from0[2] + ic) % 4
                if not stored[a, b, c]:
                    continue
                ref[(from1[0] + ic) % 4, from1[1], (from1[2] + ia) % 6, (from1[3] + ib) % 7] = \
                    2.0 * S[a, b, c]
    out = _gather(v1, dim1, p1, np.complex128)
    assert np.array_equal(out, ref.ravel())


def test_storage_save_subregion_and_append_general(gpu, tmp_path):
    """append_blocks in tensor coordinates (o0 -> o1 at from1), then a save of a sub-region:
    only the stored elements inside the region change; the file re-parses."""
    import torch
    import superbblas_amd as sb
    dim = [6, 4]  # storage "xy"
    fn = str(tmp_path / "g.s3t")
    sto = sb.create_storage(dim, sb.SlowToFast, fn, b"", 2, torch.float64)
    # blocks given on a tensor "yx" (dims 4 x 6) region [1:3) x [0:6), placed at x+2
    sb.append_blocks(sto, [([0, 0], [4, 6])], [4, 6], "yx", [1, 0], [2, 6], "xy", [2, 1])
    t = torch.arange(24, dtype=torch.float64).reshape(4, 6) + 1
    sb.save(1.0, [([0, 0], [4, 6])], "yx", [1, 0], [2, 6], [4, 6], [t.to(gpu)], "xy", [2, 1], sto)
    # a block spanning a whole dimension is indexed from 0 there (GridHash::append_block,
    # storage.h:581-582): get_blocks reports it so and its values start at x = 0, while the
    # chunk header keeps the coordinates as appended (storage.h:1740-1745)
    assert sb.get_blocks(sto, "xy", "xy", [0, 0], dim) == [([0, 1], [6, 2])]
    sto.close()
    with open(fn, "rb") as f:
        st = s3t.parse(f.read())
    (b,) = st["chunks"][0]
    assert b["from"] == [2, 1] and b["size"] == [6, 2]
    want = np.zeros((6, 2))
    for iy in range(2):
        for xs in range(6):
            want[xs, iy] = t[1 + iy, (xs - 2) % 6]
    assert np.array_equal(b["values"].reshape(6, 2), want)


def test_storage_errors(gpu, tmp_path):
    import torch
    import superbblas_amd as sb
    dim = [3, 4]
    fn, _ = _roundtrip_file(tmp_path, dim, [([0, 0], dim)], 0, torch.complex128, gpu)
    with pytest.raises(sb.SuperbblasError, match="does not match with the datatype"):
        sb.open_storage(fn, False, 2, torch.float32)
    with pytest.raises(sb.SuperbblasError, match="number of dimensions"):
        sb.open_storage(fn, False, 3, torch.complex128)
    with pytest.raises(sb.SuperbblasError, match="Error opening file"):
        sb.open_storage(str(tmp_path / "missing.s3t"), False)
    bad = tmp_path / "bad.s3t"
    bad.write_bytes(b"\0" * 64)
    with pytest.raises(sb.SuperbblasError, match="magic number"):
        sb.open_storage(str(bad), False, 2, torch.complex128)
    sto = sb.open_storage(fn, False)
    with pytest.raises(sb.SuperbblasError, match="read-only"):
        sb.append_blocks(sto, [([0, 0], dim)], dim)
    sto.close()


def test_storage_reopen_append(gpu, tmp_path):
    """Open for writing, append a second chunk and save into it; the blocks of both chunks are
    kept and the checksums are rewritten at close."""
    import torch
    import superbblas_amd as sb
    dim = [4, 6]
    fn, g = _roundtrip_file(tmp_path, dim, [([0, 0], [4, 3])], 2, torch.complex128, gpu)
    sto = sb.open_storage(fn, True)
    sb.append_blocks(sto, [([0, 0], [4, 6])], dim)  # only [0:4) x [3:6) is new
    v = torch.full((4, 6), 7 - 1j, dtype=torch.complex128)
    sb.save(1.0, [([0, 0], dim)], "ab", [0, 0], dim, dim, [v.to(gpu)], "ab", [0, 0], sto)
    sb.flush_storage(sto)
    sb.preallocate_storage(sto, 1 << 16)
    sto.close()
    with open(fn, "rb") as f:
        st = s3t.parse(f.read())  # also checks that close truncated the preallocation
    assert [[(b["from"], b["size"]) for b in ch] for ch in st["chunks"]] == \
        [[([0, 0], [4, 3])], [([0, 3], [4, 3])]]
    for ch in st["chunks"]:
        assert np.all(ch[0]["values"] == 7 - 1j)


@pytest.mark.parametrize("case", manifest("storage_general"), ids=lambda c: "general%d" % c["id"])
def test_golden_storage_general(gpu, case, tmp_path):
    """oracle/ref_golden.cpp storage_general_case: append_blocks in tensor coordinates with a
    whole-dimension block at an offset, a trimmed second append, a sub-region save, get_blocks
    and a periodic load over two components (one in host memory)."""
    import torch
    import superbblas_amd as sb
    fn = str(tmp_path / case["file"])
    dim, dt = [6, 4], [4, 6]
    sto = sb.create_storage(dim, sb.SlowToFast, fn, b"", sb.BlockChecksum, torch.float64)
    sb.append_blocks(sto, [([0, 0], dt)], dt, "yx", [1, 0], [2, 6], "xy", [2, 1])
    sb.append_blocks(sto, [([4, 2], [3, 2])], dim)
    t = torch.arange(1, 25, dtype=torch.float64).reshape(4, 6)
    sb.save(1.0, [([0, 0], dt)], "yx", [1, 0], [3, 6], dt, [t.to(gpu)], "xy", [2, 1], sto)
    gb = sb.get_blocks(sto, "xy", "yx", [1, 3], [3, 4])
    assert sorted(gb) == sorted((list(f), list(s)) for f, s in case["get_blocks"])
    sto.close()
    with open(fn, "rb") as f:
        mine = f.read()
    with open(storage_golden_path(case), "rb") as f:
        assert mine == f.read()
    dl = [3, 5]
    gl = gen("int", vol(dl), 2, np.float64)
    vl = _scatter(gl, dl, case["pl"], gpu, host_odd=True)
    sto = sb.open_storage(fn, False)
    sb.load(2.0, sto, "xy", [5, 1], [4, 3], case["pl"], "yx", [0, 1], dl, vl)
    torch.cuda.synchronize()
    sto.close()
    out = _gather(vl, dl, case["pl"], np.float64)
    assert np.array_equal(out, output(case, np.float64))
