"""s3t.py -- CPU restatement of superbblas's S3T tensor-storage file format.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (superbblas_amd/, include/) imports this file;
only tests/ use it, as the checker of the files the library writes.  It is pinned against files
written by the real reference (tests/golden/*.s3t, made by oracle/ref_golden.cpp storage_cases)
in tests/test_oracle_golden.py: parsing every golden file verifies all of its checksums, and
rebuilding it from the parsed blocks gives the same bytes.

Format (eromero-vlc/superbblas include/superbblas/storage.h:19-54):
  header: int32 magic 314, version 0, values_datatype (storage.h:63: 0 float, 1 double,
          2 complex float, 3 complex double, 4 char, 5 int), checksum type (0 none, 1 global,
          2 per block; storage.h:70), nd, metadata length; metadata; zero padding to 8 bytes;
          nd dims as doubles (SlowToFast); checksum block size as a double   (storage.h:1456-1509)
  double num_chunks                                                       (storage.h:1510-1514)
  chunks: double nblocks, nblocks x (nd doubles from, nd doubles size); the values of each block
          (dense, SlowToFast); with block checksums one double per block      (storage.h:1751-1787)
  with a checksum, a final double: the global checksum, or the running CRC of the header and
  the chunk headers                                             (storage.h:1935-2125)
CRC-32 is zlib's; above the checksum block size a checksum is the CRC of the array of the
uint32 CRCs of each block-size piece (do_checksum, storage.h:700-735).  Little-endian files only
here (the reference also reads byte-swapped ones).
"""
import struct
import zlib

import numpy as np

MAGIC = 314
VTYPES = {0: np.float32, 1: np.float64, 2: np.complex64, 3: np.complex128, 4: np.int8,
          5: np.int32}


class ChecksumError(ValueError):
    pass


def do_checksum(data: bytes, blocksize: int = 0, prev: int = 0) -> int:
    """storage.h:709-735"""
    if blocksize == 0:
        return zlib.crc32(data, prev)
    assert prev == 0
    crcs = [zlib.crc32(data[i:i + blocksize]) for i in range(0, len(data), blocksize)]
    return zlib.crc32(np.array(crcs, np.uint32).tobytes())


def header_bytes(vtype, checksum, dim, meta: bytes, blocksize):
    """storage.h:1456-1509"""
    h = struct.pack("<6i", MAGIC, 0, vtype, checksum, len(dim), len(meta)) + meta
    h += b"\0" * ((8 - len(meta) % 8) % 8)
    h += struct.pack("<%dd" % len(dim), *dim) + struct.pack("<d", blocksize)
    return h


def parse(buf: bytes):
    """Read a whole S3T file and verify every checksum it carries; returns a dict with vtype,
    checksum, meta, dim, blocksize, header_size and chunks = [[{from, size, values, disp}]]."""
    magic, version, vtype, checksum, nd, mlen = struct.unpack_from("<6i", buf, 0)
    if magic != MAGIC:
        raise ValueError("not an S3T file (magic %d)" % magic)
    if version != 0:
        raise ValueError("unsupported version %d" % version)
    off = 24
    meta = buf[off:off + mlen]
    off += mlen + (8 - mlen % 8) % 8
    dim = [int(x) for x in struct.unpack_from("<%dd" % nd, buf, off)]
    off += 8 * nd
    blocksize = int(struct.unpack_from("<d", buf, off)[0])
    off += 8
    header_size = off
    run = do_checksum(buf[:header_size]) if checksum == 2 else 0
    (num_chunks,) = struct.unpack_from("<d", buf, off)
    off += 8
    dt = np.dtype(VTYPES[vtype])
    chunks = []
    for _ in range(int(num_chunks)):
        (nb,) = struct.unpack_from("<d", buf, off)
        nb = int(nb)
        hdr_len = 8 + 16 * nd * nb
        if checksum == 2:
            run = do_checksum(buf[off:off + hdr_len], 0, run)
        fs = struct.unpack_from("<%dd" % (2 * nd * nb), buf, off + 8)
        off += hdr_len
        blocks = []
        for i in range(nb):
            frm = [int(x) for x in fs[2 * nd * i:2 * nd * i + nd]]
            size = [int(x) for x in fs[2 * nd * i + nd:2 * nd * (i + 1)]]
            n = int(np.prod(size)) if size else 1
            vals = np.frombuffer(buf, dt, n, off).copy()
            blocks.append({"from": frm, "size": size, "values": vals, "disp": off})
            off += n * dt.itemsize
        if checksum == 2:
            for b in blocks:
                (c,) = struct.unpack_from("<d", buf, off)
                got = do_checksum(buf[b["disp"]:b["disp"] + b["values"].nbytes], blocksize)
                if float(got) != c:
                    raise ChecksumError("block checksum failed")
                off += 8
        chunks.append(blocks)
    disp = off
    if checksum == 1:
        (c,) = struct.unpack_from("<d", buf, disp)
        if float(do_checksum(buf[:disp], blocksize)) != c:
            raise ChecksumError("global checksum failed")
    elif checksum == 2:
        (c,) = struct.unpack_from("<d", buf, disp)
        if float(run) != c:
            raise ChecksumError("header checksum failed")
    end = disp + (8 if checksum else 0)
    if len(buf) != end:
        raise ValueError("file size %d, expected %d" % (len(buf), end))
    return {"vtype": vtype, "checksum": checksum, "meta": meta, "dim": dim,
            "blocksize": blocksize, "header_size": header_size, "chunks": chunks}


def build(vtype, checksum, dim, meta: bytes, chunks, blocksize=64 * 1024 * 1024):
    """Serialize a storage: chunks = [[(from, size, values)]] in append order."""
    dt = np.dtype(VTYPES[vtype])
    out = bytearray(header_bytes(vtype, checksum, dim, meta, blocksize))
    run = do_checksum(bytes(out)) if checksum == 2 else 0
    out += struct.pack("<d", len(chunks))
    nd = len(dim)
    for blocks in chunks:
        hdr = struct.pack("<d", len(blocks))
        for frm, size, _ in blocks:
            hdr += struct.pack("<%dd" % (2 * nd), *(list(frm) + list(size)))
        if checksum == 2:
            run = do_checksum(hdr, 0, run)
        out += hdr
        raw = [np.ascontiguousarray(v, dt).tobytes() for _, _, v in blocks]
        for r in raw:
            out += r
        if checksum == 2:
            for r in raw:
                out += struct.pack("<d", float(do_checksum(r, blocksize)))
    if checksum == 1:
        out += struct.pack("<d", float(do_checksum(bytes(out), blocksize)))
    elif checksum == 2:
        out += struct.pack("<d", float(run))
    return bytes(out)
