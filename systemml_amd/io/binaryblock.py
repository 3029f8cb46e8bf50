"""The reference's "binary" on-disk matrix format: a Hadoop SequenceFile of
(MatrixIndexes, MatrixBlock) records, one record per blocksize x blocksize tile (reference:
runtime/io/{ReaderBinaryBlock,WriterBinaryBlock}.java, runtime/matrix/data/MatrixIndexes.java
and MatrixBlock.write / readFields).  Models and data saved by SystemML in binary format
load here, and matrices written here load in SystemML.

Container (uncompressed SequenceFile, version 6):
    "SEQ" 0x06 | Text key class | Text value class | bool compressed | bool block-compressed |
    int metadata count (+ Text pairs) | 16-byte sync marker |
    records: int record length (-1: sync escape + 16 sync bytes) | int key length | key | value
Key   MatrixIndexes: long row-block index, long col-block index (1-based)
Value MatrixBlock:   int rows | int cols | byte type, then
    EMPTY (0)        nothing
    ULTRA_SPARSE (1) int nnz, then (int i, int j, double v) per non-zero (cols > 1) or
                     (int i, double v) (single column)
    SPARSE (2)       nnz as int (long if rows*cols > 2^31-1), then per row: int n, n x (int j, double v)
    DENSE (3)        rows*cols doubles, row-major
All numbers big-endian (Java DataOutput).
"""
from __future__ import annotations

import os
import struct

import numpy as np

MAGIC = b"SEQ\x06"
KEY_CLASS = "org.apache.sysml.runtime.matrix.data.MatrixIndexes"
VALUE_CLASS = "org.apache.sysml.runtime.matrix.data.MatrixBlock"
SYNC_INTERVAL = 2000          # Hadoop SequenceFile.SYNC_INTERVAL (100 x (4 + 16) bytes)
EMPTY, ULTRA_SPARSE, SPARSE, DENSE = range(4)


def is_sequence_file(path):
    f = _files(path)
    if not f:
        return False
    with open(f[0], "rb") as fh:
        return fh.read(3) == b"SEQ"


def _files(path):
    if os.path.isdir(path):
        return sorted(os.path.join(path, f) for f in os.listdir(path)
                      if not f.startswith((".", "_")) and not f.endswith(".crc") and
                      os.path.isfile(os.path.join(path, f)))
    return [path] if os.path.exists(path) else []


# ----------------------------------------------------------------------------- reading
class _Buf:
    __slots__ = ("b", "p")

    def __init__(self, b):
        self.b = b
        self.p = 0

    def take(self, n):
        v = self.b[self.p:self.p + n]
        if len(v) != n:
            raise EOFError
        self.p += n
        return v

    def i32(self):
        return struct.unpack(">i", self.take(4))[0]

    def i64(self):
        return struct.unpack(">q", self.take(8))[0]

    def u8(self):
        return self.take(1)[0]

    def vint(self):
        """Hadoop WritableUtils.readVInt."""
        first = struct.unpack(">b", self.take(1))[0]
        if first >= -112:
            return first
        neg = first < -120
        n = (-119 - first) if neg else (-111 - first)
        v = 0
        for _ in range(n - 1):
            v = (v << 8) | self.u8()
        return ~v if neg else v

    def text(self):
        return bytes(self.take(self.vint())).decode("utf-8")


def _header(buf):
    if buf.take(3) != b"SEQ":
        raise ValueError("not a SequenceFile")
    version = buf.u8()
    if version < 5:
        raise ValueError(f"unsupported SequenceFile version {version}")
    kc, vc = buf.text(), buf.text()
    compressed, block_comp = buf.u8(), buf.u8()
    if compressed or block_comp:
        raise ValueError("compressed SequenceFiles are not supported")
    for _ in range(buf.i32()):
        buf.text()
        buf.text()
    sync = buf.take(16)
    return kc, vc, sync


def _read_block(v, rows, cols):
    """MatrixBlock.readFields -> (rlen, clen, dense ndarray | (i, j, v) triples)."""
    rlen, clen = v.i32(), v.i32()
    t = v.u8()
    if t == EMPTY:
        return rlen, clen, None
    if t == DENSE:
        a = np.frombuffer(v.take(8 * rlen * clen), dtype=">f8").astype(np.float64).reshape(rlen, clen)
        return rlen, clen, a
    if t == SPARSE:
        nnz = v.i64() if rlen * clen > 0x7FFFFFFF else v.i32()
        ii, jj, vv = [], [], []
        for r in range(rlen):
            n = v.i32()
            if n:
                rec = np.frombuffer(v.take(12 * n), dtype=np.dtype([("j", ">i4"), ("v", ">f8")]))
                ii.append(np.full(n, r, dtype=np.int64))
                jj.append(rec["j"].astype(np.int64))
                vv.append(rec["v"].astype(np.float64))
        if not ii:
            return rlen, clen, None
        return rlen, clen, (np.concatenate(ii), np.concatenate(jj), np.concatenate(vv))
    if t == ULTRA_SPARSE:
        nnz = v.i32()
        if clen > 1:
            rec = np.frombuffer(v.take(16 * nnz), dtype=np.dtype([("i", ">i4"), ("j", ">i4"), ("v", ">f8")]))
            return rlen, clen, (rec["i"].astype(np.int64), rec["j"].astype(np.int64), rec["v"].astype(np.float64))
        rec = np.frombuffer(v.take(12 * nnz), dtype=np.dtype([("i", ">i4"), ("v", ">f8")]))
        return rlen, clen, (rec["i"].astype(np.int64), np.zeros(nnz, dtype=np.int64), rec["v"].astype(np.float64))
    raise ValueError(f"invalid MatrixBlock type {t}")


def iter_blocks(path):
    """Yield (row-block index, col-block index, rlen, clen, payload) for every record."""
    for f in _files(path):
        with open(f, "rb") as fh:
            data = fh.read()
        buf = _Buf(memoryview(data))
        kc, vc, sync = _header(buf)
        if not kc.endswith("MatrixIndexes") or not vc.endswith("MatrixBlock"):
            raise ValueError(f"{f}: SequenceFile of {kc} -> {vc}, not a binary-block matrix")
        while buf.p < len(data):
            rl = buf.i32()
            if rl == -1:                      # sync escape
                buf.take(16)
                continue
            kl = buf.i32()
            key = _Buf(buf.take(kl))
            bi, bj = key.i64(), key.i64()
            val = _Buf(buf.take(rl - kl))
            rlen, clen, payload = _read_block(val, 0, 0)
            yield bi, bj, rlen, clen, payload


def read_binary_block(path, rows=-1, cols=-1, brlen=1000, bclen=1000, row_range=None):
    """Dense float64 matrix (numpy) of a binary-block file / directory.  row_range=(s, e):
    only the rows [s, e) are materialised (blocks outside are skipped) -- the per-rank read
    of an SPMD run."""
    blocks = list(iter_blocks(path))
    if rows < 0 or cols < 0:
        rows = max(((bi - 1) * brlen + rl for bi, _, rl, _, _ in blocks), default=0)
        cols = max(((bj - 1) * bclen + cl for _, bj, _, cl, _ in blocks), default=0)
    s, e = (0, rows) if row_range is None else row_range
    out = np.zeros((e - s, cols))
    for bi, bj, rl, cl, payload in blocks:
        r0, c0 = (bi - 1) * brlen, (bj - 1) * bclen
        if payload is None or r0 >= e or r0 + rl <= s:
            continue
        if isinstance(payload, np.ndarray):
            a, b = max(r0, s), min(r0 + rl, e)
            out[a - s:b - s, c0:c0 + cl] = payload[a - r0:b - r0]
        else:
            i, j, v = payload
            gi = i + r0
            keep = (gi >= s) & (gi < e)
            out[gi[keep] - s, j[keep] + c0] = v[keep]
    return out


# ----------------------------------------------------------------------------- writing
def _vint(n):
    """Hadoop WritableUtils.writeVInt (n >= 0 here)."""
    if -112 <= n <= 127:
        return struct.pack(">b", n)
    length, tmp, neg = -112, n, n < 0
    if neg:
        tmp = ~n
        length = -120
    t = tmp
    while t:
        t >>= 8
        length -= 1
    out = [struct.pack(">b", length)]
    nbytes = (-(length + 120)) if length < -120 else (-(length + 112))
    for k in range(nbytes - 1, -1, -1):
        out.append(bytes([(tmp >> (8 * k)) & 0xFF]))
    return b"".join(out)


def _text(s):
    b = s.encode("utf-8")
    return _vint(len(b)) + b


def _block_bytes(a):
    """MatrixBlock.write of a dense block (sparse on disk below 40% density, as
    MatrixBlock.evalSparseFormatOnDisk)."""
    rlen, clen = a.shape
    nnz = int(np.count_nonzero(a))
    head = struct.pack(">ii", rlen, clen)
    if nnz == 0:
        return head + bytes([EMPTY])
    if nnz < 0.4 * rlen * clen and rlen * clen >= 1:
        ii, jj = np.nonzero(a)
        if nnz < rlen and clen > 1:           # ultra-sparse: ijv triples
            rec = np.empty(nnz, dtype=np.dtype([("i", ">i4"), ("j", ">i4"), ("v", ">f8")]))
            rec["i"], rec["j"], rec["v"] = ii, jj, a[ii, jj]
            return head + bytes([ULTRA_SPARSE]) + struct.pack(">i", nnz) + rec.tobytes()
        parts = [head, bytes([SPARSE]),
                 struct.pack(">q", nnz) if rlen * clen > 0x7FFFFFFF else struct.pack(">i", nnz)]
        counts = np.bincount(ii, minlength=rlen)
        pos = 0
        for r in range(rlen):
            n = int(counts[r])
            parts.append(struct.pack(">i", n))
            if n:
                rec = np.empty(n, dtype=np.dtype([("j", ">i4"), ("v", ">f8")]))
                rec["j"] = jj[pos:pos + n]
                rec["v"] = a[r, jj[pos:pos + n]]
                parts.append(rec.tobytes())
                pos += n
        return b"".join(parts)
    return head + bytes([DENSE]) + np.ascontiguousarray(a, dtype=">f8").tobytes()


def write_binary_block(path, a, brlen=1000, bclen=1000):
    """Write a 2-D array as one uncompressed SequenceFile of binary blocks."""
    a = np.asarray(a, dtype=np.float64)
    sync = os.urandom(16)
    out = [MAGIC, _text(KEY_CLASS), _text(VALUE_CLASS), b"\x00\x00", struct.pack(">i", 0), sync]
    pos = sum(len(x) for x in out)
    last_sync = pos
    rows, cols = a.shape
    for bi in range(max(1, -(-rows // brlen))):
        for bj in range(max(1, -(-cols // bclen))):
            blk = a[bi * brlen:(bi + 1) * brlen, bj * bclen:(bj + 1) * bclen]
            if pos >= last_sync + SYNC_INTERVAL:        # SequenceFile.Writer.checkAndWriteSync
                out += [struct.pack(">i", -1), sync]
                pos += 20
                last_sync = pos
            key = struct.pack(">qq", bi + 1, bj + 1)
            val = _block_bytes(blk)
            rec = struct.pack(">ii", len(key) + len(val), len(key)) + key + val
            out.append(rec)
            pos += len(rec)
    with open(path, "wb") as fh:
        fh.write(b"".join(out))
