"""Weighted interQuartileMean (reference MatrixBlock.interQuartileMean, weights as
frequencies) and the caffe LMDB image export (reference python/systemml/converters.py
convert_lmdb_to_jpeg): Datum protobuf decoding and a read-only LMDB reader.  No lmdb / caffe
package is installed here, so the LMDB test writes a database in the on-disk format itself
(meta pages, a branch page over two leaf pages, an overflow page): parity unpinned against the
lmdb library."""
import math
import os
import struct

import numpy as np
import pytest

from systemml_amd.api import converters as CV
from systemml_amd.api import executor as EX
from systemml_amd.conf import DMLConfig


def _iqm_ref(vals, w):
    o = np.argsort(vals, kind="stable")
    v, ww = vals[o], w[o]
    sum_wt = ww.sum()
    q25d, q75d = 0.25 * sum_wt, 0.75 * sum_wt
    q25i, q75i = math.ceil(q25d), math.ceil(q75d)
    psum, i = 0.0, -1
    while psum < q25i and i < len(v):
        i += 1
        psum += ww[i]
    q25p, q25v, s = psum - q25d, v[i], 0.0
    while psum < q75i and i < len(v):
        i += 1
        psum += ww[i]
        s += v[i] * ww[i]
    return (s + q25p * q25v - (psum - q75d) * v[i]) / (sum_wt * 0.5)


@pytest.mark.parametrize("n", [4, 7, 10, 33, 100])
def test_weighted_interquartile_mean(n):
    rng = np.random.default_rng(n)
    x = rng.random((n, 1))
    w = rng.integers(1, 6, (n, 1)).astype(float)
    out = []
    EX.run("print(interQuartileMean(X, W))", inputs={"X": x, "W": w}, config=DMLConfig(gpu=False), out=out.append)
    assert float(out[0]) == pytest.approx(_iqm_ref(x.ravel(), w.ravel()), rel=1e-12)


def test_unit_weights_match_unweighted():
    x = np.arange(1.0, 13.0).reshape(-1, 1)
    a, b = [], []
    EX.run("print(interQuartileMean(X))", inputs={"X": x}, config=DMLConfig(gpu=False), out=a.append)
    EX.run("print(interQuartileMean(X, W))", inputs={"X": x, "W": np.ones_like(x)}, config=DMLConfig(gpu=False),
           out=b.append)
    assert float(a[0]) == pytest.approx(float(b[0]), rel=1e-12) == pytest.approx(6.5)


# ----------------------------------------------------------------------------- caffe Datum / LMDB
def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            return bytes(out)


def _datum(c, h, w, pixels, label):
    f = lambda no, wt: _varint((no << 3) | wt)  # noqa: E731
    return (f(1, 0) + _varint(c) + f(2, 0) + _varint(h) + f(3, 0) + _varint(w) +
            f(4, 2) + _varint(len(pixels)) + bytes(pixels) + f(5, 0) + _varint(label))


def _write_lmdb(path, items, psize=4096):
    """A minimal LMDB file: pages 0 / 1 meta, 2 / 3 leaf pages, 4 branch (root), overflow pages
    after, for the given sorted (key, value) pairs (values > 1 KiB go to overflow pages)."""
    pages = {}
    nxt = [5]

    def leaf(pg, kvs):
        buf = bytearray(psize)
        struct.pack_into("<QHHHH", buf, 0, pg, 0, 0x02, 16 + 2 * len(kvs), 0)
        top = psize
        ptrs = []
        for k, v in kvs:
            if len(v) > 1024:
                opg = nxt[0]
                npages = (16 + len(v) + psize - 1) // psize
                nxt[0] += npages
                ob = bytearray(npages * psize)
                struct.pack_into("<QHHI", ob, 0, opg, 0, 0x04, npages)
                ob[16:16 + len(v)] = v
                pages[opg] = bytes(ob)
                node = struct.pack("<HHHH", len(v) & 0xFFFF, len(v) >> 16, 0x01, len(k)) + k + struct.pack("<Q", opg)
            else:
                node = struct.pack("<HHHH", len(v) & 0xFFFF, len(v) >> 16, 0, len(k)) + k + v
            node += b"\0" * (len(node) & 1)
            top -= len(node)
            buf[top:top + len(node)] = node
            ptrs.append(top)
        struct.pack_into(f"<{len(ptrs)}H", buf, 16, *ptrs)
        struct.pack_into("<H", buf, 14, top)
        pages[pg] = bytes(buf)

    half = len(items) // 2
    leaf(2, items[:half])
    leaf(3, items[half:])
    br = bytearray(psize)
    nodes = [(b"", 2), (items[half][0], 3)]
    struct.pack_into("<QHHHH", br, 0, 4, 0, 0x01, 16 + 2 * len(nodes), 0)
    top, ptrs = psize, []
    for k, pg in nodes:
        node = struct.pack("<HHHH", pg & 0xFFFF, (pg >> 16) & 0xFFFF, pg >> 32, len(k)) + k
        node += b"\0" * (len(node) & 1)
        top -= len(node)
        br[top:top + len(node)] = node
        ptrs.append(top)
    struct.pack_into(f"<{len(ptrs)}H", br, 16, *ptrs)
    pages[4] = bytes(br)
    for pg, txn in ((0, 1), (1, 2)):
        m = bytearray(psize)
        struct.pack_into("<QHHHH", m, 0, pg, 0, 0x08, 0, 0)
        o = 16
        struct.pack_into("<IIQQ", m, o, 0xBEEFC0DE, 1, 0, 1 << 20)
        struct.pack_into("<IHHQQQQQ", m, o + 24, psize, 0, 0, 0, 0, 0, 0, 0xFFFFFFFFFFFFFFFF)   # free DB
        root = 4 if txn == 2 else 0xFFFFFFFFFFFFFFFF                                            # meta 1 is newer
        struct.pack_into("<IHHQQQQQ", m, o + 72, 0, 0, 2, 1, 2, 0, len(items), root)
        struct.pack_into("<QQ", m, o + 120, nxt[0] - 1, txn)
        pages[pg] = bytes(m)
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "data.mdb"), "wb") as f:
        for pg in range(nxt[0]):
            f.write(pages.get(pg, b"\0" * psize))


def test_datum_decode():
    px = np.arange(2 * 3 * 4, dtype=np.uint8)
    arr, label = CV.decode_datum(_datum(2, 3, 4, px, 7))
    assert label == 7 and arr.shape == (2, 3, 4)
    np.testing.assert_array_equal(arr.ravel(), px)


def test_lmdb_reader_and_jpeg_export(tmp_path):
    rng = np.random.default_rng(1)
    imgs = [rng.integers(0, 256, (3, 24, 20), dtype=np.uint8) for _ in range(5)]
    imgs[2] = np.zeros((3, 24, 20), dtype=np.uint8)     # a flat image (exact after JPEG)
    items = [(f"{i:08d}".encode(), _datum(3, 24, 20, im.ravel(), i)) for i, im in enumerate(imgs)]
    db = str(tmp_path / "db")
    _write_lmdb(db, items)
    got = list(CV.read_lmdb(db))
    assert [k for k, _ in got] == [k for k, _ in items]
    assert all(a == b for (_, a), (_, b) in zip(got, items))
    out = str(tmp_path / "jpg")
    assert CV.convert_lmdb_to_jpeg(db, out) == 5
    from PIL import Image
    assert sorted(os.listdir(out)) == [f"file_{i}.jpg" for i in range(1, 6)]
    im = np.asarray(Image.open(os.path.join(out, "file_3.jpg")))
    assert im.shape == (24, 20, 3) and im.max() <= 1
