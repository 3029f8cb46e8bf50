"""Data converters of the Python API (reference: src/main/python/systemml/converters.py).

The reference hands numpy / scipy / pandas data to the JVM as Spark MatrixBlocks; here the
runtime's matrices are torch tensors (host memory or HBM) and row-partitioned DistMatrix
blocks, so the converters map between those and numpy / scipy.sparse / pandas directly.
`convert_caffemodel` decodes the caffemodel protobuf itself (no caffe or protobuf
compiler needed) and writes each layer's weights / bias as `<layer>_weight.mtx` /
`<layer>_bias.mtx` (InnerProduct weights transposed to the nn library's D x M layout),
which `Caffe2DML.load(dir)` reads back.
"""
from __future__ import annotations

import os
import struct

import numpy as np

__all__ = ["getNumCols", "convertToMatrixBlock", "convertToNumPyArr", "convertToPandasDF", "convertToLabeledDF",
           "convertImageToNumPyArr", "getDatasetMean", "convert_caffemodel", "convert_lmdb_to_jpeg",
           "SUPPORTED_TYPES"]

SUPPORTED_TYPES = (np.ndarray,)


def getNumCols(numPyArr):
    return 1 if numPyArr.ndim == 1 else numPyArr.shape[1]


def _src(a, b):
    """Accept the reference's (sc, src) signatures and plain (src)."""
    return a if b is None else b


def convertToMatrixBlock(sc, src=None, maxSizeBlockInMB=8):
    """numpy / scipy.sparse / pandas / torch -> runtime matrix (dense tensor on the backend
    device, or CSR for sparse inputs worth keeping sparse)."""
    from .executor import convert_input
    return convert_input(_src(sc, src))


def convertToNumPyArr(sc, mb=None):
    """Runtime matrix (tensor, CSR tensor, compressed matrix, DistMatrix, Matrix handle) ->
    float64 numpy array."""
    import torch
    v = _src(sc, mb)
    if hasattr(v, "toNumPy"):
        return v.toNumPy()
    from ..ops import core as C
    if C.is_dist(v):
        v = C._dist().gather(v)
    if hasattr(v, "decompress"):
        v = v.decompress()
    if isinstance(v, torch.Tensor):
        if v.layout != torch.strided:
            v = v.to_dense()
        return v.detach().to("cpu", torch.float64).numpy()
    if hasattr(v, "toarray"):
        return np.asarray(v.toarray(), dtype=np.float64)
    return np.asarray(v, dtype=np.float64)


def convertToPandasDF(X):
    import pandas as pd
    if isinstance(X, pd.DataFrame):
        return X
    a = convertToNumPyArr(X)
    return pd.DataFrame(a, columns=[f"C{i + 1}" for i in range(a.shape[1])])


def convertToLabeledDF(sparkSession, X, y=None):
    """pandas DataFrame with a 'features' column of row vectors (and 'label' when y is given) —
    the shape of the reference's assembled Spark DataFrame."""
    import pandas as pd
    a = convertToNumPyArr(X)
    df = pd.DataFrame({"features": list(a)})
    if y is not None:
        df["label"] = np.asarray(convertToNumPyArr(y)).reshape(-1)
    return df


_DATASET_MEANS = {
    # per-channel BGR means of the ILSVRC-2012 training images used by the VGG / ResNet models
    "VGG_ILSVRC_19_2014": np.array([103.939, 116.779, 123.68]),
    "VGG_ILSVRC_16_2014": np.array([103.939, 116.779, 123.68]),
    "ResNet": np.array([103.939, 116.779, 123.68]),
}


def getDatasetMean(dataset_name):
    """Per-channel mean (BGR order) of a known pretrained model's training set."""
    for k, v in _DATASET_MEANS.items():
        if dataset_name.startswith(k) or k.startswith(dataset_name):
            return v.copy()
    raise ValueError(f"unknown dataset {dataset_name!r}; known: {sorted(_DATASET_MEANS)}")


def convertImageToNumPyArr(im, img_shape=None, add_rotated_images=False, add_mirrored_images=False,
                           color_mode="RGB", mean=None):
    """Image (PIL image or H x W [x C] array) -> rows of C*H*W values in channel-major order
    (the layout of the nn conv layers).  Optional resize to img_shape = (C, H, W), extra rows
    for the 90/180/270-degree rotations and the mirror image, 'BGR' channel order and
    per-channel mean subtraction."""
    if img_shape is not None and hasattr(im, "resize"):
        im = im.resize((img_shape[2], img_shape[1]))
    a = np.asarray(im, dtype=np.float64)
    if a.ndim == 2:
        a = a[:, :, None]
    if img_shape is not None and (a.shape[0], a.shape[1]) != (img_shape[1], img_shape[2]):
        raise ValueError(f"image is {a.shape[:2]}, expected {tuple(img_shape[1:])} (pass a PIL image to resize)")
    if color_mode == "BGR" and a.shape[2] == 3:
        a = a[:, :, ::-1]
    if mean is not None:
        a = a - np.asarray(mean, dtype=np.float64).reshape(1, 1, -1)
    imgs = [a]
    if add_rotated_images:
        imgs += [np.rot90(a, k) for k in (1, 2, 3)]
    if add_mirrored_images:
        imgs.append(a[:, ::-1, :])
    return np.vstack([np.transpose(x, (2, 0, 1)).reshape(1, -1) for x in imgs])


def convert_lmdb_to_jpeg(lmdb_img_file, output_dir):
    """Saves the images of a caffe LMDB database as output_dir/file_<i>.jpg (reference
    converters.py:111, which needs caffe, lmdb and cv2).  Here the caffe Datum records are
    decoded by this module's protobuf reader, the database is read with the `lmdb` package when
    it is installed and otherwise by a read-only reader of the LMDB file format (_lmdb_records),
    and the images are written with PIL.  Datum pixels are stored BGR (caffe); they are written
    as the colours they encode."""
    from PIL import Image
    os.makedirs(output_dir, exist_ok=True)
    i = 1
    for _, value in _lmdb_records(lmdb_img_file):
        arr, _label = decode_datum(value)
        img = np.transpose(arr, (1, 2, 0))                  # C x H x W -> H x W x C
        if img.shape[2] == 3:
            img = img[:, :, ::-1]                            # BGR -> RGB for PIL
        img = np.clip(img, 0, 255).astype(np.uint8)
        Image.fromarray(img[:, :, 0] if img.shape[2] == 1 else img).save(
            os.path.join(output_dir, "file_" + str(i) + ".jpg"), format="JPEG", quality=95)
        i += 1
    return i - 1


def decode_datum(buf):
    """caffe.proto Datum (channels 1, height 2, width 3, data 4, label 5, float_data 6, encoded 7)
    -> (C x H x W float array, label)."""
    c = h = w = 1
    data, fdata, label, encoded = None, [], 0, False
    for fno, wt, v in _fields(bytes(buf)):
        if fno == 1:
            c = v
        elif fno == 2:
            h = v
        elif fno == 3:
            w = v
        elif fno == 4:
            data = v
        elif fno == 5:
            label = v
        elif fno == 6:
            fdata.extend(np.frombuffer(v, dtype="<f4") if wt == 2 else [struct.unpack("<f", v)[0]])
        elif fno == 7:
            encoded = bool(v)
    if encoded:
        import io
        from PIL import Image
        im = np.asarray(Image.open(io.BytesIO(data)))
        im = im[:, :, None] if im.ndim == 2 else im[:, :, ::-1]      # decoded RGB -> stored BGR
        return np.transpose(im, (2, 0, 1)).astype(np.float64), label
    if data is not None and len(data):
        arr = np.frombuffer(data, dtype=np.uint8).astype(np.float64)
    else:
        arr = np.asarray(fdata, dtype=np.float64)
    return arr.reshape(c, h, w), label


def _lmdb_records(path):
    try:
        import lmdb
    except ImportError:
        yield from read_lmdb(path)
        return
    env = lmdb.open(path, readonly=True, lock=False)
    with env.begin() as txn:
        for k, v in txn.cursor():
            yield bytes(k), bytes(v)


# LMDB on-disk format (read-only, 64-bit): meta pages 0 / 1 (the newer transaction wins), a
# B+tree of branch / leaf pages from the main database's root, values larger than a node in
# overflow pages.
_P_BRANCH, _P_LEAF, _P_OVERFLOW, _P_LEAF2 = 0x01, 0x02, 0x04, 0x20
_F_BIGDATA, _F_SUBDATA, _F_DUPDATA = 0x01, 0x02, 0x04
_MDB_MAGIC = 0xBEEFC0DE


def read_lmdb(path):
    """Key / value pairs of an LMDB database (a directory with data.mdb, or the file), in key
    order, without the lmdb package."""
    import mmap
    fn = os.path.join(path, "data.mdb") if os.path.isdir(path) else path
    with open(fn, "rb") as f:
        mm = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
    try:
        # page 0: header (16 B) + MDB_meta {magic, version, address, mapsize, dbs[2] (48 B each),
        # last_pg, txnid}; the page size is the free DB's md_pad of meta 0
        magic, _version = struct.unpack_from("<II", mm, 16)
        if magic != _MDB_MAGIC:
            raise ValueError(f"{fn}: not an LMDB file (magic {magic:#x})")
        psize = struct.unpack_from("<I", mm, 16 + 24)[0]          # dbs[0].md_pad = page size

        def meta(pg):
            o = pg * psize + 16
            main = o + 24 + 48                                   # mm_dbs[1]
            root = struct.unpack_from("<Q", mm, main + 40)[0]
            entries = struct.unpack_from("<Q", mm, main + 32)[0]
            txnid = struct.unpack_from("<Q", mm, o + 24 + 96 + 8)[0]
            flags = struct.unpack_from("<H", mm, main + 4)[0]
            return txnid, root, entries, flags
        m = max(meta(0), meta(1))
        _, root, entries, dbflags = m
        if entries == 0 or root == 0xFFFFFFFFFFFFFFFF:
            return
        if dbflags & 0x04:                                       # MDB_DUPSORT
            raise ValueError("LMDB databases with duplicate keys are not supported")

        def walk(pg):
            o = pg * psize
            flags = struct.unpack_from("<H", mm, o + 10)[0]
            lower = struct.unpack_from("<H", mm, o + 12)[0]
            n = (lower - 16) // 2
            ptrs = struct.unpack_from(f"<{n}H", mm, o + 16)
            for p in ptrs:
                no = o + p
                lo, hi, nflags, ksize = struct.unpack_from("<HHHH", mm, no)
                key = bytes(mm[no + 8:no + 8 + ksize])
                if flags & _P_BRANCH:
                    child = lo | (hi << 16) | (nflags << 32)
                    yield from walk(child)
                elif flags & _P_LEAF:
                    dsize = lo | (hi << 16)
                    d = no + 8 + ksize
                    if nflags & _F_BIGDATA:
                        opg = struct.unpack_from("<Q", mm, d)[0]
                        start = opg * psize + 16
                        yield key, bytes(mm[start:start + dsize])
                    else:
                        yield key, bytes(mm[d:d + dsize])
        yield from walk(root)
    finally:
        mm.close()


# ----------------------------------------------------------------------------
# caffemodel (protobuf wire format) decoding
# ----------------------------------------------------------------------------
def _varint(buf, i):
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def _fields(buf):
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fno, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v, i = buf[i:i + 8], i + 8
        elif wt == 2:
            ln, i = _varint(buf, i)
            v, i = buf[i:i + ln], i + ln
        elif wt == 5:
            v, i = buf[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield fno, wt, v


def _packed_ints(v):
    out, i = [], 0
    while i < len(v):
        x, i = _varint(v, i)
        out.append(x)
    return out


def _blob(buf):
    """BlobProto -> numpy array (shape from BlobShape or legacy num/channels/height/width)."""
    data, ddata, shape, legacy = [], [], None, {}
    for fno, wt, v in _fields(buf):
        if fno == 5:        # data (float)
            data.append(np.frombuffer(bytes(v), dtype="<f4") if wt == 2 else np.frombuffer(bytes(v), "<f4"))
        elif fno == 8:      # double_data
            ddata.append(np.frombuffer(bytes(v), dtype="<f8"))
        elif fno == 7:      # BlobShape
            dims = []
            for f2, w2, v2 in _fields(v):
                if f2 == 1:
                    dims += _packed_ints(v2) if w2 == 2 else [v2]
            shape = dims
        elif fno in (1, 2, 3, 4) and wt == 0:
            legacy[fno] = v
    arr = np.concatenate(ddata) if ddata else (np.concatenate(data) if data else np.zeros(0, np.float32))
    if shape is None:
        shape = [legacy.get(k, 1) for k in (1, 2, 3, 4)]      # num, channels, height, width
        while len(shape) > 1 and shape[0] == 1:
            shape = shape[1:]
    if int(np.prod(shape)) == arr.size and shape:
        arr = arr.reshape(shape)
    return arr.astype(np.float64)


_V1_TYPES = {4: "Convolution", 14: "InnerProduct", 39: "Deconvolution"}


def read_caffemodel(path):
    """[(layer name, layer type, [blobs])] of a binary caffemodel (NetParameter)."""
    buf = memoryview(open(path, "rb").read())
    layers = []
    for fno, wt, v in _fields(buf):
        if fno not in (100, 2) or wt != 2:
            continue
        name, typ, blobs = "", "", []
        for f2, w2, v2 in _fields(v):
            if fno == 100:              # LayerParameter: name 1, type 2, blobs 7
                if f2 == 1:
                    name = bytes(v2).decode()
                elif f2 == 2:
                    typ = bytes(v2).decode()
                elif f2 == 7:
                    blobs.append(_blob(v2))
            else:                       # V1LayerParameter: name 4, type 5 (enum), blobs 6
                if f2 == 4:
                    name = bytes(v2).decode()
                elif f2 == 5 and w2 == 0:
                    typ = _V1_TYPES.get(v2, str(v2))
                elif f2 == 6:
                    blobs.append(_blob(v2))
        if blobs:
            layers.append((name, typ, blobs))
    return layers


def convert_caffemodel(sc, deploy_file, caffemodel_file, output_dir, format="binary", is_caffe_installed=False):
    """Save every parameterised layer's weights / bias as <layer>_weight.mtx / <layer>_bias.mtx
    (weights reshaped to F x (C*H*W); InnerProduct weights transposed to D x M)."""
    import torch
    from ..io.writers import write_matrix
    os.makedirs(output_dir, exist_ok=True)
    written = []
    for name, typ, blobs in read_caffemodel(caffemodel_file):
        if len(blobs) > 2:
            raise ValueError(f"layer {name}: unsupported number of parameters {len(blobs)}")
        transpose = typ == "InnerProduct"
        for blob, suffix in zip(blobs, ("_weight.mtx", "_bias.mtx")):
            w = blob.reshape(blob.shape[0], -1) if blob.ndim else blob.reshape(1, 1)
            if transpose:
                w = w.T
            path = os.path.join(output_dir, name + suffix)
            write_matrix(torch.from_numpy(np.ascontiguousarray(w)), path, format)
            written.append(path)
    return written
