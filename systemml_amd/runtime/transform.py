"""Frame transform: transformencode / transformapply / transformdecode / transformcolmap /
transformmeta (reference: runtime/transform/encode/*.java, decode/*.java,
meta/TfMetaUtils.java; DML semantics in parser/ParameterizedBuiltinFunctionExpression.java).

A transform spec (lenient JSON, bare identifiers allowed) names columns by 1-based id
(`"ids": true`) or by frame column name and selects per-column methods:

    recode     categorical token -> 1..#distinct (first-appearance order)
    dummycode  recode + one-hot expansion into #distinct columns
    bin        equi-width binning [{"id"|"name", "method": "equi-width", "numbins": n}]
    impute     [{"id"|"name", "method": "global_mean"|"global_mode"|"constant", "value": v}]
    omit       drop rows with a missing value in any of these columns

The metadata frame M has the input's column layout: recode columns hold
"token·code" entries, bin columns "lower·upper" bin bounds, and each column's
`col_meta` carries the number of distinct values / bins and the missing-value
replacement, exactly what `transformapply` / `transformdecode` need to reproduce the
encoding on new data.

Unlike the reference's encoder chain, dummy-coding is applied LAST, so binning,
imputation and omission always index the un-expanded column layout; binning bounds
are computed during encode (the reference's CP encoder only supports bins supplied
through metadata).
"""
from __future__ import annotations

import json
import math
import os
import re

import numpy as np
import torch

from ..parser.errors import DMLRuntimeError
from .data import FrameBlock

SEP = "·"          # reference: Lop.DATATYPE_PREFIX
_BARE = re.compile(r'(?<![\w"])([A-Za-z_][\w.\-]*)(?![\w"])')


# ---------------------------------------------------------------------------
# spec parsing (reference: TfMetaUtils.parseJsonIDList / parseJsonObjectIDList)
# ---------------------------------------------------------------------------
def parse_spec(spec) -> dict:
    if isinstance(spec, dict):
        return spec
    s = str(spec).strip()
    try:
        return json.loads(s)
    except ValueError:
        pass
    # quote bare identifiers outside of strings (keeps true/false/null literals)
    out, i = [], 0
    for m in re.finditer(r'"(?:[^"\\]|\\.)*"', s):
        out.append(_quote_bare(s[i:m.start()]))
        out.append(m.group(0))
        i = m.end()
    out.append(_quote_bare(s[i:]))
    try:
        return json.loads("".join(out))
    except ValueError as e:
        raise DMLRuntimeError(f"invalid transform specification: {spec!r} ({e})")


def _quote_bare(seg):
    return _BARE.sub(lambda m: m.group(1) if m.group(1) in ("true", "false", "null") else f'"{m.group(1)}"', seg)


class Spec:
    def __init__(self, spec, colnames, ncol):
        js = parse_spec(spec)
        self.js = js
        self.ids = bool(js.get("ids", False))
        self.colnames = list(colnames) if colnames else [f"C{i + 1}" for i in range(ncol)]
        self.ncol = ncol
        self.recode = self._ids("recode")
        self.dummy = self._ids("dummycode")
        self.recode = sorted(set(self.recode) | set(self.dummy))
        self.omit = self._ids("omit")
        self.bin = {c: o for c, o in self._objs("bin")}
        self.impute = {c: o for c, o in self._objs("impute")}
        self.passthrough = [c for c in range(1, ncol + 1) if c not in self.recode and c not in self.bin]

    def _col(self, key, ids):
        if ids:
            c = int(key)
        else:
            c = self.colnames.index(key) + 1 if key in self.colnames else 0
        if c <= 0 or c > max(self.ncol, 1) and self.ncol:
            raise DMLRuntimeError(f"Specified column '{key}' does not exist.")
        return c

    def _ids(self, group):
        v = self.js.get(group)
        if v is None:
            return []
        ids = self.ids
        if isinstance(v, dict):          # {"attributes": [...]} (file-based spec)
            v, ids = v.get("attributes", []), True
        if not isinstance(v, list):
            v = [v]
        return sorted(self._col(x if not isinstance(x, dict) else x.get("id", x.get("name")), ids) for x in v)

    def _objs(self, group):
        v = self.js.get(group)
        if not isinstance(v, list):
            return []
        out = []
        for o in v:
            if isinstance(o, dict):
                key = o.get("id") if self.ids else o.get("name", o.get("id"))
                out.append((self._col(key, self.ids or "name" not in o), o))
            else:
                out.append((self._col(o, self.ids), {}))
        return sorted(out, key=lambda t: t[0])


# ---------------------------------------------------------------------------
# helpers
# ---------------------------------------------------------------------------
def _missing(v):
    return v is None or (isinstance(v, str) and v == "") or (isinstance(v, float) and math.isnan(v))


def _token(v):
    """Canonical token string of a frame cell (reference: Object.toString())."""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float) and v.is_integer() and abs(v) < 1e15:
        return str(v)
    return str(v)


def _num(v):
    if _missing(v):
        return float("nan")
    if isinstance(v, bool):
        return 1.0 if v else 0.0
    if isinstance(v, (int, float)):
        return float(v)
    t = str(v).strip()
    if t.upper() == "TRUE":
        return 1.0
    if t.upper() == "FALSE":
        return 0.0
    try:
        return float(t)
    except ValueError:
        raise DMLRuntimeError(f"transform: cannot convert '{v}' to double (column not recoded?)")


def split_entry(e):
    e = str(e)
    pos = e.rfind(SEP)
    if pos < 0:
        raise DMLRuntimeError(f"malformed transform meta entry '{e}'")
    return e[:pos], e[pos + 1:]


def _recode_map(meta: FrameBlock, col0: int) -> dict:
    n = int(meta.col_meta[col0].get("ndistinct", 0)) if meta.col_meta[col0] else 0
    out = {}
    for v in meta.columns[col0][: n or None]:
        if v is None or v == "":
            continue
        tok, code = split_entry(v)
        out[tok] = int(float(code))
    return out


def _bin_bounds(meta: FrameBlock, col0: int):
    n = int(meta.col_meta[col0].get("ndistinct", 0))
    lo, hi = [], []
    for v in meta.columns[col0][:n]:
        a, b = split_entry(v)
        lo.append(float(a))
        hi.append(float(b))
    return np.array(lo), np.array(hi)


def _frame_of(target):
    if isinstance(target, FrameBlock):
        return target
    if isinstance(target, torch.Tensor):
        return FrameBlock.from_matrix(target)
    raise DMLRuntimeError("transform requires a frame target")


# ---------------------------------------------------------------------------
# build (encode) metadata
# ---------------------------------------------------------------------------
def build_meta(fr: FrameBlock, sp: Spec) -> FrameBlock:
    ncol = fr.ncol()
    cols = [[] for _ in range(ncol)]
    cmeta = [{} for _ in range(ncol)]
    for c in sp.recode:
        seen = {}
        for v in fr.columns[c - 1]:
            if _missing(v):
                continue
            t = _token(v)
            if t not in seen:
                seen[t] = len(seen) + 1
        cols[c - 1] = [f"{t}{SEP}{k}" for t, k in seen.items()]
        cmeta[c - 1]["ndistinct"] = len(seen)
    for c, o in sp.bin.items():
        nb = int(o.get("numbins", o.get("num_bins", 10)))
        method = str(o.get("method", "equi-width")).lower()
        x = np.array([_num(v) for v in fr.columns[c - 1]], dtype=np.float64)
        x = x[~np.isnan(x)]
        if x.size == 0:
            raise DMLRuntimeError(f"transform bin: column {c} has no values")
        if method == "equi-height":
            edges = np.quantile(x, np.linspace(0, 1, nb + 1))
        else:
            mn, mx = float(x.min()), float(x.max())
            w = (mx - mn) / nb
            edges = np.array([mn + i * w for i in range(nb + 1)])
            edges[-1] = mx
        cols[c - 1] = [f"{float(edges[i])!r}{SEP}{float(edges[i + 1])!r}" for i in range(nb)]
        cmeta[c - 1]["ndistinct"] = nb
    for c, o in sp.impute.items():
        method = str(o.get("method", "global_mean")).lower()
        col = fr.columns[c - 1]
        if method == "global_mean":
            x = np.array([_num(v) for v in col], dtype=np.float64)
            x = x[~np.isnan(x)]
            rep = repr(float(x.mean())) if x.size else "0.0"
        elif method == "global_mode":
            hist = {}
            for v in col:
                if not _missing(v):
                    t = _token(v)
                    hist[t] = hist.get(t, 0) + 1
            rep = max(hist.items(), key=lambda kv: kv[1])[0] if hist else ""
        elif method == "constant":
            rep = str(o.get("value", ""))
        else:
            raise DMLRuntimeError(f"unknown impute method '{method}'")
        cmeta[c - 1]["mv"] = rep
    rows = max((len(c) for c in cols), default=0)
    cols = [c + [None] * (rows - len(c)) for c in cols]
    return FrameBlock(cols, ["STRING"] * ncol, list(fr.names), cmeta)


# ---------------------------------------------------------------------------
# apply
# ---------------------------------------------------------------------------
def apply_meta(fr: FrameBlock, sp: Spec, meta: FrameBlock) -> torch.Tensor:
    nrow, ncol = fr.shape
    out = np.full((nrow, ncol), np.nan, dtype=np.float64)
    for c in sp.recode:
        m = _recode_map(meta, c - 1)
        out[:, c - 1] = [m.get(_token(v), np.nan) if not _missing(v) else np.nan for v in fr.columns[c - 1]]
    for c in sp.passthrough:
        out[:, c - 1] = [_num(v) for v in fr.columns[c - 1]]
    for c in sp.bin:
        lo, hi = _bin_bounds(meta, c - 1)
        x = np.array([_num(v) for v in fr.columns[c - 1]], dtype=np.float64)
        ids = np.searchsorted(hi, x, side="left") + 1.0
        ids = np.minimum(ids, len(hi))
        ids[np.isnan(x)] = np.nan
        out[:, c - 1] = ids
    for c in sp.impute:
        rep = meta.col_meta[c - 1].get("mv") if meta.col_meta[c - 1] else None
        if rep is None:
            continue
        if c in sp.recode:
            val = _recode_map(meta, c - 1).get(rep, np.nan)
        elif c in sp.bin:
            lo, hi = _bin_bounds(meta, c - 1)
            val = float(min(np.searchsorted(hi, float(rep), side="left") + 1, len(hi)))
        else:
            val = float(rep)
        col = out[:, c - 1]
        col[np.isnan(col)] = val
    if sp.omit:
        keep = ~np.isnan(out[:, [c - 1 for c in sp.omit]]).any(axis=1)
        out = out[keep]
    if sp.dummy:
        out = _dummycode(out, sp.dummy, [_ndistinct(meta, c) for c in sp.dummy])
    return torch.from_numpy(np.ascontiguousarray(out))


def _ndistinct(meta, c):
    cm = meta.col_meta[c - 1] if c - 1 < len(meta.col_meta) else {}
    n = cm.get("ndistinct")
    if n is None:
        n = sum(1 for v in meta.columns[c - 1] if v not in (None, ""))
    return int(n)


def _dummycode(X, dcols, dsizes):
    nrow, ncol = X.shape
    width = ncol + sum(d - 1 for d in dsizes)
    out = np.zeros((nrow, width), dtype=np.float64)
    pos = 0
    di = dict(zip(dcols, dsizes))
    for c in range(1, ncol + 1):
        if c in di:
            codes = X[:, c - 1]
            ok = ~np.isnan(codes)
            rows = np.nonzero(ok)[0]
            out[rows, pos + codes[ok].astype(np.int64) - 1] = 1.0
            pos += di[c]
        else:
            out[:, pos] = X[:, c - 1]
            pos += 1
    return out


def col_mapping(meta: FrameBlock, sp: Spec) -> torch.Tensor:
    """K x 3 matrix [column id, first output column, last output column]
    (reference: EncoderDummycode.getColMapping)."""
    ncol = meta.ncol()
    out = np.zeros((ncol, 3))
    pos = 1
    for c in range(1, ncol + 1):
        start = pos
        pos += _ndistinct(meta, c) if c in sp.dummy else 1
        out[c - 1] = (c, start, pos - 1)
    return torch.from_numpy(out)


# ---------------------------------------------------------------------------
# decode (reference: decode/DecoderDummycode, DecoderRecode, DecoderPassThrough)
# ---------------------------------------------------------------------------
def decode_matrix(X: torch.Tensor, sp: Spec, meta: FrameBlock) -> FrameBlock:
    X = X.detach().cpu().double().numpy()
    nrow = X.shape[0]
    ncol = meta.ncol() if sp.dummy else min(meta.ncol(), X.shape[1])
    codes = np.full((nrow, ncol), np.nan)
    if sp.dummy:
        pos = 0
        for c in range(1, ncol + 1):
            if c in sp.dummy:
                d = _ndistinct(meta, c)
                blk = X[:, pos:pos + d]
                nz = blk != 0
                codes[:, c - 1] = np.where(nz.any(axis=1), np.argmax(nz, axis=1) + 1, np.nan)
                pos += d
            else:
                codes[:, c - 1] = X[:, pos]
                pos += 1
    else:
        codes[:, :ncol] = X[:, :ncol]
    cols, schema = [], []
    for c in range(1, ncol + 1):
        v = codes[:, c - 1]
        if c in sp.recode:
            inv = {k: t for t, k in _recode_map(meta, c - 1).items()}
            cols.append([inv.get(int(x)) if not math.isnan(x) else None for x in v])
            schema.append("STRING")
        else:
            cols.append([float(x) for x in v])
            schema.append("DOUBLE")
    names = meta.names[:ncol] if meta.names else None
    return FrameBlock(cols, schema, names)


# ---------------------------------------------------------------------------
# transformmeta: read on-disk transform metadata (reference: TfMetaUtils.readTransformMetaDataFromFile)
# ---------------------------------------------------------------------------
def read_meta_dir(spec, path, sep=","):
    with open(os.path.join(path, "column.names")) as f:
        colnames = [c.strip().strip('"') for c in f.read().strip().split(sep)]
    sp = Spec(spec, colnames, len(colnames))
    ncol = len(colnames)
    cols = [[] for _ in range(ncol)]
    cmeta = [{} for _ in range(ncol)]
    for c in sp.recode:
        name = colnames[c - 1]
        fn = os.path.join(path, "Recode", name + ".map")
        if not os.path.exists(fn):
            raise DMLRuntimeError(f"Recode map for column '{name}' (id={c}) not existing.")
        with open(fn) as f:
            for line in f:
                line = line.rstrip("\n")
                if not line:
                    continue
                iq = line.rfind('"')
                if iq >= 0:
                    tok = line[:iq + 1].strip('"')
                    rest = line[iq + 2:]
                else:
                    tok, rest = line.split(sep, 1)
                code = rest.split(sep)[0]
                cols[c - 1].append(f"{tok}{SEP}{code}")
        cmeta[c - 1]["ndistinct"] = len(cols[c - 1])
    for c in sp.bin:
        name = colnames[c - 1]
        fn = os.path.join(path, "Bin", name + ".bin")
        if not os.path.exists(fn):
            raise DMLRuntimeError(f"Binning map for column '{name}' (id={c}) not existing.")
        with open(fn) as f:
            fields = f.read().strip().split(sep)
        mn, w, nb = float(fields[1]), float(fields[3]), int(fields[4])
        cols[c - 1] = [f"{mn + i * w!r}{SEP}{mn + (i + 1) * w!r}" for i in range(nb)]
        cmeta[c - 1]["ndistinct"] = nb
    for c, name in enumerate(colnames, 1):
        fn = os.path.join(path, "Impute", name + ".impute")
        if os.path.exists(fn):
            with open(fn) as f:
                cmeta[c - 1]["mv"] = f.read().strip().split(sep)[1]
    rows = max((len(c) for c in cols), default=0)
    cols = [c + [None] * (rows - len(c)) for c in cols]
    return FrameBlock(cols, ["STRING"] * ncol, colnames, cmeta)


def write_meta_dir(meta: FrameBlock, spec, path, sep=","):
    """Inverse of read_meta_dir: the on-disk transform metadata layout of the reference's
    legacy transform (column.names, Recode/<col>.map|.ndistinct, Bin/<col>.bin,
    Impute/<col>.impute)."""
    sp = Spec(spec, meta.names, meta.ncol())
    os.makedirs(path, exist_ok=True)
    with open(os.path.join(path, "column.names"), "w") as f:
        f.write(sep.join(meta.names) + "\n")
    for c in sp.recode:
        name = meta.names[c - 1]
        d = os.path.join(path, "Recode")
        os.makedirs(d, exist_ok=True)
        m = _recode_map(meta, c - 1)
        with open(os.path.join(d, name + ".map"), "w") as f:
            for tok, code in sorted(m.items(), key=lambda kv: kv[1]):
                f.write(f'"{tok}"{sep}{code}\n')
        with open(os.path.join(d, name + ".ndistinct"), "w") as f:
            f.write(f"{len(m)}\n")
    for c in sp.bin:
        name = meta.names[c - 1]
        d = os.path.join(path, "Bin")
        os.makedirs(d, exist_ok=True)
        lo, hi = _bin_bounds(meta, c - 1)
        w = (hi[-1] - lo[0]) / len(lo)
        with open(os.path.join(d, name + ".bin"), "w") as f:
            f.write(sep.join(str(x) for x in (c, repr(float(lo[0])), repr(float(hi[-1])), repr(float(w)), len(lo))))
    for c in sp.impute:
        rep = meta.col_meta[c - 1].get("mv") if meta.col_meta[c - 1] else None
        if rep is None:
            continue
        d = os.path.join(path, "Impute")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, meta.names[c - 1] + ".impute"), "w") as f:
            f.write(f"{c}{sep}{rep}")
    with open(os.path.join(path, "spec.json"), "w") as f:
        json.dump(sp.js, f)


def legacy_transform(ctx, target, transformPath=None, spec=None, applyTransformPath=None, outputNames=None, **kw):
    """Legacy `transform()` builtin (reference: ParameterizedBuiltin transform with
    transformPath / applyTransformPath): encode and write the metadata directory, or apply a
    previously written one."""
    fr = _frame_of(target)
    from ..ops.backend import place
    if applyTransformPath is not None:
        path = applyTransformPath
        with open(os.path.join(path, "spec.json")) as f:
            js = json.load(f)
        meta = _meta_for(read_meta_dir(js, path), fr)
        return place(apply_meta(fr, Spec(js, fr.names, fr.ncol()), meta))
    sp = Spec(spec, fr.names, fr.ncol())
    meta = build_meta(fr, sp)
    if transformPath is not None:
        write_meta_dir(meta, sp.js, transformPath)
    if outputNames is not None:
        with open(str(outputNames), "w") as f:
            f.write(",".join(fr.names) + "\n")
    return place(apply_meta(fr, sp, meta))


# ---------------------------------------------------------------------------
# builtin entry points
# ---------------------------------------------------------------------------
def _meta_for(meta, fr):
    """Align a metadata frame to the target's columns by name (reference:
    EncoderFactory 'robustness for superset of cols')."""
    if meta.names and fr.names and list(meta.names) != list(fr.names) and \
            all(n in meta.names for n in fr.names):
        idx = [meta.names.index(n) for n in fr.names]
        return FrameBlock([meta.columns[i] for i in idx], [meta.schema[i] for i in idx],
                          [meta.names[i] for i in idx], [meta.col_meta[i] for i in idx])
    return meta


def encode(ctx, target, spec):
    fr = _frame_of(target)
    sp = Spec(spec, fr.names, fr.ncol())
    meta = build_meta(fr, sp)
    X = apply_meta(fr, sp, meta)
    from ..ops.backend import place
    return (place(X), meta)


def apply(ctx, target, spec, meta):
    fr = _frame_of(target)
    meta = _meta_for(meta, fr)
    sp = Spec(spec, fr.names, fr.ncol())
    from ..ops.backend import place
    return place(apply_meta(fr, sp, meta))


def decode(ctx, target, spec, meta):
    if isinstance(target, FrameBlock):
        target = target.to_matrix()
    sp = Spec(spec, meta.names, meta.ncol())
    return decode_matrix(target, sp, meta)


def colmap(ctx, target, spec):
    sp = Spec(spec, target.names, target.ncol())
    from ..ops.backend import place
    return place(col_mapping(target, sp))


def read_meta(ctx, spec, meta, sep=","):
    return read_meta_dir(spec, meta, sep)
