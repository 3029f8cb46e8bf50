"""Compressed linear algebra (reference: runtime/compress/{CompressedMatrixBlock,ColGroupDDC*,
ColGroupOLE,ColGroupRLE,ColGroupUncompressed}.java, compress/cocode/*, compress/estim/*;
enabled by sysml.compressed.linalg = auto | true | false).

A column group G is a set of columns whose rows take few distinct value tuples; it stores a
dictionary D_G (#tuples x |G|) plus one of four row encodings, chosen per group by the
smallest in-memory size (reference: CompressedSizeEstimator + the planner's per-group choice):

* DDC  one uint8 / int16 / int32 code per row (dense dictionary coding);
* OLE  offset lists: for every non-zero tuple the rows holding it (the all-zero tuple is
       implicit), stored as one int32 row stream grouped by tuple + per-tuple counts;
* RLE  runs: (tuple, start, length) per maximal run of equal non-zero tuples, zero runs
       implicit -- sorted / clustered columns compress to a handful of runs;
* UNC  columns that do not compress, kept dense.

MI355X design: every operation is expressed as a small dictionary product plus one gather /
scatter over the encoded rows, so the row stream is read once and the work per row is a few
bytes -- the GPU form of the reference's per-group kernels:

* X %*% V   = sum_G  (D_G V_G)[codes_G]            DDC: gather by code; OLE / RLE: scatter-add
                                                    of the tuple's product row into its rows
* t(X) %*% Y = D_G^T  (rows of Y binned per tuple)  DDC: index_add by code; OLE / RLE: by the
                                                    entries' tuple ids
* sum / rowSums / colSums operate on dictionaries, tuple counts and entry lists.

Planning (cocode): per-column distinct counts on a sample, columns with few distinct values
are greedily merged while the joint tuple count stays <= 255 (uint8 codes).
"""
from __future__ import annotations

import math

import torch

MAX_TUPLES_U8 = 255
MAX_TUPLES = 32767
MIN_CELLS = 1 << 20
KINDS = ("ddc", "ole", "rle", "unc")


class ColGroup:
    """One column group.  ddc: codes (n,); ole: rows (nnz,) int32 grouped by tuple with
    tid (nnz,) tuple ids; rle: starts / lens / tid per run; unc: dict is the column block."""
    __slots__ = ("kind", "cols", "dict", "codes", "rows", "tid", "starts", "lens", "nrows")

    def __init__(self, kind, cols, dictionary, nrows, codes=None, rows=None, tid=None, starts=None, lens=None):
        self.kind = kind
        self.cols = cols              # int64 column indices
        self.dict = dictionary        # (#tuples x |cols|), compute dtype
        self.nrows = nrows
        self.codes = codes
        self.rows = rows
        self.tid = tid
        self.starts = starts
        self.lens = lens

    @property
    def uncompressed(self):
        return self.kind == "unc"

    def nbytes(self):
        b = self.dict.numel() * self.dict.element_size()
        for t in (self.codes, self.rows, self.tid, self.starts, self.lens):
            if t is not None:
                b += t.numel() * t.element_size()
        return b

    def entries(self):
        """(row indices, tuple ids) of the stored (non-implicit) cells, int64."""
        if self.kind == "ddc":
            return torch.arange(self.nrows, device=self.codes.device), self.codes.long()
        if self.kind == "ole":
            return self.rows.long(), self.tid.long()
        if self.kind == "rle":
            lens = self.lens.long()
            total = int(lens.sum().item())
            first = torch.cumsum(lens, 0) - lens
            rid = torch.repeat_interleave(torch.arange(lens.numel(), device=lens.device), lens)
            rows = self.starts.long()[rid] + (torch.arange(total, device=lens.device) - first[rid])
            return rows, self.tid.long()[rid]
        raise ValueError(self.kind)

    def counts(self):
        """Number of rows holding each dictionary tuple."""
        T = self.dict.shape[0]
        if self.kind == "ddc":
            c = torch.bincount(self.codes.long(), minlength=T)
        elif self.kind == "ole":
            c = torch.bincount(self.tid.long(), minlength=T)
        else:
            c = torch.zeros(T, dtype=torch.int64, device=self.dict.device)
            c.index_add_(0, self.tid.long(), self.lens.long())
        return c.to(self.dict.dtype)

    def with_dict(self, d):
        return ColGroup(self.kind, self.cols, d, self.nrows, self.codes, self.rows, self.tid, self.starts, self.lens)


class CompressedMatrix:
    def __init__(self, nrows, ncols, groups, dtype, device):
        self.shape = (nrows, ncols)
        self.groups = groups
        self.dtype = dtype
        self.device = device

    # ------------------------------------------------------------------ info
    def nbytes(self):
        return sum(g.nbytes() for g in self.groups)

    def ratio(self):
        return self.shape[0] * self.shape[1] * torch.empty((), dtype=self.dtype).element_size() / max(self.nbytes(), 1)

    def kinds(self):
        out = {}
        for g in self.groups:
            out[g.kind] = out.get(g.kind, 0) + 1
        return out

    def __repr__(self):
        return (f"CompressedMatrix({self.shape[0]}x{self.shape[1]}, {len(self.groups)} groups {self.kinds()}, "
                f"ratio {self.ratio():.1f})")

    # ------------------------------------------------------------------ decompress
    def decompress(self):
        out = torch.zeros(self.shape, dtype=self.dtype, device=self.device)
        for g in self.groups:
            if g.kind == "unc":
                out[:, g.cols] = g.dict
            elif g.kind == "ddc":
                out[:, g.cols] = g.dict.index_select(0, g.codes.long())
            else:
                rows, tid = g.entries()
                blk = torch.zeros((self.shape[0], g.cols.numel()), dtype=self.dtype, device=self.device)
                blk[rows] = g.dict.index_select(0, tid)
                out[:, g.cols] = blk
        return out

    # ------------------------------------------------------------------ products
    def matmul(self, V):
        """X %*% V."""
        V = V.to(self.dtype)
        out = torch.zeros((self.shape[0], V.shape[1]), dtype=self.dtype, device=self.device)
        for g in self.groups:
            Vg = V.index_select(0, g.cols)
            if g.kind == "unc":
                out += g.dict @ Vg
            elif g.kind == "ddc":
                out += (g.dict @ Vg).index_select(0, g.codes.long())
            else:
                rows, tid = g.entries()
                out.index_add_(0, rows, (g.dict @ Vg).index_select(0, tid))
        return out

    def tmatmul(self, Y):
        """t(X) %*% Y."""
        Y = Y.to(self.dtype)
        out = torch.zeros((self.shape[1], Y.shape[1]), dtype=self.dtype, device=self.device)
        for g in self.groups:
            if g.kind == "unc":
                out[g.cols] = g.dict.t() @ Y
                continue
            bins = torch.zeros((g.dict.shape[0], Y.shape[1]), dtype=self.dtype, device=self.device)
            if g.kind == "ddc":
                bins.index_add_(0, g.codes.long(), Y)
            else:
                rows, tid = g.entries()
                bins.index_add_(0, tid, Y.index_select(0, rows))
            out[g.cols] = g.dict.t() @ bins
        return out

    # ------------------------------------------------------------------ aggregates
    def colsums(self, sq=False):
        out = torch.zeros((1, self.shape[1]), dtype=self.dtype, device=self.device)
        for g in self.groups:
            d = g.dict * g.dict if sq else g.dict
            if g.kind == "unc":
                out[0, g.cols] = d.sum(0)
            else:
                out[0, g.cols] = g.counts() @ d
        return out

    def rowsums(self, sq=False):
        out = torch.zeros((self.shape[0], 1), dtype=self.dtype, device=self.device)
        for g in self.groups:
            d = g.dict * g.dict if sq else g.dict
            rs = d.sum(1, keepdim=True)
            if g.kind == "unc":
                out += rs
            elif g.kind == "ddc":
                out += rs.index_select(0, g.codes.long())
            else:
                rows, tid = g.entries()
                out.index_add_(0, rows, rs.index_select(0, tid))
        return out

    def scale(self, s):
        """X * s on the dictionaries; OLE / RLE keep their implicit zeros, so a non-finite
        factor (0 * inf = NaN) is applied to the decompressed matrix instead."""
        if not math.isfinite(s) and any(g.kind in ("ole", "rle") for g in self.groups):
            return self.decompress() * s
        gs = [g.with_dict(g.dict * s) for g in self.groups]
        return CompressedMatrix(self.shape[0], self.shape[1], gs, self.dtype, self.device)


def is_compressed(x):
    return isinstance(x, CompressedMatrix)


# ----------------------------------------------------------------------------
# planning + compression
# ----------------------------------------------------------------------------
def _encode(cols_data):
    """Distinct row tuples of an (n x k) block -> (dictionary, int64 codes)."""
    uniq, inv = torch.unique(cols_data, dim=0, return_inverse=True)
    return uniq, inv


def _code_dtype(ntup):
    return torch.uint8 if ntup <= MAX_TUPLES_U8 + 1 else torch.int16 if ntup <= MAX_TUPLES else torch.int32


def _sizes(d, codes, n):
    """Estimated bytes of the DDC / OLE / RLE encodings of one group (exact on the full data:
    the reference estimates them from a sample, CompressedSizeEstimatorSample)."""
    T, k = d.shape
    dict_b = T * k * d.element_size()
    zero = (d == 0).all(1)
    zid = int(torch.nonzero(zero)[0].item()) if bool(zero.any()) else -1
    nz = codes != zid if zid >= 0 else torch.ones_like(codes, dtype=torch.bool)
    nnz = int(nz.sum().item())
    change = torch.ones_like(codes, dtype=torch.bool)
    change[1:] = codes[1:] != codes[:-1]
    runs = int((change & nz).sum().item())
    ddc = n * torch.empty((), dtype=_code_dtype(T)).element_size() + dict_b
    ole = nnz * 4 + nnz * 2 + dict_b
    rle = runs * (4 + 4 + 2) + dict_b
    return {"ddc": ddc, "ole": ole, "rle": rle}, zid


def _make_group(kind, ci, d, codes, n, zid):
    if kind == "ddc":
        return ColGroup("ddc", ci, d.contiguous(), n, codes=codes.to(_code_dtype(d.shape[0])))
    # OLE / RLE: the all-zero tuple (if any) is implicit; renumber the remaining tuples
    keep = torch.ones(d.shape[0], dtype=torch.bool, device=d.device)
    if zid >= 0:
        keep[zid] = False
    newid = torch.cumsum(keep.long(), 0) - 1
    dd = d[keep].contiguous()
    tdt = torch.int16 if dd.shape[0] <= MAX_TUPLES else torch.int32
    nzmask = codes != zid if zid >= 0 else torch.ones_like(codes, dtype=torch.bool)
    if kind == "ole":
        rows = torch.nonzero(nzmask).flatten()
        tid = newid[codes[rows]]
        order = torch.argsort(tid, stable=True)           # offset lists grouped by tuple
        return ColGroup("ole", ci, dd, n, rows=rows[order].to(torch.int32), tid=tid[order].to(tdt))
    change = torch.ones_like(codes, dtype=torch.bool)
    change[1:] = codes[1:] != codes[:-1]
    bounds = torch.nonzero(change).flatten()
    lens = torch.diff(torch.cat([bounds, torch.tensor([n], device=codes.device)]))
    rcode = codes[bounds]
    nzr = rcode != zid if zid >= 0 else torch.ones_like(rcode, dtype=torch.bool)
    return ColGroup("rle", ci, dd, n, tid=newid[rcode[nzr]].to(tdt), starts=bounds[nzr].to(torch.int32),
                    lens=lens[nzr].to(torch.int32))


def compress(X: torch.Tensor, sample_rows=20000, force=False, kinds=None):
    """Compress a dense matrix; returns X itself when compression does not pay off.  `kinds`
    restricts the encodings the planner may choose (tests force OLE / RLE)."""
    allowed = tuple(kinds) if kinds else ("ddc", "ole", "rle")
    n, m = X.shape
    if n * m < MIN_CELLS and not force:
        return X
    Xc = X if X.dtype != torch.bfloat16 else X.float()
    # per-column distinct counts on a row sample (reference: compress/estim sampling estimators)
    if n > sample_rows:
        idx = torch.linspace(0, n - 1, sample_rows, device=X.device).long()
        S = Xc.index_select(0, idx)
    else:
        S = Xc
    distinct = [int(torch.unique(S[:, j]).numel()) for j in range(m)]
    cand = [j for j in range(m) if distinct[j] <= MAX_TUPLES_U8]
    others = [j for j in range(m) if distinct[j] > MAX_TUPLES_U8]
    # greedy co-coding: merge columns while the sample's joint tuple count stays small
    cand.sort(key=lambda j: distinct[j])
    plan = []
    cur = []
    for j in cand:
        trial = cur + [j]
        if cur and int(torch.unique(S[:, trial], dim=0).shape[0]) > MAX_TUPLES_U8:
            plan.append(cur)
            cur = [j]
        else:
            cur = trial
    if cur:
        plan.append(cur)
    groups = []
    for cols in plan:
        ci = torch.tensor(cols, dtype=torch.int64, device=X.device)
        d, codes = _encode(Xc.index_select(1, ci))
        if d.shape[0] > MAX_TUPLES:            # the sample under-estimated: keep dense
            others.extend(cols)
            continue
        sizes, zid = _sizes(d, codes, n)
        kind = min(allowed, key=lambda k_: sizes[k_])
        groups.append(_make_group(kind, ci, d, codes, n, zid))
    if others:
        ci = torch.tensor(sorted(others), dtype=torch.int64, device=X.device)
        groups.append(ColGroup("unc", ci, Xc.index_select(1, ci).contiguous(), n))
    cm = CompressedMatrix(n, m, groups, Xc.dtype, X.device)
    if not force and cm.nbytes() * 1.2 >= n * m * Xc.element_size():
        return X
    return cm
