"""Compressed linear algebra (reference: runtime/compress/{CompressedMatrixBlock,ColGroupDDC*,
ColGroupOLE,ColGroupRLE,ColGroupUncompressed}.java, compress/cocode/*, compress/estim/*;
enabled by sysml.compressed.linalg = auto | true | false).

MI355X design: only dictionary coding (DDC) — the GPU-friendly encoding.  A column group
G is a set of columns whose rows take few distinct value tuples; it is stored as a
dictionary D_G (#tuples x |G|) plus one uint8 / int16 code per row.  Run-length and
offset-list encodings (RLE / OLE) exist in the reference to skip zeros on a CPU; on the
GPU their irregular access loses to a byte-per-row code stream, so very sparse inputs use
the CSR path (ops/sparse.py) instead.

* X %*% V   = sum_G  (D_G V_G)[codes_G]                  (small GEMM + gather per group)
* t(X) %*% Y = for each G: D_G^T  (scatter-add of Y's rows into #tuples bins)
* sum / rowSums / colSums operate on dictionaries and code histograms
* columns that do not compress stay in one dense "uncompressed" group

Planning (cocode): per-column distinct counts on a sample, columns with few distinct
values are greedily merged while the joint tuple count stays <= 255 (uint8 codes).
"""
from __future__ import annotations

import torch

MAX_TUPLES_U8 = 255
MAX_TUPLES = 32767
MIN_CELLS = 1 << 20


class ColGroup:
    __slots__ = ("cols", "dict", "codes")

    def __init__(self, cols, dictionary, codes):
        self.cols = cols              # int64 column indices
        self.dict = dictionary        # (#tuples x |cols|), compute dtype
        self.codes = codes            # (n,) uint8 / int16 / int32 codes; None = uncompressed (dict is the data)

    @property
    def uncompressed(self):
        return self.codes is None

    def nbytes(self):
        b = self.dict.numel() * self.dict.element_size()
        if self.codes is not None:
            b += self.codes.numel() * self.codes.element_size()
        return b


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

    def __repr__(self):
        return f"CompressedMatrix({self.shape[0]}x{self.shape[1]}, {len(self.groups)} groups, ratio {self.ratio():.1f})"

    # ------------------------------------------------------------------ decompress
    def decompress(self):
        out = torch.empty(self.shape, dtype=self.dtype, device=self.device)
        for g in self.groups:
            if g.uncompressed:
                out[:, g.cols] = g.dict
            else:
                out[:, g.cols] = g.dict.index_select(0, g.codes.long())
        return out

    # ------------------------------------------------------------------ products
    def matmul(self, V):
        """X %*% V."""
        V = V.to(self.dtype)
        out = torch.zeros((self.shape[0], V.shape[1]), dtype=self.dtype, device=self.device)
        for g in self.groups:
            Vg = V.index_select(0, g.cols)
            if g.uncompressed:
                out += g.dict @ Vg
            else:
                out += (g.dict @ Vg).index_select(0, g.codes.long())
        return out

    def tmatmul(self, Y):
        """t(X) %*% Y."""
        Y = Y.to(self.dtype)
        out = torch.zeros((self.shape[1], Y.shape[1]), dtype=self.dtype, device=self.device)
        for g in self.groups:
            if g.uncompressed:
                out[g.cols] = g.dict.t() @ Y
            else:
                bins = torch.zeros((g.dict.shape[0], Y.shape[1]), dtype=self.dtype, device=self.device)
                bins.index_add_(0, g.codes.long(), Y)
                out[g.cols] = g.dict.t() @ bins
        return out

    # ------------------------------------------------------------------ aggregates
    def _counts(self, g):
        return torch.bincount(g.codes.long(), minlength=g.dict.shape[0]).to(self.dtype)

    def colsums(self, sq=False):
        out = torch.zeros((1, self.shape[1]), dtype=self.dtype, device=self.device)
        for g in self.groups:
            d = g.dict * g.dict if sq else g.dict
            if g.uncompressed:
                out[0, g.cols] = d.sum(0)
            else:
                out[0, g.cols] = self._counts(g) @ d
        return out

    def rowsums(self, sq=False):
        out = torch.zeros((self.shape[0], 1), dtype=self.dtype, device=self.device)
        for g in self.groups:
            d = g.dict * g.dict if sq else g.dict
            if g.uncompressed:
                out += d.sum(1, keepdim=True)
            else:
                out += d.sum(1, keepdim=True).index_select(0, g.codes.long())
        return out

    def scale(self, s):
        gs = [ColGroup(g.cols, g.dict * s, g.codes) for g in self.groups]
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


def compress(X: torch.Tensor, sample_rows=20000, force=False):
    """Compress a dense matrix; returns X itself when compression does not pay off."""
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
        groups.append(ColGroup(ci, d.contiguous(), codes.to(_code_dtype(d.shape[0]))))
    if others:
        ci = torch.tensor(sorted(others), dtype=torch.int64, device=X.device)
        groups.append(ColGroup(ci, Xc.index_select(1, ci).contiguous(), None))
    cm = CompressedMatrix(n, m, groups, Xc.dtype, X.device)
    if not force and cm.nbytes() * 1.2 >= n * m * Xc.element_size():
        return X
    return cm
