"""Runtime data objects (reference: runtime/instructions/cp/{ScalarObject,ListObject}.java,
runtime/controlprogram/caching/{MatrixObject,FrameObject}.java,
runtime/matrix/data/{MatrixBlock,FrameBlock}.java).

Matrices are plain 2-D ``torch.Tensor`` objects (CPU fp64 for the CP backend,
HBM-resident fp64/fp32 for the GPU backend, optionally bf16 for large read-only
inputs).  Row-partitioned matrices across ranks are
``systemml_amd.parallel.dist.DistMatrix``.  Frames and lists are small Python
containers.
"""
from __future__ import annotations

import torch

from ..parser.errors import DMLRuntimeError


class ListObject:
    __slots__ = ("data", "names")

    def __init__(self, data, names=None):
        self.data = list(data)
        self.names = list(names) if names is not None else None

    def __len__(self):
        return len(self.data)

    def get(self, key):
        if isinstance(key, str):
            if not self.names or key not in self.names:
                raise DMLRuntimeError(f"list has no element named '{key}'")
            return self.data[self.names.index(key)]
        i = int(key)
        if i < 1 or i > len(self.data):
            raise DMLRuntimeError(f"list index {i} out of bounds [1,{len(self.data)}]")
        return self.data[i - 1]

    def slice(self, lo, hi):
        names = self.names[lo - 1:hi] if self.names else None
        return ListObject(self.data[lo - 1:hi], names)

    def __repr__(self):
        return f"ListObject({len(self.data)})"


class FrameBlock:
    """Column-oriented heterogeneous frame (schema per column)."""

    def __init__(self, columns, schema=None, names=None, col_meta=None):
        # columns: list of python lists
        self.columns = [list(c) for c in columns]
        n = len(self.columns)
        self.schema = list(schema) if schema else ["STRING"] * n
        self.names = list(names) if names else [f"C{i + 1}" for i in range(n)]
        # per-column transform metadata (reference: FrameBlock.ColumnMetadata:
        # number of distinct values / bins and the missing-value replacement)
        self.col_meta = [dict(m) for m in col_meta] if col_meta else [{} for _ in range(n)]

    @property
    def shape(self):
        return (len(self.columns[0]) if self.columns else 0, len(self.columns))

    def nrow(self):
        return self.shape[0]

    def ncol(self):
        return self.shape[1]

    def row(self, i):
        return [c[i] for c in self.columns]

    def to_matrix(self, dtype=torch.float64):
        r, c = self.shape
        out = torch.empty((r, c), dtype=dtype)
        for j, col in enumerate(self.columns):
            vals = []
            for v in col:
                if v is None or v == "":
                    vals.append(float("nan"))
                else:
                    try:
                        vals.append(float(v))
                    except (TypeError, ValueError):
                        raise DMLRuntimeError(f"cannot convert frame value '{v}' to double")
            out[:, j] = torch.tensor(vals, dtype=dtype)
        return out

    @staticmethod
    def from_matrix(m):
        m = m.detach().cpu().double()
        cols = [m[:, j].tolist() for j in range(m.shape[1])]
        return FrameBlock(cols, ["DOUBLE"] * m.shape[1])

    def slice(self, rl, ru, cl, cu):
        cols = [c[rl:ru] for c in self.columns[cl:cu]]
        return FrameBlock(cols, self.schema[cl:cu], self.names[cl:cu], self.col_meta[cl:cu])

    def set_slice(self, rl, ru, cl, cu, src):
        """Left indexing: rows [rl,ru) x cols [cl,cu) <- src (frame, matrix or scalar)."""
        out = FrameBlock(self.columns, self.schema, self.names, self.col_meta)
        for j in range(cl, cu):
            col = out.columns[j]
            for i in range(rl, ru):
                if isinstance(src, FrameBlock):
                    v = src.columns[j - cl][i - rl]
                elif isinstance(src, torch.Tensor):
                    v = float(src[i - rl, j - cl])
                else:
                    v = src
                col[i] = v
        return out

    @staticmethod
    def cbind(frames):
        cols, schema, names, meta = [], [], [], []
        for f in frames:
            cols += f.columns
            schema += f.schema
            names += f.names
            meta += f.col_meta
        return FrameBlock(cols, schema, names, meta)

    def __repr__(self):
        return f"FrameBlock{self.shape}"


def is_tensor(v):
    return isinstance(v, torch.Tensor)
