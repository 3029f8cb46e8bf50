"""Random sampling constructors for the lazy matrix DSL (reference:
src/main/python/systemml/random/sampling.py — `normal`, `uniform`, `poisson`).

    from systemml_amd import random as sml_random
    m = sml_random.normal(loc=3, scale=2, size=(3, 3))     # lazy defmatrix.matrix
    m.toNumPy()

Each call emits one DML data-generation expression (run by the backend's generator:
in HBM on a GPU run), so samples compose with the rest of a lazy DAG.  With sparsity < 1
the sampled zero pattern is kept: `loc + scale * z` is applied to the non-zeros only.
"""
from __future__ import annotations

from .defmatrix import matrix

__all__ = ["normal", "uniform", "poisson"]


def _size(size):
    if not isinstance(size, (tuple, list)) or len(size) != 2:
        raise TypeError("Incorrect type for size. Expected tuple of length 2")
    return int(size[0]), int(size[1])


def _rand(r, c, extra, sparsity, seed):
    return f"rand(rows={r}, cols={c}, {extra}sparsity={float(sparsity)!r}, seed={int(seed)})"


def normal(loc=0.0, scale=1.0, size=(1, 1), sparsity=1.0, seed=-1):
    """Samples of N(loc, scale^2)."""
    r, c = _size(size)
    z = matrix._op(_rand(r, c, 'pdf="normal", ', sparsity, seed), shape=(r, c))
    shift, mul = float(loc), float(scale)
    if float(sparsity) >= 1.0:
        return matrix._op(f"{shift!r} + {mul!r} * {{0}}", z, shape=(r, c))
    return matrix._op(f"({{0}} != 0) * ({shift!r} + {mul!r} * {{0}})", z, shape=(r, c))


def uniform(low=0.0, high=1.0, size=(1, 1), sparsity=1.0, seed=-1):
    """Samples of U(low, high)."""
    r, c = _size(size)
    return matrix._op(_rand(r, c, f'min={float(low)!r}, max={float(high)!r}, pdf="uniform", ', sparsity, seed),
                      shape=(r, c))


def poisson(lam=1.0, size=(1, 1), sparsity=1.0, seed=-1):
    """Samples of Poisson(lam)."""
    r, c = _size(size)
    if float(lam) <= 0:
        raise ValueError("lam must be > 0")
    return matrix._op(_rand(r, c, f'pdf="poisson", lambda={float(lam)!r}, ', sparsity, seed), shape=(r, c))
