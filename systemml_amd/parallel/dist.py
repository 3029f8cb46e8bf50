"""Row-partitioned distributed matrices over one-process-per-GPU ranks.

This replaces the reference's Spark/MR backends (runtime/instructions/spark/*,
runtime/controlprogram/context/SparkExecutionContext.java) with an SPMD design
for a single 8×MI355X node:

* every rank runs the same compiled program (runtime/program.py);
* matrices with >= `dist_min_rows` rows are split into contiguous row blocks,
  one per rank, resident in that rank's HBM (`DistMatrix`); all other values
  are replicated;
* operators map to the reference's distributed physical operators:
    - X %*% v (v replicated)           → local matmult, stays row-partitioned   (mapmm)
    - t(X) %*% Y, Y co-partitioned     → local matmult + all-reduce             (cpmm / zipmm)
    - t(X) %*% X                       → local tsmm + all-reduce                (tsmm)
    - mmchain / row-fused H·v          → local fused kernel + all-reduce        (mapmmchain)
    - full / column aggregates         → local aggregate + all-reduce
    - row aggregates, cellwise ops     → purely local
  so each iteration of a CG / trust-region solver moves only D×K-sized
  vectors over xGMI (RCCL all-reduce); X never leaves its GPU.
* anything else falls back to an all-gather (correct, slower), counted in
  `fallback_gathers` so tests can assert the hot path stays distributed.

Collectives use torch.distributed (backend "nccl" = RCCL on ROCm; "gloo" for
CPU tests).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as tdist

from ..parser.errors import DMLRuntimeError
from ..runtime import scalars as S

_CTX = None
stats = {"allreduce": 0, "allgather": 0, "alltoall": 0, "broadcast": 0, "fallback_gathers": 0}
fallback_sites = {}          # op label -> count (why a row-partitioned operand was gathered)


def reset_stats():
    for k in stats:
        stats[k] = 0
    fallback_sites.clear()


class DistContext:
    def __init__(self, rank, world, device, group=None):
        self.rank = rank
        self.world = world
        self.device = device
        self.group = group
        self.min_rows = 1            # results with >= min_rows rows stay row-partitioned (set per run)

    def partition(self, n):
        base, rem = divmod(n, self.world)
        start = self.rank * base + min(self.rank, rem)
        size = base + (1 if self.rank < rem else 0)
        return start, start + size

    def all_partitions(self, n):
        out = []
        base, rem = divmod(n, self.world)
        s = 0
        for r in range(self.world):
            sz = base + (1 if r < rem else 0)
            out.append((s, s + sz))
            s += sz
        return out

    # -- collectives --------------------------------------------------------
    def allreduce_(self, t, op="sum"):
        from ..runtime import graphloop as _GL
        seg = _GL.capturing()
        if seg is not None:
            # a run-ahead loop iteration being captured (runtime/graphloop.py): the graph is cut
            # here and the replay issues this all-reduce on the same buffer between segments
            seg.collective(self, t, op)
            return t
        stats["allreduce"] += 1
        rop = {"sum": tdist.ReduceOp.SUM, "max": tdist.ReduceOp.MAX, "min": tdist.ReduceOp.MIN,
               "prod": tdist.ReduceOp.PRODUCT}[op]
        tdist.all_reduce(t, op=rop, group=self.group)
        return t

    def allreduce_scalar(self, v, op="sum", dtype=None, device=None):
        dev = device if device is not None else self._coll_device()
        t = torch.tensor([v], dtype=dtype or torch.float64, device=dev)
        self.allreduce_(t, op)
        return float(t.item())

    def allreduce_dev(self, v, op="sum"):
        """All-reduce of a scalar partial that stays on the device when the collective does
        (RCCL): the result is a device scalar (runtime.scalars.DevScalar), so the host reads
        it only where it must branch or print -- no host round trip per reduction.  With a
        host collective (gloo) a float."""
        dev = self._coll_device()
        if dev.type != "cuda":
            return self.allreduce_scalar(float(v.reshape(-1)[0].item()) if isinstance(v, torch.Tensor) else
                                         float(v), op)
        if isinstance(v, torch.Tensor):
            t = v.reshape(1).to(device=dev, dtype=torch.float64)
            if t.data_ptr() == v.data_ptr():
                t = t.clone()
        else:
            from ..runtime.scalars import DevScalar
            if isinstance(v, DevScalar):
                t = v.t.reshape(1).to(device=dev, dtype=torch.float64).clone()
            else:
                t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        self.allreduce_(t, op)
        from ..runtime.scalars import DevScalar
        return DevScalar(t.reshape(()))

    def _coll_device(self):
        return self.device if tdist.get_backend(self.group) != "gloo" else torch.device("cpu")

    def barrier(self):
        tdist.barrier(group=self.group)


def get_context():
    return _CTX


def init(backend=None, device=None):
    """Initialise SPMD execution from torchrun-style env vars (RANK/WORLD_SIZE/MASTER_*)."""
    global _CTX
    world = int(os.environ.get("WORLD_SIZE", "1"))
    force = os.environ.get("SYSML_DIST_FORCE") == "1"
    if world <= 1 and not force:
        _CTX = None
        return None
    rank = int(os.environ.get("RANK", "0"))
    if world <= 1:
        # SYSML_DIST_FORCE=1: a one-rank process group, so the SPMD code path (row-partitioned
        # operands, packed / device-scalar all-reduces, run-ahead under RCCL) runs on one GPU
        # and can be compared with the single-process plan
        world, rank = 1, 0
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            import socket
            sk = socket.socket()
            sk.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(sk.getsockname()[1])
            sk.close()
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        os.environ.setdefault("LOCAL_RANK", "0")
    # SYSML_DIST_BACKEND=gloo with SYSML_DIST_DEVICE=cuda rehearses the GPU SPMD path with
    # several ranks on ONE GPU (RCCL refuses two ranks per device): same partitioning,
    # kernels and collectives, host-staged transport
    backend = backend or os.environ.get("SYSML_DIST_BACKEND") or None
    if device is None and os.environ.get("SYSML_DIST_DEVICE") == "cuda" and torch.cuda.is_available():
        device = torch.device("cuda", torch.cuda.current_device())
    if not tdist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        kw = {}
        if backend == "nccl":
            local = int(os.environ.get("LOCAL_RANK", rank))
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        tdist.init_process_group(backend=backend, **kw)
    if device is None:
        if torch.cuda.is_available() and tdist.get_backend() == "nccl":
            device = torch.device("cuda", torch.cuda.current_device())
        else:
            device = torch.device("cpu")
    _CTX = DistContext(rank, world, device)
    return _CTX


def shutdown():
    global _CTX
    _CTX = None
    if tdist.is_initialized():
        tdist.destroy_process_group()


# ----------------------------------------------------------------------------
class DistMatrix:
    """Row block [start, end) of an (nrows x ncols) matrix held by this rank."""
    __slots__ = ("local", "nrows", "ncols", "start", "ctx")

    def __init__(self, local, nrows, ncols, start, ctx):
        self.local = local
        self.nrows = nrows
        self.ncols = ncols
        self.start = start
        self.ctx = ctx

    @property
    def shape(self):
        return (self.nrows, self.ncols)

    def like(self, local):
        return DistMatrix(local, self.nrows, local.shape[1], self.start, self.ctx)

    def __repr__(self):
        return f"DistMatrix({self.nrows}x{self.ncols}, rank {self.ctx.rank} rows [{self.start},{self.start + self.local.shape[0]}))"


def _is_d(x):
    return isinstance(x, DistMatrix)


def _C():
    from ..ops import core
    return core


def gather(x: DistMatrix):
    """All-gather the row blocks into a replicated tensor."""
    if not _is_d(x):
        return x
    ctx = x.ctx
    return _allgather_rows(ctx, x.local, [e - s for s, e in ctx.all_partitions(x.nrows)], x.ncols)


def _fallback(x, site=None):
    if not _is_d(x):
        return x
    stats["fallback_gathers"] += 1
    if site is None:
        import sys
        f = sys._getframe(1)
        site = f.f_code.co_name
    fallback_sites[site] = fallback_sites.get(site, 0) + 1
    return gather(x)


def local_rows(ctx, t):
    """Slice this rank's rows out of a replicated full tensor."""
    s, e = ctx.partition(t.shape[0])
    return DistMatrix(t[s:e].contiguous(), t.shape[0], t.shape[1], s, ctx)


def local_block(ctx, loc, nrows, ncols):
    """Wrap this rank's rows [partition(nrows)) of a matrix (host or device tensor) as a
    DistMatrix.  The dense/CSR decision is taken on the GLOBAL non-zero count (one scalar
    all-reduce) so all ranks agree on the format, as MatrixBlock.evalSparseFormatInMemory
    would for the whole matrix."""
    from ..ops.backend import place, maybe_bf16
    from ..ops import sparse as SP
    s, e = ctx.partition(nrows)
    if loc.shape[0] != e - s:
        raise DMLRuntimeError(f"local block has {loc.shape[0]} rows, expected {e - s}")
    if SP.is_sparse(loc):
        loc = loc.to(ctx.device)
    elif loc.dtype == torch.bfloat16:
        loc = loc.to(ctx.device).contiguous()
    else:
        nz = float(torch.count_nonzero(loc).item()) if loc.numel() else 0.0
        gnz = ctx.allreduce_scalar(nz, "sum")
        if SP.want_sparse(nrows, ncols, gnz):
            loc = place(loc.contiguous()).to_sparse_csr()
        else:
            loc = maybe_bf16(place(loc.contiguous())).contiguous()
    return DistMatrix(loc, nrows, ncols, s, ctx)


def scatter_rows_from_global(ctx, t):
    """Every rank holds the full matrix `t` (e.g. a driver-side input): keep this rank's rows."""
    from ..ops import sparse as SP
    s, e = ctx.partition(t.shape[0])
    loc = SP.csr_rows(t, s, e) if SP.is_sparse(t) else t[s:e]
    return local_block(ctx, loc, t.shape[0], t.shape[1])


def scatter_rows(exec_ctx, t):
    return scatter_rows_from_global(exec_ctx.dist, t)


def from_local(ctx, local, nrows):
    s, e = ctx.partition(nrows)
    if local.shape[0] != e - s:
        raise DMLRuntimeError(f"local block has {local.shape[0]} rows, expected {e - s}")
    return DistMatrix(local, nrows, local.shape[1], s, ctx)


# ----------------------------------------------------------------------------
# datagen
# ----------------------------------------------------------------------------
def rand(exec_ctx, r, c, lo, hi, sp, pdf, seed, lam):
    from ..runtime.builtins import _rand_local
    ctx = exec_ctx.dist
    s, e = ctx.partition(r)
    # seed already agreed across ranks (builtins._seed); chunked generation makes the
    # local block equal rows [s, e) of the single-process rand
    loc = _rand_local(e - s, c, lo, hi, sp, pdf, seed, lam, device=ctx.device, row_offset=s, total_rows=r)
    return DistMatrix(loc, r, c, s, ctx)


def full(exec_ctx, r, c, v):
    from ..ops.backend import backend
    ctx = exec_ctx.dist
    s, e = ctx.partition(r)
    return DistMatrix(torch.full((e - s, c), v, dtype=backend.dtype, device=ctx.device), r, c, s, ctx)


def seq(exec_ctx, a, inc, n):
    from ..ops.backend import backend
    ctx = exec_ctx.dist
    s, e = ctx.partition(n)
    loc = a + inc * torch.arange(s, e, dtype=torch.float64, device=ctx.device)
    return DistMatrix(loc.to(backend.dtype).reshape(-1, 1), n, 1, s, ctx)


# ----------------------------------------------------------------------------
# operators
# ----------------------------------------------------------------------------
def _dense(t):
    from ..ops import sparse as SP
    return SP.densify(t) if isinstance(t, torch.Tensor) and SP.is_sparse(t) else t


def _align(x, like: DistMatrix):
    """Bring operand x to like's row partition (returns local tensor or scalar)."""
    if _is_d(x):
        if x.nrows != like.nrows:
            raise DMLRuntimeError(f"dimension mismatch: {x.nrows} vs {like.nrows} rows")
        return x.local
    if isinstance(x, torch.Tensor):
        if x.shape[0] == like.nrows and like.nrows != 1:
            e = like.start + like.local.shape[0]
            return x[like.start:e]
        return x
    return x


def _bcast(x, site):
    """Replicate a row-partitioned operand an operator needs whole -- the broadcast side
    of the reference's mapmm / mapmmchain (e.g. a weight vector whose length crossed the
    distribution threshold).  Counted apart from fallbacks."""
    if not _is_d(x):
        return x
    stats["broadcast"] = stats.get("broadcast", 0) + 1
    return _dense(gather(x))


# -- point-to-point exchange -------------------------------------------------
def _exchange(ctx, sends, recv_shapes, dtype, device):
    """sends[q]: tensor for rank q (None / 0 rows: nothing); recv_shapes[q]: shape of the
    block rank q sends here.  One grouped isend/irecv batch (RCCL groups it into a single
    launch over xGMI).  Returns the received blocks (own block passed through)."""
    out = [None] * ctx.world
    ops = []
    for q in range(ctx.world):
        if q == ctx.rank:
            out[q] = sends[q] if sends[q] is not None else torch.empty(recv_shapes[q], dtype=dtype, device=device)
            continue
        if sends[q] is not None and sends[q].numel() > 0:
            ops.append(tdist.P2POp(tdist.isend, sends[q].contiguous(), q, group=ctx.group))
        if recv_shapes[q][0] * recv_shapes[q][1] > 0:
            out[q] = torch.empty(recv_shapes[q], dtype=dtype, device=device)
            ops.append(tdist.P2POp(tdist.irecv, out[q], q, group=ctx.group))
        else:
            out[q] = torch.empty(recv_shapes[q], dtype=dtype, device=device)
    if ops:
        stats["alltoall"] += 1
        for w in tdist.batch_isend_irecv(ops):
            w.wait()
    return out


def _isect(a, b):
    s, e = max(a[0], b[0]), min(a[1], b[1])
    return (s, e) if s < e else (s, s)


def _repartition(ctx, loc, src, dst, ncols):
    """Move rows between layouts: this rank holds global rows src[rank] (as `loc`), and
    afterwards holds dst[rank]; src/dst are per-rank [s, e) ranges ascending by rank."""
    me = ctx.rank
    loc = _dense(loc)
    sends = []
    for q in range(ctx.world):
        s, e = _isect(src[me], dst[q])
        sends.append(loc[s - src[me][0]:e - src[me][0]])
    shapes = []
    for q in range(ctx.world):
        s, e = _isect(src[q], dst[me])
        shapes.append((e - s, ncols))
    parts = _exchange(ctx, sends, shapes, loc.dtype, loc.device)
    parts = [p for p in parts if p.shape[0] > 0]
    if not parts:
        return torch.empty((0, ncols), dtype=loc.dtype, device=loc.device)
    return torch.cat(parts, 0) if len(parts) > 1 else parts[0].contiguous()


def _allgather_rows(ctx, loc, sizes, ncols):
    """All-gather variable-size row blocks (sizes known on every rank) into one tensor:
    blocks are padded to the largest so one fixed-size collective moves them."""
    loc = _dense(loc).contiguous()
    stats["allgather"] += 1
    maxr = max(sizes) if sizes else 0
    if maxr == 0:
        return torch.empty((0, ncols), dtype=loc.dtype, device=loc.device)
    pad = loc if loc.shape[0] == maxr else \
        torch.cat([loc, torch.zeros((maxr - loc.shape[0], ncols), dtype=loc.dtype, device=loc.device)], 0)
    if tdist.get_backend(ctx.group) == "gloo" or loc.device.type == "cpu":
        bufs = [torch.empty((maxr, ncols), dtype=loc.dtype, device=loc.device) for _ in sizes]
        tdist.all_gather(bufs, pad, group=ctx.group)
        return torch.cat([b[:n] for b, n in zip(bufs, sizes)], 0)
    out = torch.empty((ctx.world * maxr, ncols), dtype=loc.dtype, device=loc.device)
    tdist.all_gather_into_tensor(out, pad, group=ctx.group)
    return torch.cat([out[r * maxr: r * maxr + n] for r, n in enumerate(sizes)], 0)


def _keep_dist(ctx, n):
    return n >= getattr(ctx, "min_rows", 1)


def _result(ctx, dst_rows, loc, ncols):
    """Wrap a result of `dst_rows` rows: row-partitioned when large enough, else replicated
    (small result: variable all-gather)."""
    if _keep_dist(ctx, dst_rows):
        s, _ = ctx.partition(dst_rows)
        return DistMatrix(loc, dst_rows, ncols, s, ctx)
    return loc


# ----------------------------------------------------------------------------
def binary(op, a, b):
    C = _C()
    if _is_d(a):
        ref = a
    elif _is_d(b):
        ref = b
    else:
        return C.binary(op, a, b)
    if _is_d(a) and _is_d(b) and a.nrows != b.nrows:
        raise DMLRuntimeError(f"Block sizes are not matched for binary cell operations: {a.shape} vs {b.shape}")
    la = _align(a, ref)
    lb = _align(b, ref)
    r = C.binary(op, la, lb)
    return DistMatrix(r, ref.nrows, r.shape[1], ref.start, ref.ctx)


_SCAN = {"cumsum": (torch.add, 0.0), "cumprod": (torch.mul, 1.0),
         "cummin": (torch.minimum, float("inf")), "cummax": (torch.maximum, -float("inf"))}


def cumagg(op, x):
    """Column-wise cumulative aggregate of a row-partitioned matrix: local scan, then the
    ranks' block totals are all-gathered (world x ncols) and each rank folds in the
    exclusive prefix of the ranks before it (reference: the Spark CumulativeAggregate/
    CumulativeOffset instruction pair, as one collective)."""
    C = _C()
    ctx = x.ctx
    comb, ident = _SCAN[op]
    loc = C.unary(op, _dense(x.local)) if x.local.shape[0] else _dense(x.local)
    last = loc[-1:].to(torch.float64) if loc.shape[0] else \
        torch.full((1, x.ncols), ident, dtype=torch.float64, device=loc.device)
    tot = _allgather_rows(ctx, last.to(ctx.device) if tdist.get_backend(ctx.group) != "gloo" else last.cpu(),
                          [1] * ctx.world, x.ncols)
    if ctx.rank > 0 and loc.shape[0]:
        carry = tot[0:1]
        for r in range(1, ctx.rank):
            carry = comb(carry, tot[r:r + 1])
        loc = comb(loc, carry.to(device=loc.device, dtype=loc.dtype))
    return x.like(loc)


def unary(op, x):
    C = _C()
    if op in ("nrow", "ncol", "length"):
        return {"nrow": x.nrows, "ncol": x.ncols, "length": x.nrows * x.ncols}[op]
    if op in ("cast_scalar", "cast_double", "cast_int", "cast_bool", "cast_frame"):
        return C.unary(op, gather(x))
    if op == "cast_matrix":
        return x
    if op in _SCAN:
        return cumagg(op, x)
    r = C.unary(op, _dense(x.local))
    return x.like(r)


def agg(o, d, x):
    C = _C()
    ctx = x.ctx
    loc = x.local
    if d == "row":
        return x.like(C.agg(o, "row", loc))
    if o in ("sum", "sumsq", "min", "max", "prod"):
        if loc.shape[0] == 0:
            init = {"sum": 0.0, "sumsq": 0.0, "min": float("inf"), "max": -float("inf"), "prod": 1.0}[o]
            part = init if d == "all" else torch.full((1, x.ncols), init, dtype=torch.float64, device=ctx.device)
        else:
            part = C.agg(o, d, loc)
        rop = {"sum": "sum", "sumsq": "sum", "min": "min", "max": "max", "prod": "prod"}[o]
        if d == "all":
            return ctx.allreduce_dev(part, rop)
        t = part.contiguous().clone()
        ctx.allreduce_(t, rop)
        return t
    if o == "mean":
        n = x.nrows * x.ncols if d == "all" else x.nrows
        s = agg("sum", d, x)
        return s / n
    if o in ("var", "sd"):
        n = x.nrows * x.ncols if d == "all" else x.nrows
        s = agg("sum", d, x)
        ss = agg("sumsq", d, x)
        if d == "all":
            v = (ss - s * s / n) / (n - 1) if n > 1 else 0.0
            return v ** 0.5 if o == "sd" else v
        v = (ss - s * s / n) / (n - 1)
        return torch.sqrt(v) if o == "sd" else v
    if o in ("rowIndexMax", "rowIndexMin"):
        return x.like(C.agg(o, d, _dense(loc)))
    if o == "trace":
        # diagonal cells (i, i) with i in this rank's row range
        s0 = x.start
        n = min(loc.shape[0], max(0, x.ncols - s0))
        part = float(torch.diagonal(_dense(loc)[:n, s0:s0 + n]).double().sum().item()) if n > 0 else 0.0
        return ctx.allreduce_scalar(part, "sum", device=loc.device if loc.is_cuda else None)
    return C.agg(o, d, _fallback(x, "agg:" + o))


def tak(a, b):
    C = _C()
    if _is_d(a) and _is_d(b):
        part = C.tak(a.local, b.local) if a.local.shape[0] else 0.0
        return a.ctx.allreduce_scalar(part, "sum", device=a.local.device if a.local.is_cuda else None)
    return agg("sum", "all", binary("*", a, b))


def _ring_mm(ctx, A_loc, B, b_parts, transB=False):
    """A_loc (n_r x M) %*% B where B's rows (or, transB, B^T's columns) are row-partitioned
    as b_parts: the B blocks travel around the ring (rank r -> r+1) while each rank
    multiplies the block it holds -- the receive of the next block overlaps the current
    product, and no rank ever holds more than two blocks of B (reference analogue: the
    rmm / cpmm shuffles, without materialising the replicated operand).  transB: result
    column block q = A_loc @ B_q^T."""
    C = _C()
    me, P = ctx.rank, ctx.world
    blk = _dense(B.local).contiguous()
    cols = B.ncols
    if transB:
        out = torch.empty((A_loc.shape[0], B.nrows), dtype=torch.promote_types(A_loc.dtype, blk.dtype),
                          device=A_loc.device)
    else:
        out = None
    owner = me
    for step in range(P):
        nxt_owner = (owner - 1) % P
        pending = None
        if step < P - 1:
            s, e = b_parts[nxt_owner]
            nxt = torch.empty((e - s, cols), dtype=blk.dtype, device=blk.device)
            ops = []
            if blk.numel():
                ops.append(tdist.P2POp(tdist.isend, blk, (me + 1) % P, group=ctx.group))
            if nxt.numel():
                ops.append(tdist.P2POp(tdist.irecv, nxt, (me - 1) % P, group=ctx.group))
            pending = (nxt, tdist.batch_isend_irecv(ops) if ops else [])
            stats["alltoall"] += 1
        s, e = b_parts[owner]
        if e > s:
            if transB:
                out[:, s:e] = C.mm(A_loc, C.transpose(blk)) if A_loc.shape[0] else out[:, s:e]
            else:
                part = C.mm(A_loc[:, s:e], blk) if A_loc.shape[0] else \
                    torch.zeros((0, cols), dtype=blk.dtype, device=blk.device)
                out = part if out is None else out + part
        if pending is not None:
            for w in pending[1]:
                w.wait()
            blk = pending[0]
        owner = nxt_owner
    if out is None:
        out = torch.zeros((A_loc.shape[0], cols), dtype=blk.dtype, device=blk.device)
    return out


def mm(a, b, transA=False):
    C = _C()
    if transA:
        if _is_d(a):
            if _is_d(b) or (isinstance(b, torch.Tensor) and b.shape[0] == a.nrows):
                lb = _align(b, a)
            else:
                raise DMLRuntimeError("t(X) %*% Y: row dimension mismatch")
            r = C.mm(a.local, lb, True).contiguous()
            a.ctx.allreduce_(r, "sum")
            return r
        # t(A) %*% B, A replicated and B row-partitioned: t(A[rows, ]) %*% B_local, all-reduce
        if b.nrows != a.shape[0]:
            raise DMLRuntimeError("t(X) %*% Y: row dimension mismatch")
        e = b.start + b.local.shape[0]
        r = C.mm(a[b.start:e], b.local, True).contiguous()
        b.ctx.allreduce_(r, "sum")
        return r
    if _is_d(a) and not _is_d(b):
        r = C.mm(a.local, b)
        return DistMatrix(r, a.nrows, r.shape[1], a.start, a.ctx)
    if _is_d(a) and _is_d(b):
        if a.ncols != b.nrows:
            raise DMLRuntimeError(f"Matrix multiplication dimension mismatch: {a.shape} %*% {b.shape}")
        r = _ring_mm(a.ctx, _dense(a.local), b, a.ctx.all_partitions(b.nrows))
        return DistMatrix(r, a.nrows, r.shape[1], a.start, a.ctx)
    # replicated A %*% distributed B: A[:, local rows] @ B_local, all-reduce
    if _is_d(b):
        e = b.start + b.local.shape[0]
        r = C.mm(C.rix(a, None, None, b.start + 1, e, False) if b.local.shape[0] else a[:, :0], b.local).contiguous()
        b.ctx.allreduce_(r, "sum")
        return r
    return C.mm(a, b, transA)


def tsmm(x: DistMatrix, left=True):
    C = _C()
    if left:
        r = C.tsmm(x.local, True).contiguous()
        x.ctx.allreduce_(r, "sum")
        return r
    # X %*% t(X): result rows follow X, column block q from X_q travelling the ring
    r = _ring_mm(x.ctx, _dense(x.local), x, x.ctx.all_partitions(x.nrows), transB=True)
    return DistMatrix(r, x.nrows, x.nrows, x.start, x.ctx)


def mmchain(ctype, X, v, w=None):
    C = _C()
    if not _is_d(X):
        return C.mmchain(ctype, X, _bcast(v, "mmchain"), _bcast(w, "mmchain") if w is not None else None)
    v = _bcast(v, "mmchain")
    lw = _align(w, X) if w is not None else None
    r = C.mmchain(ctype, X.local, v, lw).contiguous()
    X.ctx.allreduce_(r, "sum")
    return r


def smgrad(X, V, Y, cu=None):
    """Row-partitioned fused softmax gradient: each rank streams its rows of X once, U stays
    row-distributed, the D x K gradient partials are all-reduced."""
    C = _C()
    if not _is_d(X):
        return C.smgrad(X, _bcast(V, "smgrad"), _fallback(Y, "smgrad:Y"), cu)
    V = _bcast(V, "smgrad")
    u, g = C.smgrad(X.local, V, _align(Y, X), cu)
    g = g.contiguous()
    X.ctx.allreduce_(g, "sum")
    return DistMatrix(u, X.nrows, u.shape[1], X.start, X.ctx), g


def smobj(X, V, Y, kc):
    """Row-partitioned fused softmax objective / gradient: each rank streams its rows once,
    P stays row-distributed; the D x K gradient and the two objective sums travel in ONE
    all-reduce (packed), and the sums are read by the host once, after it."""
    C = _C()
    if not _is_d(X):
        return C.smobj(X, _bcast(V, "smobj"), _fallback(Y, "smobj:Y"), kc)
    V = _bcast(V, "smobj")
    p, g, s1, s2 = C.smobj(X.local, V, _align(Y, X), kc, defer=True)
    ctx = X.ctx
    dev = ctx._coll_device()
    parts = [g.reshape(-1).to(device=dev, dtype=torch.float64)]
    for s in (s1, s2):
        parts.append(s.reshape(1).to(device=dev, dtype=torch.float64) if isinstance(s, torch.Tensor)
                     else torch.tensor([float(s)], dtype=torch.float64, device=dev))
    buf = torch.cat(parts)
    ctx.allreduce_(buf, "sum")
    n = g.numel()
    g = buf[:n].reshape(g.shape).to(device=g.device, dtype=g.dtype)
    s = buf[n:].tolist()
    return DistMatrix(p, X.nrows, p.shape[1], X.start, X.ctx), g, s[0], s[1]


def transpose(x):
    """t(X) of a row-partitioned X (N x M).  Large M: the result is row-partitioned too and
    built with one all-to-all (rank r sends the transposed column block q of its rows to
    rank q).  Small M: the M x N result is replicated (variable all-gather of the local
    transposes along columns)."""
    C = _C()
    ctx = x.ctx
    loc = _dense(x.local)
    N, M = x.nrows, x.ncols
    src = ctx.all_partitions(N)
    if _keep_dist(ctx, M):
        dst = ctx.all_partitions(M)
        sends = [loc[:, s:e].t().contiguous() for s, e in dst]
        me = ctx.rank
        shapes = [(dst[me][1] - dst[me][0], e - s) for s, e in src]
        parts = _exchange(ctx, sends, shapes, loc.dtype, loc.device)
        r = torch.cat(parts, 1).contiguous()
        return DistMatrix(r, M, N, dst[me][0], ctx)
    # the rows of X all-gathered, then transposed: the result is replicated by construction
    return C.transpose(_allgather_rows(ctx, loc, [e - s for s, e in src], M))


def _bnd(v):
    if v is None:
        return None
    if isinstance(v, torch.Tensor):
        v = v.reshape(-1)[0].item()
    return int(S.as_double(v))


def rix(x: DistMatrix, rl, ru, cl, cu):
    """X[r0:r1, c0:c1] of a row-partitioned X: full row range -> local column slice; a row
    range -> this rank's intersection, then repartitioned (large result) or all-gathered
    (small result, e.g. one row inside a loop) -- never the whole of X."""
    ctx = x.ctx
    r0 = _bnd(rl) or 1
    r1 = _bnd(ru) or x.nrows
    c0 = _bnd(cl) or 1
    c1 = _bnd(cu) or x.ncols
    if r0 < 1 or r1 > x.nrows or r0 > r1 or c0 < 1 or c1 > x.ncols or c0 > c1:
        raise DMLRuntimeError(f"Invalid values for matrix indexing: [{r0}:{r1},{c0}:{c1}] "
                              f"must be within matrix dimensions [{x.nrows},{x.ncols}]")
    loc = x.local
    if c0 != 1 or c1 != x.ncols:
        loc = _dense(loc)[:, c0 - 1:c1]
    if r0 == 1 and r1 == x.nrows:
        return x.like(loc)
    n = r1 - r0 + 1
    nc = c1 - c0 + 1
    src = [(s - (r0 - 1), e - (r0 - 1)) for s, e in ctx.all_partitions(x.nrows)]
    win = [_isect(p, (0, n)) for p in src]
    me = ctx.rank
    mine = _dense(loc)[win[me][0] - src[me][0]:win[me][1] - src[me][0]]
    if _keep_dist(ctx, n):
        out = _repartition(ctx, mine, win, ctx.all_partitions(n), nc)
        return DistMatrix(out, n, nc, ctx.partition(n)[0], ctx)
    return _allgather_rows(ctx, mine, [e - s for s, e in win], nc).contiguous()


def lix(x, y, rl, ru, cl, cu):
    """X[r0:r1, c0:c1] = Y with X row-partitioned: each rank updates the rows it owns, taking
    the matching rows of Y (replicated: sliced; row-partitioned: repartitioned to X's
    layout).  A replicated X with a distributed Y gathers Y (the target is replicated)."""
    C = _C()
    if not _is_d(x):
        return C.lix(x, _fallback(y, "lix:replicated-target"), rl, ru, cl, cu)
    ctx = x.ctx
    r0 = _bnd(rl) or 1
    r1 = _bnd(ru) or x.nrows
    c0 = _bnd(cl) or 1
    c1 = _bnd(cu) or x.ncols
    if r0 < 1 or r1 > x.nrows or r0 > r1 or c0 < 1 or c1 > x.ncols or c0 > c1:
        raise DMLRuntimeError(f"Invalid values for matrix indexing: [{r0}:{r1},{c0}:{c1}] "
                              f"must be within matrix dimensions [{x.nrows},{x.ncols}]")
    n, nc = r1 - r0 + 1, c1 - c0 + 1
    parts = ctx.all_partitions(x.nrows)
    me = ctx.rank
    # rows of the target window owned by each rank, in window coordinates
    win = [_isect((s - (r0 - 1), e - (r0 - 1)), (0, n)) for s, e in parts]
    ws, we = win[me]
    loc = _dense(x.local)
    if _is_d(y):
        if y.nrows != n or y.ncols != nc:
            raise DMLRuntimeError(f"left indexing: {y.shape} does not match [{r0}:{r1},{c0}:{c1}]")
        ly = _repartition(ctx, y.local, ctx.all_partitions(n), win, nc)
    elif isinstance(y, torch.Tensor):
        # validated on every rank before any rank returns early, so a mismatch raises
        # everywhere instead of leaving the ranks with rows in the window blocked in the
        # next collective
        if tuple(y.shape) != (n, nc) and y.numel() != 1:
            raise DMLRuntimeError(f"left indexing dimension mismatch: target [{r0}:{r1},{c0}:{c1}] "
                                  f"vs source {y.shape[0]}x{y.shape[1]}")
        ly = y if y.numel() == 1 else y[ws:we]
    else:
        ly = y
    if we <= ws:
        return x
    lr0 = ws + (r0 - 1) - x.start
    out = C.lix(loc, ly, lr0 + 1, lr0 + (we - ws), c0, c1)
    return x.like(out)


def cbind(args):
    ref = next(a for a in args if _is_d(a))
    parts = []
    for a in args:
        la = _align(a, ref)
        if not isinstance(la, torch.Tensor):
            raise DMLRuntimeError("cbind of a distributed matrix with a scalar")
        parts.append(_C().cvt(_dense(la)))
    r = torch.cat(parts, 1)
    return DistMatrix(r, ref.nrows, r.shape[1], ref.start, ref.ctx)


def rbind(args):
    """rbind with at least one row-partitioned argument: every argument's rows are mapped
    into the result's row space and repartitioned with one p2p exchange per distributed
    argument (replicated arguments are sliced locally)."""
    C = _C()
    ctx = next(a for a in args if _is_d(a)).ctx
    mats = []
    for a in args:
        if _is_d(a) or isinstance(a, torch.Tensor):
            mats.append(a)
        else:
            mats.append(torch.full((1, 1), float(S.as_double(a)), dtype=torch.float64, device=ctx.device))
    ncols = mats[0].shape[1]
    for m in mats:
        if m.shape[1] != ncols:
            raise DMLRuntimeError(f"rbind: number of columns does not match ({m.shape[1]} vs {ncols})")
    N = sum(m.shape[0] for m in mats)
    keep = _keep_dist(ctx, N)
    dst = ctx.all_partitions(N) if keep else [(0, N)] * ctx.world
    me = ctx.rank
    pieces = []
    off = 0
    for m in mats:
        n = m.shape[0]
        mydst = _isect((dst[me][0] - off, dst[me][1] - off), (0, n))
        if _is_d(m):
            src = ctx.all_partitions(n)
            if keep:
                wins = [_isect((d0 - off, d1 - off), (0, n)) for d0, d1 in dst]
                pieces.append(_repartition(ctx, m.local, src, wins, ncols))
            else:
                pieces.append(_allgather_rows(ctx, m.local, [e - s for s, e in src], ncols))
        else:
            pieces.append(C.cvt(m)[mydst[0]:mydst[1]])
        off += n
    dt = pieces[0].dtype
    r = torch.cat([p.to(dt) for p in pieces], 0) if len(pieces) > 1 else pieces[0]
    if keep:
        return DistMatrix(r.contiguous(), N, ncols, dst[me][0], ctx)
    return r.contiguous()


def wquat(p, a):
    """Weighted quaternary operators with a row-partitioned W / X (reference: the Spark
    quaternary instructions with a broadcast factor): U is co-partitioned with the rows of
    X (or sliced from a replicated U), V is replicated (broadcast if it crossed the
    distribution threshold).  Every rank runs the fused sparse kernel on its rows; scalar
    losses and t(U) %*% (...) are all-reduced, row-shaped results stay partitioned."""
    from ..ops import quaternary as Q
    k = p["kind"]
    big = next(x for x in a if _is_d(x))
    ctx = big.ctx
    loc = []
    for i, x in enumerate(a):
        if k in ("wsloss", "wcemm", "wumm") and i in (0, 1, 3) or k in ("wsigmoid", "wdivmm") and i in (0, 1):
            loc.append(_align(x, big) if isinstance(x, (torch.Tensor, DistMatrix)) and
                       (not isinstance(x, torch.Tensor) or x.shape[0] == big.nrows) else x)
        elif i == 2:
            loc.append(_bcast(x, "wquat:V"))
        else:
            loc.append(_align(x, big) if _is_d(x) else x)
    if big.local.shape[0] == 0:
        r = _empty_wquat(p, loc, big)
    else:
        r = Q.execute(p, loc)
    if k in ("wsloss", "wcemm"):
        return ctx.allreduce_scalar(float(r), "sum", device=big.local.device if big.local.is_cuda else None)
    if k == "wdivmm" and p["left"]:
        r = _dense(r).to(torch.float64).contiguous()     # one dtype on every rank (empty blocks too)
        ctx.allreduce_(r, "sum")
        return r
    return DistMatrix(r, big.nrows, r.shape[1], big.start, ctx)


def _empty_wquat(p, loc, big):
    k = p["kind"]
    if k in ("wsloss", "wcemm"):
        return 0.0
    V = loc[2]
    if k == "wdivmm":
        if p["left"]:
            return torch.zeros((loc[1].shape[1], V.shape[0]), dtype=torch.float32, device=big.local.device)
        return torch.zeros((0, V.shape[1]), dtype=torch.float32, device=big.local.device)
    return torch.zeros((0, big.ncols), dtype=torch.float32, device=big.local.device)


def remove_empty_rows(x, select=None):
    """removeEmpty(target=X, margin="rows"[, select=s]) on a row-partitioned X: local filter,
    an all-gather of the per-rank counts, then a repartition of the surviving rows."""
    ctx = x.ctx
    loc = _dense(x.local)
    if select is not None:
        keep = (_dense(_align(select, x)).reshape(-1) != 0)
    else:
        keep = (loc != 0).any(1) if loc.shape[0] else torch.zeros(0, dtype=torch.bool, device=loc.device)
    kept = loc[keep]
    cnt = torch.tensor([[float(kept.shape[0])]], dtype=torch.float64,
                       device=ctx.device if tdist.get_backend(ctx.group) != "gloo" else "cpu")
    counts = [int(v) for v in _allgather_rows(ctx, cnt, [1] * ctx.world, 1).reshape(-1).tolist()]
    total = sum(counts)
    src, s = [], 0
    for c in counts:
        src.append((s, s + c))
        s += c
    if total == 0:
        return torch.zeros((1, x.ncols), dtype=loc.dtype, device=loc.device)   # reference: one empty row
    if _keep_dist(ctx, total):
        out = _repartition(ctx, kept, src, ctx.all_partitions(total), x.ncols)
        return DistMatrix(out, total, x.ncols, ctx.partition(total)[0], ctx)
    return _allgather_rows(ctx, kept, counts, x.ncols)


def onehot(exec_ctx, y, n, k):
    """Row-aligned one-hot of a row-partitioned label vector (table(seq(1,N), y, N, K))."""
    from ..runtime import builtins as B
    if n is not None and int(n) >= 0 and int(n) != y.nrows:
        return B.b_onehot(exec_ctx, _fallback(y, "onehot"), n, k)
    if k is None or int(k) < 0:
        loc = y.local
        kmax = float(loc.max().item()) if loc.numel() else 0.0
        k = int(y.ctx.allreduce_scalar(kmax, "max", device=loc.device if loc.is_cuda else None))
    return y.like(B.b_onehot(exec_ctx, _dense(y.local), y.local.shape[0], k))


def table(exec_ctx, A, B, W, dims):
    """ctable(seq(1,N), y, [w], N, K) → one-hot rows stay local; general case: each rank
    builds the contingency table of its rows and the (small) tables are all-reduced
    (reference: the Spark ctable + aggregation by key)."""
    from ..runtime.builtins import b_table
    from ..ops.backend import backend
    ref = A if _is_d(A) else B
    ctx = ref.ctx
    if _is_d(A) and _is_d(B) and A.nrows == B.nrows and not isinstance(W, (torch.Tensor, DistMatrix)):
        a = _dense(A.local).reshape(-1)
        expect = torch.arange(A.start + 1, A.start + a.numel() + 1, dtype=a.dtype, device=a.device)
        is_seq = bool(torch.equal(a, expect))
        flag = ctx.allreduce_scalar(0.0 if is_seq else 1.0, "max", device=a.device if a.is_cuda else None)
        if flag == 0.0 and (dims is None or dims[0] == A.nrows):
            b = _dense(B.local).reshape(-1)
            k = dims[1] if dims is not None else int(agg("max", "all", B))
            w = 1.0 if W is None else float(W)
            out = torch.zeros((a.numel(), k), dtype=backend.dtype, device=a.device)
            bi = torch.round(b).long() - 1
            keep = (bi >= 0) & (bi < k)
            rows = torch.arange(a.numel(), device=a.device)
            out[rows[keep], bi[keep]] = w
            return DistMatrix(out, A.nrows, k, A.start, ctx)
    # general: co-partitioned (or scalar) operands -> local tables of a common shape, summed
    la = _dense(_align(A, ref)) if isinstance(A, (torch.Tensor, DistMatrix)) else A
    lb = _dense(_align(B, ref)) if isinstance(B, (torch.Tensor, DistMatrix)) else B
    lw = _dense(_align(W, ref)) if isinstance(W, (torch.Tensor, DistMatrix)) else W
    if dims is None:
        ma = agg("max", "all", A) if _is_d(A) else (float(la.max().item()) if isinstance(la, torch.Tensor) else la)
        mb = agg("max", "all", B) if _is_d(B) else (float(lb.max().item()) if isinstance(lb, torch.Tensor) else lb)
        dims = (int(S.as_double(ma)), int(S.as_double(mb)))
    args = [la, lb] + ([lw] if W is not None else []) + list(dims)
    if ref.local.shape[0]:
        t = _dense(b_table(exec_ctx, *args)).to(torch.float64).contiguous()
    else:
        t = torch.zeros((int(dims[0]), int(dims[1])), dtype=torch.float64)
    t = t.to(ctx.device if tdist.get_backend(ctx.group) != "gloo" else "cpu")
    ctx.allreduce_(t, "sum")
    from ..ops.backend import place
    return place(t.to(backend.dtype))
