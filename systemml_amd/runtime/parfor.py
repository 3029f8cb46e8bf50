"""Parallel for-loops (reference: runtime/controlprogram/ParForProgramBlock.java,
parfor/{LocalParWorker,TaskPartitioner*,ResultMergeLocalMemory}.java).

Execution model:
  * iterations are split into tasks by a task partitioner (`naive` = one iteration per
    task, `static` = one contiguous chunk per worker, `fixed` = chunks of `taskSize`,
    `factoring` = geometrically shrinking chunks as in TaskPartitionerFactoring);
  * local workers (threads; large torch kernels release the GIL) execute tasks on
    private copies of the symbol table;
  * result variables (written in the body and live after the loop) are merged into
    the original with the reference's "merge with compare" semantics: every cell a
    worker changed relative to the pre-loop value is copied into the result;
    accumulators (variables only updated by `+=`, ResultMergeLocalMemory's accumulate
    mode) are merged as the pre-loop value plus every worker's increment.
On the GPU / SPMD backends workers run on one stream in task order (same result,
no host thread contention); `par=1` or `mode=LOCAL` with one worker is sequential.
"""
from __future__ import annotations

import math
import threading
from concurrent.futures import ThreadPoolExecutor

import torch

from ..parser.errors import DMLRuntimeError


def parfor_iterations(start, end, incr, as_int):
    """Iteration values of a parfor: ceil((to - from + 1) / incr) of them starting at `from`
    (reference ParForProgramBlock.computeNumIterations, ParForProgramBlock.java:1756) -- so a
    parfor over 1:0 runs zero times, where a plain for loop counts down."""
    n = int(math.ceil((float(end) - float(start) + 1.0) / float(incr)))
    return [int(start + k * incr) if as_int else float(start + k * incr) for k in range(max(0, n))]


def _iterations(start, end, incr, as_int):
    out = []
    i = start
    cnt = 0
    while (incr > 0 and i <= end) or (incr < 0 and i >= end):
        out.append(int(i) if as_int else float(i))
        cnt += 1
        i = start + cnt * incr
    return out


def partition_tasks(iters, k, mode="factoring", task_size=None):
    n = len(iters)
    if n == 0:
        return []
    mode = (mode or "factoring").lower()
    if mode == "naive":
        return [[x] for x in iters]
    if mode == "static":
        size = math.ceil(n / k)
        return [iters[i:i + size] for i in range(0, n, size)]
    if mode in ("fixed", "fixedsize"):
        size = int(task_size or 1)
        return [iters[i:i + size] for i in range(0, n, size)]
    # factoring: each round hands out k tasks of size ceil(remaining / (2k))
    tasks, pos = [], 0
    while pos < n:
        size = max(1, math.ceil((n - pos) / (2 * k)))
        for _ in range(k):
            if pos >= n:
                break
            tasks.append(iters[pos:pos + size])
            pos += size
    return tasks


def _merge(base, results):
    """ResultMergeLocalMemory with compare: copy every changed cell."""
    if isinstance(base, torch.Tensor):
        out = None
        for r in results:
            if not isinstance(r, torch.Tensor) or r is base:
                continue
            if r.shape != base.shape:
                raise DMLRuntimeError("parfor result merge: dimension change of a result variable")
            if out is None:
                out = base.clone()
            same = (r == base) | (torch.isnan(r) & torch.isnan(base))
            changed = ~same
            out[changed] = r[changed].to(out.dtype)
        return base if out is None else out
    changed = [r for r in results if r is not base and not _eq(r, base)]
    return changed[-1] if changed else base


def _eq(a, b):
    try:
        return a == b
    except Exception:  # noqa: BLE001
        return False


def _body_reads(blocks, out=None):
    from ..compiler.blocks import BasicBlock, IfBlock, WhileBlock, ForBlock
    out = set() if out is None else out
    for x in blocks:
        if isinstance(x, BasicBlock):
            out |= set(x.reads)
        elif isinstance(x, IfBlock):
            out |= x.pred.reads
            _body_reads(x.then_blocks, out)
            _body_reads(x.else_blocks, out)
        elif isinstance(x, WhileBlock):
            out |= x.pred.reads
            _body_reads(x.body, out)
        elif isinstance(x, ForBlock):
            for p in (x.start, x.end, x.incr):
                if p is not None:
                    out |= p.reads
            _body_reads(x.body, out)
    return out


def _run_iters(wctx, b, iters, idx, fork):
    from .program import exec_blocks, SeedSource
    for k, it in zip(idx, iters):
        wctx.seeds = SeedSource.iteration_source(fork, k)
        wctx.vars[b.var] = it
        exec_blocks(wctx, b.body)


def exec_parfor(ctx, b, start, end, incr, as_int):
    from .program import ExecutionContext
    iters = parfor_iterations(start, end, incr, as_int)
    if not iters:
        return
    fork = ctx.seeds.fork()
    par = b.params.get("par")
    k = int(par) if isinstance(par, (int, float)) and par else ctx.config.parallelism
    k = max(1, min(k, len(iters)))
    result_vars = list(b.result_vars)
    base = {v: ctx.vars.get(v) for v in result_vars}
    if ctx.dist is not None and ctx.dist.world > 1 and _spmd_ok(ctx, b):
        exec_parfor_spmd(ctx, b, iters, fork, result_vars, base)
        return
    sequential = k == 1 or ctx.dist is not None or (torch.cuda.is_available() and _on_gpu())
    if sequential:
        saved = ctx.seeds
        try:
            _run_iters(ctx, b, iters, range(len(iters)), fork)
        finally:
            ctx.seeds = saved
        return
    tasks = partition_tasks(list(enumerate(iters)), k, b.params.get("taskpartitioner", "factoring"),
                            b.params.get("tasksize"))
    lock = threading.Lock()
    queue = list(tasks)

    def worker():
        wctx = ExecutionContext(ctx.program, ctx.config, stats=ctx.stats, out=ctx._out, dist=None)
        wctx.vars = dict(ctx.vars)
        wctx.parfor_worker = True        # program.exec_block: serialise recompiling blocks
        while True:
            with lock:
                if not queue:
                    break
                task = queue.pop(0)
            _run_iters(wctx, b, [it for _, it in task], [i for i, _ in task], fork)
        return {v: wctx.vars.get(v) for v in result_vars}

    with ThreadPoolExecutor(max_workers=k) as ex:
        futs = [ex.submit(worker) for _ in range(k)]
        results = [f.result() for f in futs]
    acc = set(getattr(b, "accumulators", ()))
    for v in result_vars:
        rs = [r[v] for r in results]
        ctx.vars[v] = _accumulate(base[v], rs) if v in acc else _merge(base[v], rs)
    ctx.vars[b.var] = iters[-1]


def _accumulate(base, results):
    """Accumulator merge: base + sum over workers of (worker value - base)."""
    out = base
    for r in results:
        if r is base:
            continue
        if isinstance(base, torch.Tensor) or isinstance(r, torch.Tensor):
            rt = torch.as_tensor(r)
            if isinstance(base, torch.Tensor) and rt.shape != base.shape:
                raise DMLRuntimeError("parfor result merge: dimension change of an accumulator")
            out = out + (rt.to(base.device if isinstance(base, torch.Tensor) else rt.device) - base)
        else:
            out = out + (r - base)
    return out


# ----------------------------------------------------------------------------
# SPMD ("remote") parfor across GPU ranks
# ----------------------------------------------------------------------------
def _spmd_ok(ctx, b):
    """Iterations can run rank-locally when the body reads no row-partitioned matrix (a
    body touching one would issue collectives a different number of times per rank).
    mode=LOCAL keeps every rank executing every iteration."""
    from ..ops import core as C
    if str(b.params.get("mode", "")).upper() == "LOCAL":
        return False
    for v in _body_reads(b.body):
        if C.is_dist(ctx.vars.get(v)):
            return False
    return True


def exec_parfor_spmd(ctx, b, iters, fork, result_vars, base):
    """Remote parfor over the ranks of an SPMD run (reference: RemoteParForSpark -- there
    each task runs on a Spark executor; here each rank runs a contiguous range of iterations
    on its own GPU with rank-local operators), then the result variables are merged like
    ResultMergeLocalMemory with compare, across ranks: every rank all-reduces the cells its
    iterations changed (values and a change mask), so each rank ends with the merged
    matrix.  Scalars take the value of the last iteration that changed them."""
    from .program import ExecutionContext
    dist = ctx.dist
    parts = dist.all_partitions(len(iters))
    lo, hi = parts[dist.rank]
    wctx = ExecutionContext(ctx.program, ctx.config, stats=ctx.stats,
                            out=ctx._out if dist.rank == 0 else (lambda s: None), dist=None)
    wctx.vars = dict(ctx.vars)
    _run_iters(wctx, b, iters[lo:hi], range(lo, hi), fork)
    from ..parallel import dist as D
    D.stats["parfor_remote"] = D.stats.get("parfor_remote", 0) + 1
    acc = set(getattr(b, "accumulators", ()))
    for v in result_vars:
        if v in acc:
            ctx.vars[v] = _accumulate_spmd(dist, base[v], wctx.vars.get(v), lo < hi)
        else:
            ctx.vars[v] = _merge_spmd(dist, base[v], wctx.vars.get(v), lo < hi, hi)
    ctx.vars[b.var] = iters[-1]


def _accumulate_spmd(dist, base, mine, ran):
    """Accumulator merge across ranks: base + all-reduce-sum of every rank's increment."""
    import torch.distributed as tdist
    mine = mine if ran else base
    if isinstance(base, torch.Tensor):
        dev = dist.device if tdist.get_backend(dist.group) != "gloo" else torch.device("cpu")
        b = base.to(dev)
        m = torch.as_tensor(mine).to(device=dev, dtype=torch.float64)
        if m.shape != b.shape:
            raise DMLRuntimeError("parfor result merge: dimension change of an accumulator")
        d = m - b.double()
        dist.allreduce_(d, "sum")
        return (b.double() + d).to(base.dtype).to(base.device)
    return base + dist.allreduce_scalar(float(mine) - float(base), "sum")


def _merge_spmd(dist, base, mine, ran, last_idx):
    import torch.distributed as tdist
    if isinstance(base, torch.Tensor) and base.layout == torch.strided:
        dev = dist.device if tdist.get_backend(dist.group) != "gloo" else torch.device("cpu")
        b = base.to(dev)
        if isinstance(mine, torch.Tensor) and mine is not base and ran:
            if mine.shape != base.shape:
                raise DMLRuntimeError("parfor result merge: dimension change of a result variable")
            m = mine.to(device=dev, dtype=b.dtype)
            changed = ~((m == b) | (torch.isnan(m) & torch.isnan(b)))
        else:
            m = b
            changed = torch.zeros(b.shape, dtype=torch.bool, device=dev)
        # a cell changed on several ranks (possible with check=0) takes the value of the
        # highest-ranked writer -- the rank that ran the latest iterations, as the sequential
        # loop would leave it -- never a sum of the writers' values
        owner = torch.where(changed, torch.full((), float(dist.rank), dtype=torch.float64, device=dev),
                            torch.full((), -1.0, dtype=torch.float64, device=dev))
        dist.allreduce_(owner, "max")
        mine_wins = owner == float(dist.rank)
        val = torch.where(mine_wins, m.double(), torch.zeros((), dtype=torch.float64, device=dev))
        dist.allreduce_(val, "sum")
        out = torch.where(owner >= 0, val.to(b.dtype), b)
        return out.to(base.device)
    # scalars / other values: the rank that ran the highest-numbered iteration changing it wins
    changed = ran and not _eq(mine, base)
    objs = [None] * dist.world
    tdist.all_gather_object(objs, (last_idx if changed else -1, mine if changed else None), group=dist.group)
    best = max(objs, key=lambda o: o[0])
    return base if best[0] < 0 else best[1]


def _on_gpu():
    from ..ops.backend import backend
    return backend.on_gpu
