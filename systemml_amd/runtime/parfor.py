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
    worker changed relative to the pre-loop value is copied into the result.
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


def exec_parfor(ctx, b, start, end, incr, as_int):
    from .program import exec_blocks, ExecutionContext
    iters = parfor_iterations(start, end, incr, as_int)
    if not iters:
        return
    par = b.params.get("par")
    k = int(par) if isinstance(par, (int, float)) and par else ctx.config.parallelism
    k = max(1, min(k, len(iters)))
    sequential = k == 1 or ctx.dist is not None or (torch.cuda.is_available() and _on_gpu())
    result_vars = list(b.result_vars)
    base = {v: ctx.vars.get(v) for v in result_vars}
    if sequential:
        for it in iters:
            ctx.vars[b.var] = it
            exec_blocks(ctx, b.body)
        return
    tasks = partition_tasks(iters, k, b.params.get("taskpartitioner", "factoring"), b.params.get("tasksize"))
    lock = threading.Lock()
    queue = list(tasks)

    def worker():
        wctx = ExecutionContext(ctx.program, ctx.config, stats=ctx.stats, out=ctx._out, dist=None)
        wctx.vars = dict(ctx.vars)
        wctx.seeds = ctx.seeds
        while True:
            with lock:
                if not queue:
                    break
                task = queue.pop(0)
            for it in task:
                wctx.vars[b.var] = it
                exec_blocks(wctx, b.body)
        return {v: wctx.vars.get(v) for v in result_vars}

    with ThreadPoolExecutor(max_workers=k) as ex:
        futs = [ex.submit(worker) for _ in range(k)]
        results = [f.result() for f in futs]
    for v in result_vars:
        ctx.vars[v] = _merge(base[v], [r[v] for r in results])
    ctx.vars[b.var] = iters[-1]


def _on_gpu():
    from ..ops.backend import backend
    return backend.on_gpu
