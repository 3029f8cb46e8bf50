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
On the GPU backend each worker thread issues its iterations on a stream of its own (and,
with config.parfor_gpus > 1, on a device of its own: reference GPUContextPool.java:209
reserves one GPU context per parfor worker), so independent iterations overlap on the
MI355X's hardware queues; results merge on the main stream after every worker stream
has drained into it.  `par=1` or an SPMD run of a row-partitioned body is sequential.
The degree of parallelism, exec type and task partitioner are chosen by a rule-based
optimizer (`optimize`, reference opt/OptimizerRuleBased.java:197) unless the script
fixes them (par=, mode=, taskpartitioner=).
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
            if r.device != base.device:            # a worker's result placed on the host (or another GPU)
                r = r.to(base.device)
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


class PartView:
    """One worker's (or rank's) block of a partitioned matrix: rows (axis 0) or columns
    (axis 1) [start, start + extent) of a matrix of `shape`.  A parfor body reads and writes
    such a variable only as X[i, ] / X[, i] with i the loop variable (data_partitions), so
    indexing is all it supports (ops/core.py rix / lix dispatch here): the index is moved
    into the block, and an index outside it is an error instead of a silent wrong row."""
    __slots__ = ("local", "start", "axis", "shape")
    is_part_view = True

    def __init__(self, local, start, axis, shape):
        self.local = local
        self.start = int(start)
        self.axis = int(axis)
        self.shape = (int(shape[0]), int(shape[1]))

    def _move(self, lo, hi):
        from ..ops.core import _bound
        n = self.shape[self.axis]
        a, z = _bound(lo, 1), _bound(hi, n)
        ext = self.local.shape[self.axis]
        if a - 1 < self.start or z > self.start + ext:
            raise DMLRuntimeError(f"parfor data partition: {'row' if self.axis == 0 else 'column'} "
                                  f"range [{a}:{z}] outside this worker's block "
                                  f"[{self.start + 1}:{self.start + ext}]")
        return a - self.start, z - self.start

    def part_rix(self, rl, ru, cl, cu):
        from ..ops import core as C
        if self.axis == 0:
            a, z = self._move(rl, ru)
            return C.rix(self.local, a, z, cl, cu)
        a, z = self._move(cl, cu)
        return C.rix(self.local, rl, ru, a, z)

    def part_lix(self, y, rl, ru, cl, cu, owned=None):
        from ..ops import core as C
        if self.axis == 0:
            a, z = self._move(rl, ru)
            out = C.lix(self.local, y, a, z, cl, cu, owned=owned)
        else:
            a, z = self._move(cl, cu)
            out = C.lix(self.local, y, rl, ru, a, z, owned=owned)
        return self if out is self.local else PartView(out, self.start, self.axis, self.shape)

    def __repr__(self):
        return f"PartView({'rows' if self.axis == 0 else 'cols'} [{self.start},{self.start + self.local.shape[self.axis]}) of {self.shape})"


def _part_view(x, axis, lo, hi, dev=None):
    """Block [lo, hi) of matrix x along axis as a PartView (copied to `dev` when given)."""
    blk = x[lo:hi] if axis == 0 else x[:, lo:hi]
    if dev is not None and blk.device != dev:
        blk = blk.to(dev, non_blocking=True)
    return PartView(blk, lo, axis, x.shape)


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


class ParForPlan:
    """Decisions of the parfor optimizer (reference ParForProgramBlock's opt tree after
    OptimizerRuleBased.optimize): exec type, degree of parallelism, task partitioner and the
    row / column access pattern of the body's matrix reads (data partitioning candidates)."""
    __slots__ = ("exec_type", "k", "partitioner", "task_size", "partitions", "devices", "part_writes",
                 "inplace", "mem_worker", "mem_budget", "dist_parts")

    def __repr__(self):
        return (f"ParForPlan({self.exec_type}, k={self.k}, {self.partitioner}, devices={self.devices}, "
                f"partitions={self.partitions}, inplace={self.inplace})")


def _body_has(blocks, kinds):
    from ..compiler.blocks import IfBlock, WhileBlock, ForBlock
    for x in blocks:
        if isinstance(x, kinds):
            return True
        if isinstance(x, IfBlock) and (_body_has(x.then_blocks, kinds) or _body_has(x.else_blocks, kinds)):
            return True
        if isinstance(x, (WhileBlock, ForBlock)) and _body_has(x.body, kinds):
            return True
    return False


def data_partitions(b, writes=None):
    """Matrices the body reads only as X[i, ] or X[, i] with i the loop variable: the
    candidates of the reference's data partitioner (DataPartitionerLocal.java:79 writes them as
    row / column blocks so each task reads its own).  Returns {var: 'row' | 'col'}.  Left-
    indexing targets written only as R[i, ] = ... (or R[, i]) qualify too; `writes` (a set)
    collects their names.  A variable also read by a predicate, passed whole to any operator
    or indexed with anything but the loop variable is not a candidate."""
    from ..compiler.blocks import BasicBlock
    from ..compiler import hops as H
    acc = {}
    bad = set()
    wr = set() if writes is None else writes

    def is_var(z):
        return z.op == "tread" and z.p.get("name") == b.var

    def kind_of(rl, ru, cl, cu):
        # row i (any columns) / column i (any rows): the block owning row / column i holds it
        if is_var(rl) and (ru is rl or is_var(ru)):
            return "row"
        if is_var(cl) and (cu is cl or is_var(cu)):
            return "col"
        return None

    def note(name, kind):
        if kind is None or acc.get(name, kind) != kind:
            bad.add(name)
        else:
            acc[name] = kind

    def visit(blocks):
        from ..compiler.blocks import IfBlock, WhileBlock, ForBlock
        for x in blocks:
            if isinstance(x, BasicBlock):
                tops = list(x.roots) + list(x.env_out.values())
                for h in H.walk(tops):
                    if h.op == "lix":
                        base = h
                        while base.op == "lix":
                            base = base.inputs[0]
                        if base.op == "tread" and base.dt == "M":
                            wr.add(base.p["name"])
                            note(base.p["name"], kind_of(*h.inputs[2:6]))
                    for pos, c in enumerate(h.inputs):
                        if c.op != "tread" or c.dt != "M":
                            continue
                        name = c.p["name"]
                        if h.op == "lix" and pos == 0:
                            continue                      # the target: classified above
                        if h.op == "rix" and pos == 0:
                            note(name, kind_of(*h.inputs[1:5]))
                        else:
                            bad.add(name)
                for v, h in x.env_out.items():
                    if h.op == "tread" and h.dt == "M" and h.p.get("name") != v:
                        bad.add(h.p["name"])              # aliased whole (Y = X)
            elif isinstance(x, IfBlock):
                bad.update(x.pred.reads)
                visit(x.then_blocks)
                visit(x.else_blocks)
            elif isinstance(x, WhileBlock):
                bad.update(x.pred.reads)
                visit(x.body)
            elif isinstance(x, ForBlock):
                for p in (x.start, x.end, x.incr):
                    if p is not None:
                        bad.update(p.reads)
                visit(x.body)
    visit(b.body)
    wr -= bad
    return {k: v for k, v in acc.items() if k not in bad}


def optimize(ctx, b, n_iters, as_int=True):
    """Rule-based parfor optimizer (reference opt/OptimizerRuleBased.java:144-197):
      exec type  REMOTE_SPMD when the run has several ranks and the body reads no
                 row-partitioned matrix; REMOTE_SPMD_PARTITIONED when every row-partitioned
                 matrix the body touches is indexed only by the loop variable's row (each
                 rank runs the iterations of the rows it owns, no collective in the body);
                 LOCAL_GPU (worker streams / devices) on a GPU backend; LOCAL_CPU threads
                 otherwise;
      k          the script's par=, else the exec type's parallelism (GPU: one worker per
                 device used, times config.parfor_gpu_streams -- default 1, so a one-GPU
                 run without par= executes sequentially: worker streams sharing one GPU lost
                 to the serial loop, profiles/parfor_gpu_r5*.txt), capped by the
                 iterations and by the memory budget (rewriteSetDegreeOfParallelism,
                 :1178: free device / host memory over one worker's estimate);
      tasks      the script's taskpartitioner=, else STATIC for bodies of uniform cost (no
                 branches or inner while-loops) and FACTORING otherwise;
      data       row / column access patterns of the body's matrix reads and left-indexing
                 writes (data_partitions), applied by the SPMD and multi-device paths;
      results    in-place result indexing for variables the compiler marked
                 (compiler/loops.py: one shared private copy, no compare-matrix merge)."""
    from ..compiler.blocks import IfBlock, WhileBlock
    cfg = ctx.config
    pl = ParForPlan()
    mode = str(b.params.get("mode", "")).upper()
    par = b.params.get("par")
    pl.devices = 1
    pl.part_writes = set()
    pl.partitions = data_partitions(b, pl.part_writes)
    pl.dist_parts = None
    pl.mem_worker = pl.mem_budget = None
    if ctx.dist is not None and ctx.dist.world > 1 and mode != "LOCAL" and _spmd_ok(ctx, b):
        pl.exec_type = "REMOTE_SPMD"
        k = ctx.dist.world
    elif ctx.dist is not None and ctx.dist.world > 1 and mode != "LOCAL" and as_int and \
            (dp := _spmd_partitioned(ctx, b, pl)) is not None:
        pl.exec_type = "REMOTE_SPMD_PARTITIONED"
        pl.dist_parts = dp
        k = ctx.dist.world
    elif ctx.dist is not None:
        pl.exec_type = "SEQUENTIAL"          # every rank runs every iteration (row-partitioned body)
        k = 1
    elif _on_gpu() and torch.cuda.is_available():
        pl.exec_type = "LOCAL_GPU"
        ndev = max(1, min(int(getattr(cfg, "parfor_gpus", 1) or 1), torch.cuda.device_count()))
        pl.devices = ndev
        k = max(1, int(getattr(cfg, "parfor_gpu_streams", 1) or 1)) * ndev
    else:
        pl.exec_type = "LOCAL_CPU"
        k = cfg.parallelism
    if isinstance(par, (int, float)) and par and pl.exec_type not in ("REMOTE_SPMD", "REMOTE_SPMD_PARTITIONED", "SEQUENTIAL"):
        k = int(par)
    pl.k = max(1, min(k, n_iters))
    pl.inplace = [v for v in getattr(b, "parfor_inplace", ()) if v in b.result_vars and _inplace_ok(ctx.vars.get(v))]
    if pl.exec_type in ("LOCAL_GPU", "LOCAL_CPU") and pl.k > 1 and not (isinstance(par, (int, float)) and par):
        kb = _memory_k(ctx, b, pl)
        if kb is not None and kb < pl.k:
            pl.k = kb
    if pl.k == 1 and pl.exec_type in ("LOCAL_GPU", "LOCAL_CPU"):
        pl.exec_type = "SEQUENTIAL"
    pl.devices = min(pl.devices, pl.k)
    if pl.devices > 1:
        pl.inplace = []                      # workers on other GPUs update copies: merge them
    tp = b.params.get("taskpartitioner")
    if tp is None:
        tp = "factoring" if _body_has(b.body, (IfBlock, WhileBlock)) else "static"
    pl.partitioner = str(tp).lower()
    pl.task_size = b.params.get("tasksize")
    return pl


def _inplace_ok(x):
    return type(x) is torch.Tensor and x.layout == torch.strided and x.dim() == 2


def _body_mem(ctx, b, pl):
    """Bytes one worker needs: the largest basic block's matrix intermediates (sum of output
    sizes with the shapes of the current variables; an unknown size counts as the largest
    matrix the body reads) plus its private copies of result variables merged by compare."""
    from ..compiler import cost as CO
    from ..compiler import hops as H
    from ..compiler.blocks import BasicBlock, IfBlock, WhileBlock, ForBlock
    env = {}
    big = 0
    for v in _body_reads(b.body):
        x = ctx.vars.get(v)
        d = CO._shape_of(x)
        env[v] = d
        if CO._known(d) and d != CO.SCALAR:
            big = max(big, d[0] * d[1])
    env[b.var] = CO.SCALAR
    cell = 4 if (pl.exec_type == "LOCAL_GPU") else 8
    worst = 0

    def visit(blocks):
        nonlocal worst
        for x in blocks:
            if isinstance(x, BasicBlock):
                dims = {}
                tot = 0
                for h in H.walk(list(x.roots) + list(x.env_out.values())):
                    try:
                        d = CO.infer(h, dims, env)
                    except Exception:  # noqa: BLE001 -- an estimate only
                        d = CO.UNK
                    dims[h.id] = d
                    if h.dt != "M" or h.op in ("tread", "lit"):
                        continue
                    m = CO.mem_estimate(d, cell)
                    tot += big * cell if m is None else m
                for k, h in x.env_out.items():
                    env[k] = dims.get(h.id, CO.UNK)
                worst = max(worst, tot)
            elif isinstance(x, IfBlock):
                visit(x.then_blocks)
                visit(x.else_blocks)
            elif isinstance(x, (WhileBlock, ForBlock)):
                visit(x.body)
    visit(b.body)
    for v in b.result_vars:
        if v in pl.inplace:
            continue
        x = ctx.vars.get(v)
        if isinstance(x, torch.Tensor):
            worst += x.numel() * x.element_size()
    return worst


def _memory_k(ctx, b, pl):
    """Largest k whose workers fit the memory budget (reference computeMaxK): 70% of the free
    device memory (LOCAL_GPU) or of the available host memory (LOCAL_CPU), shared read-only
    inputs counted once (they are not copied per worker)."""
    try:
        need = _body_mem(ctx, b, pl)
    except Exception:  # noqa: BLE001
        return None
    if not need:
        return None
    try:
        if pl.exec_type == "LOCAL_GPU":
            free = torch.cuda.mem_get_info()[0] * pl.devices
        else:
            import psutil
            free = psutil.virtual_memory().available
    except Exception:  # noqa: BLE001
        return None
    budget = 0.7 * free * MEM_FRACTION
    pl.mem_worker, pl.mem_budget = need, budget
    return max(1, int(budget // need))


MEM_FRACTION = 1.0        # tests shrink the budget


def _spmd_partitioned(ctx, b, pl):
    """The row-partitioned matrices of an SPMD run the body touches, when every one of them is
    read and written only at row i (the loop variable) and all share one row partitioning:
    each rank then runs exactly the iterations whose rows it owns against its own block
    (reference DataPartitionerRemoteSpark + RemoteParForSpark over the partitioned input,
    here with the partition already in place).  None otherwise."""
    from ..ops import core as C
    dist = ctx.dist
    dv = [v for v in sorted(_body_reads(b.body)) if C.is_dist(ctx.vars.get(v))]
    if not dv:
        return None
    n = None
    for v in dv:
        x = ctx.vars[v]
        if pl.partitions.get(v) != "row" or x.local.layout != torch.strided:
            return None
        if n is None:
            n = x.nrows
        if x.nrows != n or x.start != dist.partition(n)[0] or x.local.shape[0] != dist.partition(n)[1] - x.start:
            return None
    for v in b.result_vars:
        if C.is_dist(ctx.vars.get(v)) and v not in pl.part_writes:
            return None
    return dv


def exec_parfor(ctx, b, start, end, incr, as_int):
    iters = parfor_iterations(start, end, incr, as_int)
    if not iters:
        return
    fork = ctx.seeds.fork()
    pl = optimize(ctx, b, len(iters), as_int)
    b.last_plan = pl                       # -explain / tests
    if ctx.stats is not None:
        ctx.stats.count(f"parfor {pl.exec_type.lower()} k={pl.k}")
    result_vars = list(b.result_vars)
    base = {v: ctx.vars.get(v) for v in result_vars}
    if pl.exec_type == "REMOTE_SPMD":
        exec_parfor_spmd(ctx, b, iters, fork, result_vars, base)
        return
    if pl.exec_type == "REMOTE_SPMD_PARTITIONED":
        exec_parfor_spmd_partitioned(ctx, b, iters, fork, result_vars, base, pl.dist_parts)
        return
    if pl.exec_type == "SEQUENTIAL":
        saved = ctx.seeds
        try:
            _run_iters(ctx, b, iters, range(len(iters)), fork)
        finally:
            ctx.seeds = saved
        return
    k = pl.k
    tasks = partition_tasks(list(enumerate(iters)), k, pl.partitioner, pl.task_size)
    lock = threading.Lock()
    queue = list(tasks)
    gpu = pl.exec_type == "LOCAL_GPU"
    main = torch.cuda.current_stream() if gpu else None
    main_dev = torch.cuda.current_device() if gpu else None
    # in-place result indexing: every worker updates one private copy of the pre-loop value
    from ..ops import core as C
    shared = {v: C.cvt(base[v]).clone(memory_format=torch.contiguous_format) for v in pl.inplace}
    # data partitions on other GPUs: each worker owns a fixed set of tasks and receives only
    # the rows / columns of the read-only partitioned matrices those iterations index
    parts = {v: a for v, a in pl.partitions.items() if v not in pl.part_writes and v not in result_vars
             and type(ctx.vars.get(v)) is torch.Tensor and ctx.vars[v].layout == torch.strided} \
        if gpu and pl.devices > 1 else {}
    own = [tasks[w::k] for w in range(k)] if parts else None

    def worker(w):
        from .program import ExecutionContext
        wctx = ExecutionContext(ctx.program, ctx.config, stats=ctx.stats, out=ctx._out, dist=None)
        wctx.vars = dict(ctx.vars)
        wctx.parfor_worker = True        # program.exec_block: serialise recompiling blocks
        for v, t in shared.items():
            wctx.vars[v] = t
            wctx.owned.add(t)
        wctx.shared_results = frozenset(id(t) for t in shared.values())

        def run():
            if own is not None:
                for task in own[w]:
                    _run_iters(wctx, b, [it for _, it in task], [i for i, _ in task], fork)
                return
            while True:
                with lock:
                    if not queue:
                        break
                    task = queue.pop(0)
                _run_iters(wctx, b, [it for _, it in task], [i for i, _ in task], fork)

        if not gpu:
            run()
            return {v: wctx.vars.get(v) for v in result_vars}, None
        dev = (main_dev + w) % torch.cuda.device_count() if pl.devices > 1 and w < pl.devices else main_dev
        from ..ops.backend import backend
        with torch.cuda.device(dev):
            s = _worker_stream(dev, w)
            s.wait_stream(main)              # inputs produced on the main stream
            backend.set_thread_device(torch.device("cuda", dev))
            try:
                with torch.cuda.stream(s):
                    if dev != main_dev:
                        wctx.vars = _to_device(wctx.vars, torch.device("cuda", dev), parts,
                                               [it for t in own[w] for _, it in t] if own is not None else None)
                    run()
            finally:
                backend.set_thread_device(None)
        out = {v: wctx.vars.get(v) for v in result_vars}
        if dev != main_dev:
            with torch.cuda.stream(s):
                out = _to_device(out, torch.device("cuda", main_dev), None)
        for v in out.values():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                v.record_stream(main)        # used on the main stream from now on
        return out, s

    # host workers share the cores: each one's operators get cores / k intra-op threads (the
    # reference's local workers run single-threaded CP operators), restored afterwards
    nt = torch.get_num_threads()
    if not gpu and not getattr(ctx, "parfor_worker", False):
        torch.set_num_threads(max(1, nt // k))
    try:
        if getattr(ctx, "parfor_worker", False):
            with ThreadPoolExecutor(max_workers=k) as ex:      # nested parfor: a pool of its own
                done = [f.result() for f in [ex.submit(worker, w) for w in range(k)]]
        else:
            ex = _pool(k)
            done = [f.result() for f in [ex.submit(worker, w) for w in range(k)]]
    finally:
        if torch.get_num_threads() != nt:
            torch.set_num_threads(nt)
    results = [r for r, _ in done]
    for _, s in done:
        if s is not None:
            main.wait_stream(s)
    acc = set(getattr(b, "accumulators", ()))
    for v in result_vars:
        if v in shared:
            # updated in place by every worker -- unless a worker's writes went to a copy (an
            # operand moved between host and device for the operator's exec type, a dtype
            # cast): those copies merge by comparison against the pre-loop value
            rs = [r[v] for r in results if r[v] is not shared[v]]
            ctx.vars[v] = shared[v] if not rs else _merge(base[v], [shared[v]] + rs)
            continue
        rs = [r[v] for r in results]
        ctx.vars[v] = _accumulate(base[v], rs) if v in acc else _merge(base[v], rs)
    ctx.vars[b.var] = iters[-1]


_STREAMS = {}
_POOL = [None, 0]


def _pool(k):
    """Worker threads kept for the process (thread start-up costs ~0.3 ms each here, more
    than a small parfor body), grown to the largest k seen."""
    ex, n = _POOL
    if ex is None or n < k:
        if ex is not None:
            ex.shutdown(wait=False)
        ex = ThreadPoolExecutor(max_workers=k, thread_name_prefix="parfor")
        _POOL[0], _POOL[1] = ex, k
    return ex


def _worker_stream(dev, w):
    """Worker w's stream on device dev, kept for the process: the caching allocator serves a
    stream from the blocks freed on it, so a fresh stream per parfor execution would pay a
    device allocation for every temporary of its first iterations."""
    s = _STREAMS.get((dev, w))
    if s is None:
        s = _STREAMS[(dev, w)] = torch.cuda.Stream(device=dev)
    return s


def _to_device(vars_, dev, partitions, its=None):
    """Copies of a worker's device-resident values on its own GPU (matrices only).  A
    partitioned matrix (partitions: {var: 'row' | 'col'}) read by iterations `its` is copied
    as the block of rows / columns min(its)..max(its) only, wrapped as a PartView."""
    out = {}
    if its:
        lo, hi = int(min(its)) - 1, int(max(its))
    for k, v in vars_.items():
        if isinstance(v, torch.Tensor) and v.is_cuda and v.device != dev:
            ax = {"row": 0, "col": 1}.get(partitions.get(k)) if partitions and its else None
            if ax is not None and 0 <= lo < hi <= v.shape[ax]:
                v = _part_view(v, ax, lo, hi, dev)
                part_stats["blocks"] += 1
                part_stats["bytes_saved"] += (v.shape[0] * v.shape[1] - v.local.numel()) * v.local.element_size()
            else:
                v = v.to(dev, non_blocking=True)
        out[k] = v
    return out


part_stats = {"blocks": 0, "bytes_saved": 0, "spmd_loops": 0}


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


def exec_parfor_spmd_partitioned(ctx, b, iters, fork, result_vars, base, dvars):
    """Each rank runs the iterations i whose row i it owns in the common row partitioning of
    the body's row-partitioned matrices, against its local blocks (PartView: indexing moved
    into the block, no collective).  Row-partitioned results are updated in the rank's own
    block and need no merge; replicated results merge as in exec_parfor_spmd.  An iteration
    outside 1..nrow runs on rank 0, where indexing raises as the sequential loop would."""
    from .program import ExecutionContext
    from ..ops import core as C
    dist = ctx.dist
    n = ctx.vars[dvars[0]].nrows
    lo, hi = dist.partition(n)
    mine = [(k, it) for k, it in enumerate(iters)
            if lo <= int(it) - 1 < hi or (dist.rank == 0 and not 0 <= int(it) - 1 < n)]
    wctx = ExecutionContext(ctx.program, ctx.config, stats=ctx.stats,
                            out=ctx._out if dist.rank == 0 else (lambda s: None), dist=None)
    wctx.vars = dict(ctx.vars)
    for v in dvars:
        x = ctx.vars[v]
        loc = x.local
        if v in result_vars:
            loc = C.cvt(loc).clone(memory_format=torch.contiguous_format)
            wctx.owned.add(loc)
        wctx.vars[v] = PartView(loc, x.start, 0, x.shape)
    _run_iters(wctx, b, [it for _, it in mine], [k for k, _ in mine], fork)
    from ..parallel import dist as D
    D.stats["parfor_remote_partitioned"] = D.stats.get("parfor_remote_partitioned", 0) + 1
    part_stats["spmd_loops"] += 1
    acc = set(getattr(b, "accumulators", ()))
    last = (mine[-1][0] + 1) if mine else 0
    for v in result_vars:
        x = base[v]
        if C.is_dist(x):
            pv = wctx.vars.get(v)
            ctx.vars[v] = x.like(pv.local) if getattr(pv, "is_part_view", False) else x
        elif v in acc:
            ctx.vars[v] = _accumulate_spmd(dist, x, wctx.vars.get(v), bool(mine))
        else:
            ctx.vars[v] = _merge_spmd(dist, x, wctx.vars.get(v), bool(mine), last)
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
