"""Program execution (reference: runtime/controlprogram/{Program,ProgramBlock,
IfProgramBlock,WhileProgramBlock,ForProgramBlock,ParForProgramBlock,
FunctionProgramBlock}.java, context/ExecutionContext.java).

SPMD model for multi-GPU: every rank executes the same control program;
row-partitioned matrices live in each rank's HBM and all scalars that steer
control flow are produced by collectives, so ranks stay in lock-step without
a driver/worker split.
"""
from __future__ import annotations

import collections
import sys
import threading
import time
import weakref

import torch

from ..parser.errors import DMLRuntimeError, DMLScriptStop
from ..compiler.blocks import BasicBlock, IfBlock, WhileBlock, ForBlock
from . import scalars as S
from .bufferpool import Evicted
from ..utils import hosttrace as _HT


class ExecutionContext:
    def __init__(self, program, config, stats=None, out=None, dist=None):
        self.vars = {}
        self.program = program
        self.config = config
        self.stats = stats
        self.dist = dist
        self._out = out
        self.depth = 0
        self.frame_stack = []        # callers' variable frames (buffer-pool eviction candidates)
        self.debugger = None         # utils/debugger.Debugger when run with -debug
        self.pool = None
        self.seeds = SeedSource(config, dist)
        self.owned = OwnedBuffers()      # buffers owned by update-in-place loops (compiler/loops.py)
        self.shared_results = frozenset()   # ids of parfor in-place result buffers (runtime/parfor.py)
        if dist is not None and config is not None:
            dist.min_rows = config.dist_min_rows
        if config is not None and getattr(config, "bufferpool", False) and torch.cuda.is_available():
            from .bufferpool import BufferPool
            self.pool = BufferPool(config)

    def frames(self):
        return self.frame_stack + [self.vars]

    def print(self, s):
        if self.dist is not None and self.config.print_rank0_only and self.dist.rank != 0:
            return
        if self._out is not None:
            self._out(s)
        else:
            sys.stdout.write(s + "\n")
            sys.stdout.flush()


class OwnedBuffers:
    """Identity set of tensors held weakly (a WeakSet would compare tensors with their
    elementwise ==)."""

    def __init__(self):
        self._d = {}

    def __contains__(self, t):
        r = self._d.get(id(t))
        return r is not None and r() is t

    def add(self, t):
        k = id(t)
        d = self._d
        d[k] = weakref.ref(t, lambda _r, k=k: d.pop(k, None) if d.get(k) is _r else None)

    def discard(self, t):
        if t in self:
            del self._d[id(t)]


class SeedSource:
    """Seeds for rand/sample calls without an explicit seed.  With `sysml.random.seed` set
    (config.seed >= 0) they are a deterministic sequence; in an SPMD run rank 0's random
    base seed is broadcast so every rank draws the same replicated values (ranks execute
    the same program, so their call sequences agree)."""

    def __init__(self, config, dist=None):
        import threading
        self.lock = threading.Lock()
        self.count = 0
        base = getattr(config, "seed", -1) if config is not None else -1
        if (base is None or base < 0) and dist is not None:
            import random
            v = float(random.getrandbits(40)) if dist.rank == 0 else 0.0
            base = int(dist.allreduce_scalar(v, "sum"))
        self.base = base if base is not None and base >= 0 else None

    def next(self):
        if self.base is None:
            return -1
        with self.lock:
            self.count += 1
            return (self.base * 7919 + self.count * 104729) % (1 << 62)

    def fork(self):
        """One draw of this stream for a parfor loop: every iteration derives its own stream
        from it (iteration_source), so an iteration sees the same random numbers whichever
        worker, thread or rank runs it, and this stream advances the same on every rank."""
        return None if self.base is None else self.next()

    @staticmethod
    def iteration_source(fork, key):
        import threading
        c = SeedSource.__new__(SeedSource)
        c.lock = threading.Lock()
        c.count = 0
        c.base = None if fork is None else (fork * 31 + int(key) * 1000003 + 17) % (1 << 62)
        return c


# ----------------------------------------------------------------------------
def _to_bool(v):
    if type(v) is S.DevScalar:
        return bool(v.value())
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise DMLRuntimeError("predicate must evaluate to a scalar")
        return bool(v.reshape(-1)[0].item() != 0)
    return S.as_bool(v)


def _to_num(v):
    if type(v) is S.DevScalar:
        return v.value()
    if isinstance(v, torch.Tensor):
        if v.numel() != 1:
            raise DMLRuntimeError("loop bound must be a scalar")
        return float(v.reshape(-1)[0].item())
    if isinstance(v, bool):
        return int(v)
    if isinstance(v, str):
        return S.parse_literal_arg(v)
    return v


def _attach_pos(e, pos):
    msg = str(e)
    if pos is not None and "line" not in msg:
        return type(e)(f"{pos}: {msg}")
    return e


def _run_ins(ctx, ins, slots):
    if ctx.debugger is not None:
        ctx.debugger.on_instruction(ctx, ins, slots)
    try:
        return ins.fn(ctx, [slots[i] for i in ins.ins])
    except torch.OutOfMemoryError:
        # reactive buffer-pool eviction (reference: CacheableData eviction on heap pressure)
        if ctx.pool is None or not ctx.pool.on_oom(ctx.frames()):
            raise
        return ins.fn(ctx, [slots[i] for i in ins.ins])


def _plan(owner, instrs, nslots):
    """Fast-path plan of an instruction list: literals pre-filled into a slot template,
    transient reads as (slot, name) pairs fetched up front, and the remaining compute
    instructions.  Literals and variable reads are a majority of a solver loop's instructions;
    within a basic block variables only change at the block's end, so reading them first is
    equivalent.  Cached on the owning block / predicate for its current instruction list
    (dynamic recompilation swaps the list)."""
    cached = getattr(owner, "_plan", None)
    if cached is not None and cached[0] is instrs:
        return cached[1]
    tmpl = [None] * nslots
    reads = []
    rest = []
    for ins in instrs:
        if ins.opcode == "lit":
            tmpl[ins.out] = ins.hop.p["v"]
        elif ins.opcode == "tread":
            reads.append((ins.out, ins.hop.p["name"]))
        else:
            rest.append(ins)
    plan = (tmpl, tuple(reads), tuple(rest))
    owner._plan = (instrs, plan)
    return plan


_SLOW = object()
DeferredError = None        # runtime/instructions.DeferredError, bound on first use (import cycle)


def _exec_fast(ctx, plan):
    global DeferredError
    if DeferredError is None:
        from .instructions import DeferredError as _D
        DeferredError = _D
    tmpl, reads, rest = plan
    slots = tmpl.copy()
    vars_ = ctx.vars
    pool = ctx.pool
    for s, name in reads:
        v = vars_.get(name, _SLOW)
        tv = type(v)
        if v is _SLOW or tv is DeferredError:
            return None             # undefined / deferred: the ordered path raises where it should
        if pool is not None:
            if tv is Evicted:
                v = pool.restore(vars_, name, v)
            pool.touch(vars_, name)
        slots[s] = v
    for ins in rest:
        try:
            try:
                slots[ins.out] = ins.fn(ctx, [slots[i] for i in ins.ins])
            except torch.OutOfMemoryError:
                if ctx.pool is None or not ctx.pool.on_oom(ctx.frames()):
                    raise
                slots[ins.out] = ins.fn(ctx, [slots[i] for i in ins.ins])
        except DMLScriptStop:
            raise
        except DMLRuntimeError as e:
            raise _attach_pos(e, ins.hop.pos) from e
        except (RuntimeError, ValueError, TypeError, IndexError, ZeroDivisionError) as e:
            raise DMLRuntimeError(f"{ins.hop.pos}: error in {ins.opcode}: {e}") from e
        for f in ins.free:
            slots[f] = None
    return slots


FAST_PATH = True


def exec_instrs(ctx, instrs, nslots, owner=None):
    stats = ctx.stats
    if FAST_PATH and owner is not None and ctx.debugger is None and (stats is None or not stats.enabled):
        slots = _exec_fast(ctx, _plan(owner, instrs, nslots))
        if slots is not None:
            return slots
    slots = [None] * nslots
    if stats is not None and stats.enabled:
        sync = stats.sync
        for ins in instrs:
            t0 = time.perf_counter()
            try:
                r = _run_ins(ctx, ins, slots)
            except DMLScriptStop:
                raise
            except DMLRuntimeError as e:
                raise _attach_pos(e, ins.hop.pos) from e
            except (RuntimeError, ValueError, TypeError, IndexError, ZeroDivisionError) as e:
                raise DMLRuntimeError(f"{ins.hop.pos}: error in {ins.opcode}: {e}") from e
            if sync and torch.cuda.is_available() and isinstance(r, torch.Tensor) and r.is_cuda:
                torch.cuda.synchronize()
            stats.record(ins.opcode, time.perf_counter() - t0)
            slots[ins.out] = r
            for f in ins.free:
                slots[f] = None
        return slots
    for ins in instrs:
        try:
            slots[ins.out] = _run_ins(ctx, ins, slots)
        except DMLScriptStop:
            raise
        except DMLRuntimeError as e:
            raise _attach_pos(e, ins.hop.pos) from e
        except (RuntimeError, ValueError, TypeError, IndexError, ZeroDivisionError) as e:
            raise DMLRuntimeError(f"{ins.hop.pos}: error in {ins.opcode}: {e}") from e
        for f in ins.free:
            slots[f] = None
    return slots


def eval_pred(ctx, pred):
    _HT.mark("pred")
    if pred.is_const:
        return pred.const
    slots = exec_instrs(ctx, pred.instrs, pred.nslots, pred)
    return slots[pred.out]


def exec_blocks(ctx, blocks):
    for b in blocks:
        exec_block(ctx, b)


_BLOCK_LOCKS = weakref.WeakKeyDictionary()
_LOCKS_GUARD = threading.Lock()


def _block_lock(b):
    with _LOCKS_GUARD:
        lk = _BLOCK_LOCKS.get(b)
        if lk is None:
            lk = _BLOCK_LOCKS[b] = threading.Lock()
        return lk


def exec_block(ctx, b):
    if isinstance(b, BasicBlock) and getattr(ctx, "parfor_worker", False) and \
            (b.recompile or getattr(b, "exec_recompile", False)):
        # dynamic recompilation replaces the block's plan (instructions, slot count, output
        # slots) for the operand shapes at hand; parfor workers sharing the block must not
        # interleave a recompilation with another worker's execution of the same block
        with _block_lock(b):
            return _exec_basic(ctx, b)
    if isinstance(b, BasicBlock):
        return _exec_basic(ctx, b)
    return _exec_control(ctx, b)


def _exec_basic(ctx, b):
    _HT.mark("block-start")
    if True:
        if ctx.debugger is not None:
            ctx.debugger.cur_block = b
        if b.recompile:
            from ..compiler.cost import recompile_block
            from .instructions import make_impl
            if recompile_block(b, ctx.vars, make_impl, ctx.config) and ctx.stats is not None:
                ctx.stats.count("recompiled blocks")
        if getattr(b, "exec_recompile", False):
            from ..compiler.cost import recompile_exec_types, runtime_plan
            if recompile_exec_types(b, ctx.vars, ctx.config):
                if ctx.stats is not None:
                    ctx.stats.count("recompiled exec types")
                if ctx.config is not None and ctx.config.explain == "recompile_runtime":
                    ctx.print(f"# EXPLAIN (recompile_runtime): block at line "
                              f"{b.pos.line if b.pos else '?'}\n" + runtime_plan(b, "  "))
        _HT.mark("block-plan")
        if getattr(b, "licm_pre", False):
            # hoisted loop invariants: a failure surfaces only if the loop reads the value
            try:
                slots = exec_instrs(ctx, b.instrs, b.nslots, b)
            except DMLRuntimeError as e:
                from .instructions import DeferredError
                for name, _ in b.writes_slots:
                    ctx.vars[name] = DeferredError(e)
                return
        else:
            slots = exec_instrs(ctx, b.instrs, b.nslots, b)
        vars_ = ctx.vars
        for name, s in b.writes_slots:
            vars_[name] = slots[s]
        for name in b.rmvars:
            vars_.pop(name, None)
        if ctx.pool is not None:
            ctx.pool.maybe_evict(ctx.frames())
        _HT.mark("block-end")
        return


def _exec_control(ctx, b):
    if isinstance(b, IfBlock):
        if _to_bool(eval_pred(ctx, b.pred)):
            if getattr(b, "vguard", False):
                # if-converted block (compiler/ifconv.py): it evaluates both branches; an error
                # there may belong to the branch not taken, so the original control flow decides
                try:
                    exec_blocks(ctx, b.then_blocks)
                except DMLRuntimeError:
                    exec_blocks(ctx, b.else_blocks)
                return
            exec_blocks(ctx, b.then_blocks)
        else:
            exec_blocks(ctx, b.else_blocks)
        return
    uip = getattr(b, "inplace_vars", None)
    if uip:
        # loop entry: buffers of update-in-place variables may be aliased by now (e.g. `Y = X`
        # after a previous run of this loop), so the first left-indexing copies again
        for v in uip:
            x = ctx.vars.get(v)
            # a parfor worker's shared in-place result stays shared: its workers write
            # disjoint cells of that one buffer (runtime/parfor.py)
            if isinstance(x, torch.Tensor) and id(x) not in ctx.shared_results:
                ctx.owned.discard(x)
    if isinstance(b, WhileBlock):
        if RUNAHEAD and _runahead_ok(ctx, b):
            t0 = time.perf_counter()
            try:
                return _exec_while_runahead(ctx, b)
            finally:
                runahead_stats["t"] += time.perf_counter() - t0
        while _to_bool(eval_pred(ctx, b.pred)):
            exec_blocks(ctx, b.body)
        return
    if isinstance(b, ForBlock):
        start = _to_num(eval_pred(ctx, b.start))
        end = _to_num(eval_pred(ctx, b.end))
        if b.incr is not None:
            incr = _to_num(eval_pred(ctx, b.incr))
        else:
            incr = 1 if start <= end else -1
        if incr == 0:
            raise DMLRuntimeError("for loop increment must not be zero")
        as_int = all(isinstance(x, int) or (isinstance(x, float) and x.is_integer()) for x in (start, end, incr)) \
            and not any(isinstance(x, float) and not x.is_integer() for x in (start, incr))
        if b.parfor:
            from .parfor import exec_parfor
            exec_parfor(ctx, b, start, end, incr, as_int)
            return
        i = start
        cnt = 0
        while (incr > 0 and i <= end) or (incr < 0 and i >= end):
            ctx.vars[b.var] = int(i) if as_int else float(i)
            exec_blocks(ctx, b.body)
            cnt += 1
            i = start + cnt * incr
        return
    raise DMLRuntimeError(f"unknown block type {type(b).__name__}")


# ----------------------------------------------------------------------------
# run-ahead while loops
# ----------------------------------------------------------------------------
# A data-dependent while loop on the GPU backend costs one device round trip per iteration:
# the host reads the predicate back, and only then queues the next iteration, so the device
# idles for the host's whole per-iteration time (reference: WhileProgramBlock.execute
# evaluates the predicate synchronously; on a CPU that is free).  A run-ahead loop queues
# iteration k+1 BEFORE it reads iteration k's predicate:
#   * vector programs leave their scalar results in HBM (ops/vprog.py, backend.defer), so the
#     next iteration's kernels take them from there and the predicate is a device value;
#   * the predicate's copy to pinned host memory is queued with an event behind it
#     (DevScalar.start_read); the host waits for that event one iteration later, while the
#     device already works on the next iteration;
#   * the queued iteration carries the device address of that predicate (backend.live): the
#     streaming kernels (ops/hip/chain4.hip, mfma_chain.hip) and vector programs read it first
#     and return at once when it is 0, so the one speculative iteration past the loop's end
#     costs a few microseconds of launches, not a pass over X;
#   * variables are immutable tensors / values, so a dead iteration is undone by restoring
#     the variable map it started from.
# Only bodies without side effects qualify (no print / write / stop, function calls, random
# generators, nested loops or update-in-place indexing): compiler facts checked once per loop.
RUNAHEAD = __import__("os").environ.get("SYSML_RUNAHEAD", "1") != "0"
_RA_BAD_BI = frozenset({"print", "write", "stop", "assert", "printf", "rand", "sample", "time", "read", "eval",
                        "list", "exists", "toString", "setwd"})
_RA_BAD_OPS = frozenset({"fcall", "sink"})
# SYSML_RUNAHEAD_PRINTS=1: a loop that prints runs ahead too (its lines buffered per iteration).
# Off by default: on the headline's LinearRegCG loop it measured within box noise (10M rows
# 400.6 vs 407.8 ms on one box, 397.7 vs 394.6 on another; profiles/runahead_prints_r6.txt)
_RA_PRINTS = __import__("os").environ.get("SYSML_RUNAHEAD_PRINTS", "0") == "1"


def _pure_hops(roots):
    from ..compiler import hops as H
    for h in H.walk(roots):
        if h.op in _RA_BAD_OPS:
            # print(x): a run-ahead iteration buffers its lines and the loop prints them once
            # the iteration is known to be live (builtins.b_print, _exec_while_runahead)
            if _RA_PRINTS and h.op == "sink" and h.p.get("name") == "print" and len(h.inputs) == 1 \
                    and not h.named:
                continue
            return False
        if h.op == "bi" and h.p.get("name") in _RA_BAD_BI:
            return False
        if h.op == "lix" and h.p.get("inplace"):
            return False
    return True


def _pure_blocks(blocks):
    for b in blocks:
        if isinstance(b, BasicBlock):
            if not _pure_hops(list(b.roots) + list(b.env_out.values())):
                return False
        elif isinstance(b, IfBlock):
            if not (b.pred.is_const or _pure_hops([b.pred.root])):
                return False
            if not (_pure_blocks(b.then_blocks) and _pure_blocks(b.else_blocks)):
                return False
        else:
            return False            # nested loops keep their own control flow
    return True


def _runahead_ok(ctx, b):
    if ctx.debugger is not None or getattr(ctx, "parfor_worker", False) or (ctx.stats is not None and ctx.stats.enabled):
        return False
    from ..ops.backend import backend
    if not (backend.on_gpu and backend.use_kernels) or backend.lazy:
        return False
    ok = getattr(b, "_runahead", None)
    if ok is None:
        ok = b._runahead = (not getattr(b, "inplace_vars", None) and not b.pred.is_const
                            and _pure_hops([b.pred.root]) and _pure_blocks(b.body))
        if ok:
            from .graphloop import _has_print
            b._ra_has_print = _has_print(b.body)
    if ok and b._ra_has_print:
        # a printing loop's deferred strings and device-side scalar algebra cost the host more
        # per iteration than its synchronous prints: worth it only when the device work of an
        # iteration is large (10M x 1K: 400.6 vs 407.8 ms; 1.25M x 1K: 77.8 vs 72.7 ms)
        return _streams_big(ctx, b)
    return ok


RA_PRINT_MIN_CELLS = 1 << 32


def _streams_big(ctx, b):
    from ..ops import augmented as AUG
    for v in getattr(b, "body_live_in", ()) or ():
        x = ctx.vars.get(v)
        if hasattr(x, "local") and hasattr(x, "nrows"):
            # a row-partitioned matrix: the global size over the ranks -- every rank must take
            # the same decision (a speculative iteration issues collectives)
            if x.nrows * x.ncols // max(1, x.ctx.world) >= RA_PRINT_MIN_CELLS:
                return True
            continue
        x = x.X if AUG.is_cc(x) else x
        if isinstance(x, torch.Tensor) and x.numel() >= RA_PRINT_MIN_CELLS:
            return True
    return False


runahead_stats = {"loops": 0, "iterations": 0, "dead": 0, "host_pred": 0, "t": 0.0}


def _pred_var(b):
    """(variable, inverted) when the loop predicate is `v` or `!v` for a variable v, else None:
    then a device-resident v serves as the live flag itself (inverted: bit 0 of its address,
    ops/hip/chain4.hip sysml_dead) and no negation is queued per iteration."""
    r = getattr(b, "_pred_var", False)
    if r is False:
        h = b.pred.root
        r = None
        if h.op == "tread":
            r = (h.p["name"], False)
        elif h.op == "u" and h.p.get("o") == "not" and h.inputs[0].op == "tread":
            r = (h.inputs[0].p["name"], True)
        b._pred_var = r
    return r


# Iterations queued past an unresolved predicate: with depth k the host reads iteration i's
# predicate only after queueing iteration i + k, so host and device overlap even when their
# per-iteration times are equal (depth 1 stalls the device whenever the host jitters).
# Deeper iterations may run on the (skipped, garbage) outputs of a dead one; bodies with
# operators that index memory by data values (table / one-hot / gathers / order / grouped
# aggregates) therefore stay at depth 1, where a dead iteration still reads live data.
# Default 1: on the headline the host's per-iteration time exceeds the device's at the 8-GPU
# per-rank size (1.25M rows: depth 3 70.9 vs depth 1 71.1 ms/step) and the chained flags cost
# a launch per iteration at 10M (388 vs 382 ms; profiles/headline_check_r6a.txt).
RUNAHEAD_DEPTH = max(1, int(__import__("os").environ.get("SYSML_RUNAHEAD_DEPTH", "1")))
_RA_INDEXING_BI = frozenset({"table", "ctable", "_onehot", "_gather_rows", "removeEmpty", "order", "aggregate",
                             "rexpand", "_seq_expand", "replace", "transformapply", "transformdecode"})


def _runahead_depth(b):
    d = getattr(b, "_ra_depth", None)
    if d is None:
        from ..compiler import hops as H
        roots = [b.pred.root]
        stack = list(b.body)
        while stack:
            x = stack.pop()
            if isinstance(x, BasicBlock):
                roots.extend(list(x.roots) + list(x.env_out.values()))
            elif isinstance(x, IfBlock):
                roots.append(x.pred.root)
                stack.extend(x.then_blocks)
                stack.extend(x.else_blocks)
        deep = not any(h.op == "bi" and h.p.get("name") in _RA_INDEXING_BI for h in H.walk(roots))
        d = b._ra_depth = RUNAHEAD_DEPTH if deep else 1
    return d


def _exec_while_runahead(ctx, b):
    from ..ops.backend import backend
    if not _to_bool(eval_pred(ctx, b.pred)):
        return
    runahead_stats["loops"] += 1
    from . import graphloop as _GL
    if _GL.try_entry(ctx, b, runahead_stats):      # replay of a graph captured at an earlier entry
        return
    vars_ = ctx.vars
    pv = _pred_var(b)
    depth = _runahead_depth(b)
    n_queued = 0
    # queued iterations whose predicates are unread: (predicate after the iteration, inverted,
    # variable map after the iteration)
    pending = collections.deque()

    def emit(buf):
        for x in buf:
            ctx.print(x if type(x) is str else str(x))

    def drain(keep, unqueued=0):
        """Read predicates oldest first until `keep` remain; True when one ends the loop (the
        variable map is then the one after that last live iteration).  `unqueued`: iterations
        run but not in `pending` (dead too when an earlier predicate ends the loop).  An
        iteration reached here is live (every earlier predicate continued the loop): its
        buffered prints go out, before its own predicate is tested."""
        while len(pending) > keep:
            q, inv, after, buf = pending.popleft()
            emit(buf)
            if bool(q.value()) == inv:
                runahead_stats["dead"] += len(pending) + unqueued
                vars_.clear()
                vars_.update(after)
                pending.clear()
                return True
        return False

    flag = None        # depth > 1: device flag "every queued iteration so far is live"
    try:
        while True:
            live = 0
            if pending:
                q0, inv0 = pending[-1][0], pending[-1][1]
                if q0.t.is_cuda and q0.t.dtype == torch.float64:
                    live = q0.t.data_ptr() | (1 if inv0 else 0)
                    if depth > 1:
                        # chain the flags: a dead iteration's predicate is never written, so the
                        # next one is live only if all earlier ones were (one 1-thread kernel)
                        from ..ops import kernels as _K
                        flag = _K.live_and(flag.data_ptr() if flag is not None else 0, live)
                        live = flag.data_ptr()
            else:
                flag = None            # nothing unresolved: this iteration is known live
            backend.set_runahead(True, live)
            err = None
            q = None
            qinv = False
            buf = ctx._ra_prints = []
            try:
                exec_blocks(ctx, b.body)
                v = vars_.get(pv[0]) if pv is not None else None
                if type(v) is S.DevScalar and v.t.is_cuda and v.t.dtype == torch.float64:
                    q, qinv = v, pv[1]              # the variable itself, read back late
                else:
                    q = eval_pred(ctx, b.pred)
                if type(q) is S.DevScalar:
                    q.start_read()
            except DMLScriptStop:
                raise
            except Exception as e:      # noqa: BLE001 - re-raised below unless the iteration was dead
                err = e
            ctx._ra_prints = None
            runahead_stats["iterations"] += 1
            if err is not None:
                # an error in an iteration past the loop's end is not an error
                if drain(0, 1):
                    return
                emit(buf)
                raise err
            if type(q) is S.DevScalar:
                pending.append((q, qinv, vars_.copy(), buf))
                if drain(depth):
                    return
                n_queued += 1
                if _GL.want_capture(ctx, b, n_queued):
                    # the rest of the loop as HIP-graph replays (runtime/graphloop.py): settle
                    # the queued iterations first, so the captured state is a live one
                    if drain(0):
                        return
                    flag = None
                    if _GL.capture_and_run(ctx, b, pv, exec_blocks, eval_pred, runahead_stats):
                        return
            else:
                runahead_stats["host_pred"] += 1
                if drain(0, 1):
                    return
                emit(buf)
                if not _to_bool(q):
                    return
    finally:
        ctx._ra_prints = None
        backend.set_runahead(False, 0)
        # strings built from unread device scalars leave the loop resolved (their reads were
        # queued with them; the variable map is a live iteration's)
        for k, v in list(vars_.items()):
            if type(v) is S.LazyStr:
                vars_[k] = str(v)


# ----------------------------------------------------------------------------
# functions
# ----------------------------------------------------------------------------
def _coerce(v, param):
    if param.dtype == "SCALAR" and not isinstance(v, torch.Tensor):
        vt = param.vtype
        try:
            if vt == "DOUBLE" and isinstance(v, (int, bool)) :
                return float(v)
            if vt == "INT" and isinstance(v, float) and v.is_integer():
                return int(v)
            if vt == "BOOLEAN" and not isinstance(v, bool) and isinstance(v, (int, float)):
                return bool(v)
        except (TypeError, ValueError):
            return v
    return v


def call_function(ctx, fkey, args, given):
    fb = ctx.program.functions.get(fkey)
    if fb is None:
        raise DMLRuntimeError(f"function {fkey[1]} not found")
    if fb.external:
        from .udf import call_external
        return call_external(ctx, fb, args, given)
    new_vars = {}
    params = {p.name: p for p in fb.inputs}
    for name, v in zip(given, args):
        new_vars[name] = _coerce(v, params[name])
    saved = ctx.vars
    for p in fb.inputs:
        if p.name not in new_vars:
            if p.name in fb.default_preds:
                ctx.vars = new_vars
                try:
                    new_vars[p.name] = _coerce(eval_pred(ctx, fb.default_preds[p.name]), p)
                finally:
                    ctx.vars = saved
            else:
                raise DMLRuntimeError(f"missing argument '{p.name}' in call to function {fb.name}")
    ctx.vars = new_vars
    ctx.depth += 1
    ctx.frame_stack.append(saved)
    if ctx.depth > 500:
        raise DMLRuntimeError("maximum function recursion depth exceeded")
    try:
        exec_blocks(ctx, fb.body)
    finally:
        ctx.vars = saved
        ctx.frame_stack.pop()
        ctx.depth -= 1
    outs = []
    for o in fb.outputs:
        if o.name not in new_vars:
            raise DMLRuntimeError(f"function {fb.name}: output variable '{o.name}' was not assigned")
        outs.append(_coerce(new_vars[o.name], o))
    return tuple(outs)


def eval_call(ctx, fname, args, named, nskey, imports):
    """DML `eval("fname", args...)` (reference: EvalNaryCPInstruction)."""
    from . import builtins as B
    fname = S.to_str(fname)
    ns = None
    if "::" in fname:
        ns, fname = fname.split("::", 1)
    key = imports.get(ns) if ns else nskey
    fb = ctx.program.functions.get((key, fname))
    if fb is None and ns is None:
        fb = ctx.program.functions.get((".defaultNS", fname))
    if fb is not None:
        names = [p.name for p in fb.inputs]
        given = names[:len(args)] + list(named.keys())
        out = call_function(ctx, (fb.namespace, fb.name), list(args) + list(named.values()), given)
        return out[0] if len(out) == 1 else out
    fn = B.REGISTRY.get(fname)
    if fn is None:
        from ..ops import core as C
        unary = {"abs", "exp", "log", "sqrt", "round", "floor", "ceil", "sign", "sin", "cos", "tan"}
        if fname in unary:
            return C.unary(fname, args[0])
        agg = {"sum": "sum", "mean": "mean", "min": "min", "max": "max", "prod": "prod"}
        if fname in agg:
            return C.agg(agg[fname], "all", args[0])
        raise DMLRuntimeError(f"eval: function '{fname}' not found")
    return fn(ctx, *args, **named)
