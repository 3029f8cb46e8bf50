"""Run-ahead while loops replayed as HIP graphs (runtime/program.py _exec_while_runahead; no
reference counterpart -- the reference interprets every WhileProgramBlock iteration,
runtime/controlprogram/WhileProgramBlock.java:95-136).

A run-ahead loop body is pure device work on device-resident state (run-ahead already
requires that), so after a few iterations op by op -- vector-program plans compiled, shapes
settled -- one iteration is captured into a HIP graph and every further iteration is one
`hipGraphLaunch`: the host's per-iteration interpretation (tens of instruction dispatches)
leaves the critical path, which at the 8-GPU per-rank size is what bounds the solvers' inner
CG loops (profiles/idle_gaps_1250k_r6b.txt).

The captured iteration reads and writes fixed buffers:

  * loop state -- every variable the body assigns that is live after an iteration
    (`WhileBlock.iter_live`, compiler/translator.py) -- lives in static buffers; host
    scalars among it (iteration counters) are promoted to device scalars for the graph;
  * invariants the body reads (`body_live_in` minus its writes) are bound by address when
    large (X), staged in static buffers when small or scalar (refilled when the loop is
    entered again: the next outer iteration's P, delta^2), or baked into the graph when they
    are host integers / strings (checked for equality on re-entry);
  * the graph ends with ONE commit launch (chain4.hip commit_live_kernel) that copies the
    iteration's state and predicate into the static buffers only when the iteration is live.
    Its first node snapshots the previous predicate into the live flag its kernels test, so
    a speculative replay past the loop's end changes nothing: run-ahead can be DEPTH
    iterations deep without the garbage-input hazard of op-by-op run-ahead.

SPMD runs (SYSML_GRAPH_DIST=1, RCCL): collectives stay outside the graphs -- the capture is
cut at every all-reduce into segments, and a replay is segment, all-reduce (issued by the host
on the segment's fixed buffer), segment, ... so every rank issues exactly the collectives of
the op-by-op iteration, in the same order; the ranks agree on the capture's success with one
all-reduce, and replay exactly as deep as op-by-op run-ahead would queue.

Any host synchronisation the body needs (a data-dependent branch, an upload, an `.item()`)
makes the capture fail; the loop then continues op by op and is never captured again.
SYSML_RUNAHEAD_GRAPH=1 enables graph replay; SYSML_GRAPH_DEPTH (default 2) sets how many
replays may be queued past an unread predicate (single process)."""
from __future__ import annotations

import collections
import gc
import os
import threading
import time
import weakref

import torch

from . import scalars as S

ENABLED = os.environ.get("SYSML_RUNAHEAD_GRAPH", "0") == "1"
DIST = os.environ.get("SYSML_GRAPH_DIST", "0") == "1"
DEPTH = max(1, int(os.environ.get("SYSML_GRAPH_DEPTH", "2")))
MIN_ITERS = 2                  # op-by-op iterations of the first entry before the capture
COPY_MAX_BYTES = 1 << 30       # invariant matrices up to this size are staged in static buffers
MAX_COMMIT = 15                # state variables (+ the predicate) of the one commit launch

stats = {"captures": 0, "failed": 0, "entries": 0, "replays": 0, "dead": 0, "rebind_fail": 0, "segments": 0,
         "host_uploads": 0, "t_bind": 0.0, "t_replay": 0.0, "t_wait": 0.0, "t_exit": 0.0, "t_capture": 0.0,
         "why": ""}

_SEG = [None]                  # the segmented capture in progress (DistContext.allreduce_ hook)
# Graphs are destroyed only under _LOCK, which every capture holds: a hipGraph destroyed while
# any stream captures is an error (the plans of a finished step die on whichever thread drops
# them -- the bench's plan-hydration thread, the cyclic collector).  _ALL keeps every graph
# alive past its loop block; _sweep frees those whose block is gone.
_LOCK = threading.Lock()
_ALL = []
_BYKEY = {}                          # loop key (api/executor._tag_loops) -> GraphLoop of a recompiled loop
_BYKEY_MAX = 32
_RETIRED = []


def _sweep():
    if any(r() is None for r, _ in _ALL):
        _ALL[:] = [e for e in _ALL if e[0]() is not None]


def capturing():
    return _SEG[0]


def _all_writes(blocks):
    from ..compiler.translator import _all_writes as aw
    return aw(blocks)


def _has_print(blocks):
    from ..compiler import hops as H
    from ..compiler.blocks import BasicBlock, IfBlock
    roots = []
    stack = list(blocks)
    while stack:
        x = stack.pop()
        if isinstance(x, BasicBlock):
            roots.extend(list(x.roots) + list(x.env_out.values()))
        elif isinstance(x, IfBlock):
            roots.append(x.pred.root)
            stack.extend(x.then_blocks)
            stack.extend(x.else_blocks)
    return any(h.op == "sink" for h in H.walk(roots))


def _is_dm(x):
    from ..parallel.dist import DistMatrix
    return type(x) is DistMatrix


def _local(x):
    """The device tensor behind a matrix value (a row-partitioned one's local block)."""
    return x.local if _is_dm(x) else x


def _dev_tensor(x):
    t = _local(x)
    return type(t) is torch.Tensor and t.is_cuda and t.layout is torch.strided


def _host_tensor(x):
    return type(x) is torch.Tensor and not x.is_cuda and x.layout is torch.strided


def _dev_scalar(x):
    return type(x) is S.DevScalar and x.t.is_cuda and x.t.dtype == torch.float64 and x.t.numel() == 1


def _host_num(x):
    return type(x) in (int, float, bool)


def _same_kind(a, b):
    return a == b or (a.is_floating_point and b.is_floating_point)


def _vt(x):
    return "b" if type(x) is bool else ("i" if type(x) is int else "d")


def _dm_meta(x):
    return (x.nrows, x.ncols, x.start, id(x.ctx)) if _is_dm(x) else None


class _Segments:
    """Graphs of one captured iteration, cut at the collectives (SPMD) -- one graph otherwise."""

    def __init__(self):
        self.pool = torch.cuda.graph_pool_handle()
        self.items = []
        self.g = None

    def begin(self):
        self.g = torch.cuda.CUDAGraph()
        self.g.capture_begin(pool=self.pool, capture_error_mode="relaxed")

    def end(self):
        g, self.g = self.g, None
        g.capture_end()
        self.items.append(("g", g))

    def collective(self, dctx, t, op):
        self.end()
        self.items.append(("c", dctx, t, op))
        self.begin()

    def replay(self):
        for it in self.items:
            if it[0] == "g":
                it[1].replay()
            else:
                it[1].allreduce_(it[2], it[3])


class GraphLoop:
    """Static buffers, the captured graph and the binding rules of one while loop."""

    def __init__(self, b, pv, dist):
        # no reference to the block: b._graph = self must not form a cycle, or the cyclic
        # collector could free a graph (hipGraphExecDestroy) while another loop is capturing
        self.pv = pv
        self.dist = dist
        self.inv = bool(pv[1]) if pv is not None else False
        self.seg = None
        self.st = {}          # state / staged-invariant name -> static device tensor (a local block)
        self.kind = {}        # name -> 'T' state matrix | 'D' state scalar (vt) | 'C' staged matrix
        #                        | 'E' staged scalar | 'A' by address | 'B' baked host value
        self.vt = {}
        self.dm = {}          # name -> (nrows, ncols, start, id(ctx)) of a row-partitioned value
        self.dmx = {}         # name -> the DistMatrix the static block stands for (its ctx)
        self.meta = {}        # 'A': (data_ptr, shape, stride, dtype); 'B': (type, value); 'C': (shape, dtype)
        self.src = {}         # 'C' / 'E': (value, _version) last staged (skip unchanged re-copies)
        self.commit = []
        self.carried = set()
        self.st_q = torch.empty((), dtype=torch.float64, device="cuda")
        self.fl = torch.empty((), dtype=torch.float64, device="cuda")
        self.one = torch.ones((), dtype=torch.float64, device="cuda")     # always-live flag (staging)
        self.hstage = None
        self.busy = False     # replaying (a loop of another thread's plan must not share the buffers)

    # ------------------------------------------------------------------ classification
    def _static_for(self, v, x):
        t = _local(x)
        self.st[v] = torch.empty(tuple(t.shape), dtype=t.dtype, device="cuda")
        if _is_dm(x):
            self.dm[v] = _dm_meta(x)
            self.dmx[v] = x

    def classify(self, b, vars_):
        live = getattr(b, "iter_live", None)
        lin = getattr(b, "body_live_in", None)
        if live is None or lin is None:
            return False
        if _has_print(b.body):
            stats["why"] = "prints"            # buffered per live iteration: op by op only
            return False
        writes = _all_writes(b.body)
        self.commit = sorted(writes & live)
        self.carried = set(lin) & writes
        if len(self.commit) > MAX_COMMIT:
            stats["why"] = "commit set"
            return False
        for v in self.commit:
            x = vars_.get(v)
            if x is None:
                if v in self.carried:
                    return False
                self.kind[v] = "T?"             # written before read: static made at capture
            elif _dev_tensor(x) or _host_tensor(x):
                self.kind[v] = "T"
                self._static_for(v, x)
            elif _dev_scalar(x) or _host_num(x):
                self.kind[v] = "D"
                self.vt[v] = x.vt if type(x) is S.DevScalar else _vt(x)
                self.st[v] = torch.empty((), dtype=torch.float64, device="cuda")
            else:
                stats["why"] = f"state {v}: {type(x).__name__}"
                return False
        for v in (set(lin) | set(b.pred.reads)) - writes:
            if v not in vars_:
                return False
            x = vars_[v]
            if _dev_tensor(x):
                t = _local(x)
                if t.numel() * t.element_size() <= COPY_MAX_BYTES:
                    self.kind[v] = "C"
                    self._static_for(v, x)
                    self.meta[v] = (tuple(t.shape), t.dtype)
                else:
                    self.kind[v] = "A"
                    self.meta[v] = (t.data_ptr(), tuple(t.shape), t.stride(), t.dtype, _dm_meta(x))
            elif _host_tensor(x) and x.numel() <= 1 << 22:
                self.kind[v] = "C"
                self._static_for(v, x)
                self.meta[v] = (tuple(x.shape), x.dtype)
            elif _dev_scalar(x) or type(x) in (float, bool):
                self.kind[v] = "E"
                self.vt[v] = x.vt if type(x) is S.DevScalar else _vt(x)
                self.st[v] = torch.empty((), dtype=torch.float64, device="cuda")
            elif type(x) in (int, str) or x is None:
                self.kind[v] = "B"
                self.meta[v] = (type(x), x)
            else:
                stats["why"] = f"input {v}: {type(x).__name__}"
                return False
        return True

    # ------------------------------------------------------------------ binding
    def _fits(self, v, k, x):
        if k == "A":
            t = _local(x)
            return _dev_tensor(x) and (t.data_ptr(), tuple(t.shape), t.stride(), t.dtype, _dm_meta(x)) == self.meta[v]
        if k == "B":
            return (type(x), x) == self.meta[v]
        if k == "C":
            t = _local(x)
            return (type(t) is torch.Tensor and t.layout is torch.strided and tuple(t.shape) == self.meta[v][0]
                    and _same_kind(t.dtype, self.meta[v][1]) and _dm_meta(x) == self.dm.get(v))
        if k == "E":
            return _dev_scalar(x) or type(x) in (float, bool, int)
        if k == "T":
            if v not in self.carried:
                return True
            t, st = _local(x), self.st[v]
            return (type(t) is torch.Tensor and t.layout is torch.strided and tuple(t.shape) == tuple(st.shape)
                    and _same_kind(t.dtype, st.dtype) and _dm_meta(x) == self.dm.get(v))
        if k == "D":
            return v not in self.carried or _dev_scalar(x) or _host_num(x)
        return True

    def bind(self, vars_):
        """Stage the entry state into the static buffers; False when the graph does not fit
        (a baked value or an address-bound matrix changed, or a shape did).  Floating-point
        state and staged matrices are converted to the captured dtype (a fresh host-placed
        zero matrix entering a loop whose graph was captured on its fp32 device state)."""
        t0 = time.perf_counter()
        for v, k in self.kind.items():
            x = vars_.get(v)
            if not self._fits(v, k, x):
                t = _local(x)
                stats["why"] = f"{v}:{k}:{type(x).__name__}:" + (
                    str((tuple(t.shape), t.dtype, t.device.type)) if isinstance(t, torch.Tensor) else repr(x)[:40])
                return False
        # staging: device sources and host scalars (packed into one upload) go into the static
        # buffers with one copy launch (commit_live with an always-live flag)
        pairs, hv, hd = [], [], []
        for v, k in self.kind.items():
            x = vars_.get(v)
            if k in ("A", "B", "T?") or (k in ("T", "D") and v not in self.carried):
                continue
            if k in ("C", "E"):
                last = self.src.get(v)
                ver = _local(x)._version if k == "C" else None
                if last is not None and last[0] is x and last[1] == ver:
                    continue                       # the same (unmodified) value as last time
                self.src[v] = (x, ver)
            st = self.st[v]
            if k in ("T", "C"):
                t = _local(x)
                if not t.is_cuda:
                    st.copy_(t)
                    stats["host_uploads"] += 1
                    continue
                if t.dtype != st.dtype:
                    t = t.to(st.dtype)
                pairs.append((t.contiguous(), st))
            elif type(x) is S.DevScalar:
                pairs.append((x.t.reshape(()).contiguous(), st))
            else:
                hv.append(float(x))
                hd.append(st)
        hv.append(0.0 if self.inv else 1.0)           # the loop was entered: its predicate holds
        hd.append(self.st_q)
        n = len(hv)
        if self.hstage is None or self.hstage.numel() < n:
            self.hstage = torch.empty(max(n, 8), dtype=torch.float64, device="cuda")
        self.hstage[:n].copy_(torch.tensor(hv, dtype=torch.float64).pin_memory(), non_blocking=True)
        pairs.extend((self.hstage[i], d) for i, d in enumerate(hd))
        self._copy(pairs)
        stats["t_bind"] += time.perf_counter() - t0
        return True

    def _copy(self, pairs):
        from ..ops import kernels as K
        for i in range(0, len(pairs), K.COMMIT_MAX):
            K.commit_live(pairs[i:i + K.COMMIT_MAX], self.one.data_ptr())

    def _wrap(self, v, t):
        if v in self.dm:
            x = self.dmx[v]
            from ..parallel.dist import DistMatrix
            return DistMatrix(t, x.nrows, t.shape[1] if t.dim() > 1 else x.ncols, x.start, x.ctx)
        return t

    def _cap_vars(self, vars_):
        cv = dict(vars_)
        for v, k in self.kind.items():
            if k in ("T", "C"):
                cv[v] = self._wrap(v, self.st[v])
            elif k in ("D", "E"):
                cv[v] = S.DevScalar(self.st[v], self.vt[v])
            elif k == "T?":
                cv.pop(v, None)
        return cv

    # ------------------------------------------------------------------ capture
    def _commit_pairs(self, cv, q):
        statics = {t.data_ptr() for t in self.st.values()}
        pairs = []
        for v in self.commit:
            y = cv.get(v)
            k = self.kind[v]
            if k == "T?":
                if not _dev_tensor(y):
                    raise _NoGraph(v)
                self.kind[v] = "T"
                self._static_for(v, y)
                k = "T"
            if k == "T":
                st, t = self.st[v], _local(y)
                if not _dev_tensor(y) or tuple(t.shape) != tuple(st.shape) or t.dtype != st.dtype \
                        or _dm_meta(y) != self.dm.get(v):
                    raise _NoGraph(v)
                src = t.contiguous()
            else:
                if not _dev_scalar(y):
                    raise _NoGraph(v)
                src = y.t.reshape(())
            if src.data_ptr() in statics and src.data_ptr() != self.st[v].data_ptr():
                src = src.clone()            # a static read by another commit pair
            pairs.append((src, self.st[v]))
        qs = q.t.reshape(())
        pairs.append((qs.clone() if qs.data_ptr() in statics else qs, self.st_q))
        return pairs

    def capture(self, ctx, b, exec_blocks, eval_pred):
        from ..ops.backend import backend
        from ..ops import kernels as K
        vars_ = ctx.vars
        cv = self._cap_vars(vars_)
        cur = torch.cuda.current_stream()
        stream = torch.cuda.Stream()
        stream.wait_stream(cur)
        seg = _Segments()
        prev_live = backend.live
        live = self.fl.data_ptr() | (1 if self.inv else 0)
        ok = False
        gc_on = gc.isenabled()
        gc.disable()
        try:
            with torch.cuda.stream(stream):
                seg.begin()
                if self.dist is not None:
                    _SEG[0] = seg
                try:
                    self.fl.copy_(self.st_q)
                    backend.set_runahead(True, live)
                    ctx.vars = cv
                    exec_blocks(ctx, b.body)
                    q = cv.get(self.pv[0]) if self.pv is not None else eval_pred(ctx, b.pred)
                    if not _dev_scalar(q):
                        raise _NoGraph("host predicate")
                    K.commit_live(self._commit_pairs(cv, q), live)
                    ok = True
                finally:
                    _SEG[0] = None
                    if seg.g is not None:
                        seg.end()
        except Exception as e:      # noqa: BLE001 - any failure: the loop stays op by op
            stats["why"] = f"capture: {type(e).__name__}: {str(e)[:80]}"
            ok = False
        finally:
            ctx.vars = vars_
            backend.set_runahead(True, prev_live)
            cur.wait_stream(stream)
            if gc_on:
                gc.enable()
        if self.dist is not None:
            # every rank replays or none does: the ranks' collective sequences must match
            ok = self.dist.allreduce_scalar(1.0 if ok else 0.0, "min") == 1.0
        if ok:
            self.seg = seg
            stats["captures"] += 1
            stats["segments"] += sum(1 for it in seg.items if it[0] == "g")
        else:
            stats["failed"] += 1
            seg.items.clear()            # destroyed here, under the capture lock
        return ok

    # ------------------------------------------------------------------ replay
    def run(self, vars_, runahead_stats, depth):
        """Replay iterations until a predicate ends the loop; then the loop state (static
        buffers, last live iteration) goes back into the variable map."""
        stats["entries"] += 1
        pending = collections.deque()
        seg = self.seg
        while True:
            t0 = time.perf_counter()
            seg.replay()
            stats["replays"] += 1
            runahead_stats["iterations"] += 1
            pending.append(S.DevScalar(self.st_q, "b").start_read())
            t1 = time.perf_counter()
            stats["t_replay"] += t1 - t0
            ended = False
            while len(pending) > depth:
                if bool(pending.popleft().value()) == self.inv:
                    ended = True
                    break
            stats["t_wait"] += time.perf_counter() - t1
            if ended:
                stats["dead"] += len(pending)
                runahead_stats["dead"] += len(pending)
                break
        # the state leaves the static buffers (the next entry overwrites them): one copy launch
        t0 = time.perf_counter()
        pairs = [(self.st[v], torch.empty_like(self.st[v])) for v in self.commit]
        self._copy(pairs)
        for v, (_, t) in zip(self.commit, pairs):
            vars_[v] = self._wrap(v, t) if self.kind[v] == "T" else S.DevScalar(t, self.vt[v])
        stats["t_exit"] += time.perf_counter() - t0


class _NoGraph(Exception):
    pass


def _usable(ctx):
    from ..ops.backend import backend
    if not (ENABLED and backend.on_gpu and backend.use_kernels):
        return False
    if ctx.dist is None:
        return True
    import torch.distributed as tdist
    return DIST and tdist.get_backend(ctx.dist.group) == "nccl"


def _depth(ctx, b):
    if ctx.dist is None:
        return DEPTH
    from .program import _runahead_depth
    return _runahead_depth(b)      # SPMD: as deep as op-by-op run-ahead (same collective count)


def try_entry(ctx, b, runahead_stats):
    """At loop entry (predicate true): replay a graph captured in an earlier entry. True when
    the loop ran to its end here."""
    gl = getattr(b, "_graph", None)
    if gl is None and not getattr(b, "_gnocache", False):
        key = getattr(b, "_gkey", None)
        gl = _BYKEY.get(key) if key is not None else None
        if gl is not None and _usable(ctx):
            b._graph = gl              # the same loop of an earlier compilation of this script
    if not isinstance(gl, GraphLoop) or not _usable(ctx) or gl.busy:
        return False
    if not gl.bind(ctx.vars):
        # another address-bound input / shape than at the capture: this loop may capture anew
        # (replacing the cached graph); twice in a row and it stays op by op
        stats["rebind_fail"] += 1
        n = getattr(b, "_gfails", 0) + 1
        b._gfails = n
        b._graph = False if n >= 2 else None
        b._gnocache = True
        return False
    gl.busy = True
    try:
        gl.run(ctx.vars, runahead_stats, _depth(ctx, b))
    finally:
        gl.busy = False
    return True


def want_capture(ctx, b, n_live):
    return (n_live >= MIN_ITERS and getattr(b, "_graph", None) is None and _usable(ctx))


def capture_and_run(ctx, b, pv, exec_blocks, eval_pred, runahead_stats):
    """After live op-by-op iterations (nothing pending): capture one iteration and replay the
    rest of the loop. True when the loop ran to its end here; False leaves it op by op."""
    with _LOCK:
        _sweep()
        t0 = time.perf_counter()
        try:
            return _capture_and_run(ctx, b, pv, exec_blocks, eval_pred, runahead_stats)
        finally:
            stats["t_capture"] += time.perf_counter() - t0


def _capture_and_run(ctx, b, pv, exec_blocks, eval_pred, runahead_stats):
    gl = GraphLoop(b, pv, ctx.dist)
    try:
        ok = gl.classify(b, ctx.vars) and gl.bind(ctx.vars)
    except Exception as e:      # noqa: BLE001
        stats["why"] = f"bind: {type(e).__name__}: {str(e)[:80]}"
        ok = False
    if ctx.dist is not None and not ok:
        # the capture below holds a collective agreement; a rank that cannot even bind joins it
        ctx.dist.allreduce_scalar(0.0, "min")
    elif ok:
        ok = gl.capture(ctx, b, exec_blocks, eval_pred)
    if not ok:
        b._graph = False
        return False
    b._graph = gl
    key = getattr(b, "_gkey", None)
    if key is not None and (key in _BYKEY or len(_BYKEY) < _BYKEY_MAX):
        if key in _BYKEY:
            _RETIRED.append(_BYKEY[key])        # blocks may still hold it: never freed mid-capture
        _BYKEY[key] = gl                        # kept for the process
    else:
        _ALL.append((weakref.ref(b), gl))
    gl.busy = True
    try:
        gl.run(ctx.vars, runahead_stats, _depth(ctx, b))
    finally:
        gl.busy = False
    return True
