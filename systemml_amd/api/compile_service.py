"""Out-of-process compilation (a pipelined driver's compiler service).

The compiler (parse -> HOP DAGs -> rewrites -> size / cost annotation -> instruction lists) is
pure Python; run in a thread next to the executor it competes for the interpreter lock, and on
a fast multi-GPU step its ~60 ms per script pair exceed the device time.  A `CompileService`
runs the compiler in a separate process (started with the `spawn` method, it never touches the
GPU): requests carry the script text, arguments, the shapes / kinds of the inputs and the
configuration; the worker compiles against shape-only stand-ins (`meta` tensors), strips the
instruction closures and returns the pickled plan.  The driver re-binds every instruction's
implementation (`make_impl`, a few microseconds each) and renumbers the HOPs into its own id
space, so dynamic recompilation in the driver cannot collide with ids the worker issued.

Reference analogue: none -- the reference compiles inside the JVM that executes; this is the
MI355X driver's way of keeping the compiler off the executor's critical path.
"""
from __future__ import annotations

import multiprocessing as mp
import pickle
import sys
import threading

_REC_LIMIT = 50000


# ----------------------------------------------------------------------------
# plan (de)hydration
# ----------------------------------------------------------------------------
def _instr_lists(blocks):
    from ..compiler.blocks import BasicBlock, IfBlock, WhileBlock, ForBlock
    for b in blocks or ():
        if isinstance(b, BasicBlock):
            if b.instrs is not None:
                yield b.instrs
        elif isinstance(b, IfBlock):
            if b.pred.instrs is not None:
                yield b.pred.instrs
            yield from _instr_lists(b.then_blocks)
            yield from _instr_lists(b.else_blocks)
        elif isinstance(b, WhileBlock):
            if b.pred.instrs is not None:
                yield b.pred.instrs
            yield from _instr_lists(b.body)
        elif isinstance(b, ForBlock):
            for p in (b.start, b.end, b.incr):
                if p is not None and p.instrs is not None:
                    yield p.instrs
            yield from _instr_lists(b.body)


def _all_instr_lists(cp):
    yield from _instr_lists(cp.blocks)
    for fb in cp.functions.values():
        yield from _instr_lists(fb.body)


def dehydrate(cs) -> bytes:
    """Pickled plan without the instruction closures."""
    for lst in _all_instr_lists(cs.cp):
        for ins in lst:
            ins.fn = None
    return pickle.dumps(cs, protocol=pickle.HIGHEST_PROTOCOL)


def hydrate(blob: bytes, inputs=None):
    """Unpickle a plan, renumber its HOPs into this process's id space and re-bind every
    instruction's implementation."""
    from ..compiler import hops as H
    from ..runtime.instructions import make_impl
    old = sys.getrecursionlimit()
    sys.setrecursionlimit(max(old, _REC_LIMIT))
    try:
        cs = pickle.loads(blob)
    finally:
        sys.setrecursionlimit(old)
    seen = set()

    def renumber(h):
        stack = [h]
        while stack:
            x = stack.pop()
            if id(x) in seen:
                continue
            seen.add(id(x))
            x.id = next(H._ids)
            stack.extend(x.inputs)
            d = x.p.get("licm_def") if isinstance(x.p, dict) else None
            if d is not None:
                stack.append(d)

    for lst in _all_instr_lists(cs.cp):
        for ins in lst:
            renumber(ins.hop)
    _renumber_blocks(cs.cp, renumber)
    for lst in _all_instr_lists(cs.cp):
        for ins in lst:
            ins.fn, _ = make_impl(ins.hop)
    if inputs is not None:
        cs.compile_args = dict(cs.compile_args, inputs=inputs)
    return cs


def _renumber_blocks(cp, renumber):
    from ..compiler.blocks import BasicBlock, IfBlock, WhileBlock, ForBlock

    def blocks(bl):
        for b in bl or ():
            if isinstance(b, BasicBlock):
                for h in list(b.roots or ()) + list((b.env_out or {}).values()):
                    renumber(h)
                raw = getattr(b, "_raw", None)
                if raw is not None:
                    for h in list(raw[0]) + list(raw[1].values()):
                        renumber(h)
            elif isinstance(b, IfBlock):
                renumber(b.pred.root)
                blocks(b.then_blocks)
                blocks(b.else_blocks)
            elif isinstance(b, WhileBlock):
                renumber(b.pred.root)
                blocks(b.body)
            elif isinstance(b, ForBlock):
                for p in (b.start, b.end, b.incr):
                    if p is not None:
                        renumber(p.root)
                blocks(b.body)

    blocks(cp.blocks)
    for fb in cp.functions.values():
        blocks(fb.body)


# ----------------------------------------------------------------------------
# worker
# ----------------------------------------------------------------------------
def input_spec(v):
    """Shape-only description of a compile-time input (what the compiler reads of it)."""
    shape = getattr(v, "shape", None)
    if isinstance(v, (bool, int, float, str)):
        return ("S", v)
    if shape is not None and len(shape) == 2:
        return ("M", (int(shape[0]), int(shape[1])))
    return ("V", v)


def _stand_in(spec):
    import torch
    kind, v = spec
    if kind == "M":
        return torch.empty(v, device="meta")
    return v


def _worker(conn):
    import gc
    sys.setrecursionlimit(_REC_LIMIT)
    from . import executor as EX
    first = True
    while True:
        msg = conn.recv()
        if msg is None:
            return
        seq, src, args, specs, outputs, config, world, kw = msg
        try:
            import time
            t0 = time.perf_counter()
            config._world = world
            inputs = {k: _stand_in(s) for k, s in specs.items()}
            cs = EX.compile_script(src, args, inputs=inputs, outputs=outputs, config=config, **kw)
            blob = dehydrate(cs)
            conn.send((seq, "ok", (blob, time.perf_counter() - t0)))
            if first:
                # the compiler's modules and caches are loaded now: freeze them out of the cyclic
                # collector so later collections only scan a compilation's own garbage
                first = False
                gc.collect()
                gc.freeze()
        except BaseException as e:  # noqa: BLE001 - reported to the driver
            conn.send((seq, "err", f"{type(e).__name__}: {e}"))


class _Pending:
    def __init__(self, svc, inputs, seq):
        self.svc = svc
        self.seq = seq
        self.inputs = inputs
        self._value = None
        self._done = False
        self.times = None      # (worker compile s, driver wait s, driver hydrate s)

    def result(self):
        if not self._done:
            import time
            t0 = time.perf_counter()
            status, payload = self.svc.reply(self.seq)
            t1 = time.perf_counter()
            if status != "ok":
                raise RuntimeError(f"compile service: {payload}")
            blob, tc = payload
            self._value = hydrate(blob, self.inputs)
            self.times = (tc, t1 - t0, time.perf_counter() - t1)
            self._done = True
        return self._value


class CompileService:
    """One compiler process; requests are answered in order and each reply carries its
    request's sequence number, so results may be claimed in any order."""

    def __init__(self):
        ctx = mp.get_context("spawn")
        self.conn, child = ctx.Pipe()
        self.proc = ctx.Process(target=_worker, args=(child,), daemon=True)
        self.proc.start()
        child.close()
        self.lock = threading.Lock()
        self.seq = 0
        self.replies = {}       # seq -> (status, payload) received while waiting for another

    def submit(self, source, args, inputs, outputs, config, world=1, **kw):
        specs = {k: input_spec(v) for k, v in (inputs or {}).items()}
        with self.lock:
            self.seq += 1
            seq = self.seq
            self.conn.send((seq, source, args, specs, list(outputs), config, world, kw))
        return _Pending(self, inputs, seq)

    def reply(self, seq):
        with self.lock:
            while seq not in self.replies:
                s, status, payload = self.conn.recv()
                self.replies[s] = (status, payload)
            return self.replies.pop(seq)

    def close(self):
        try:
            self.conn.send(None)
        except (BrokenPipeError, OSError):
            pass
        self.proc.join(timeout=10)
        if self.proc.is_alive():
            self.proc.kill()
