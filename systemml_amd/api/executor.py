"""Script executor: parse → validate/translate → rewrite → instruction generation →
execute (reference: api/ScriptExecutorUtils.java, api/mlcontext/ScriptExecutor.java,
api/DMLScript.java:execute).

Used by the MLContext, JMLC, CLI and bench front ends."""
from __future__ import annotations

import os
import sys
import time

import numpy as np
import torch

from ..conf import DMLConfig, get_default_config
from ..parser.dml_parser import parse_dml
from ..compiler.translator import Translator
from ..compiler.lops import compile_program
from ..compiler.hops import explain_dag
from ..compiler.blocks import BasicBlock, IfBlock, WhileBlock, ForBlock
from ..runtime.instructions import make_impl
from ..runtime.program import ExecutionContext, exec_blocks
from ..runtime.data import FrameBlock, ListObject
from ..ops.backend import backend, place, maybe_bf16
from ..utils.stats import Statistics


def parse(source, pydml=False, filename=""):
    if pydml:
        from ..parser.pydml_parser import parse_pydml
        return parse_pydml(source, filename=filename)
    return parse_dml(source, filename=filename)


class CompiledScript:
    def __init__(self, cp, config, inputs, outputs, t_parse, t_compile):
        self.cp = cp
        self.config = config
        self.inputs = inputs
        self.outputs = outputs
        self.t_parse = t_parse
        self.t_compile = t_compile


_REC_LIMIT = 50000


_STACK_BYTES = 1 << 29       # 512 MiB: room for _REC_LIMIT Python frames on CPython 3.10's C stack


def _on_big_stack(fn):
    """Run fn in a thread with a stack sized for the raised recursion limit (a deep DAG on the
    8 MiB main-thread stack would overflow it -- a segfault, not a RecursionError)."""
    import threading
    box = {}

    def run():
        try:
            box["r"] = fn()
        except BaseException as e:     # re-raised in the caller
            box["e"] = e
    old = threading.stack_size()
    threading.stack_size(_STACK_BYTES)
    try:
        t = threading.Thread(target=run, name="sysml-compile")
        t.start()
    finally:
        threading.stack_size(old)
    t.join()
    if "e" in box:
        raise box["e"]
    return box["r"]


def compile_script(source, args=None, inputs=(), outputs=(), config=None, pydml=False, filename="",
                   base_dir=None):
    """Parse, translate and plan a DML / PyDML script (on a large-stack thread: inlined layer
    libraries make one basic block of a whole training step, thousands of HOPs deep, and the
    recursive DAG passes need more than Python's default 1000 frames)."""
    if sys.getrecursionlimit() < _REC_LIMIT:
        sys.setrecursionlimit(_REC_LIMIT)
    return _on_big_stack(lambda: _compile_script(source, args, inputs, outputs, config, pydml, filename, base_dir))


def _compile_script(source, args, inputs, outputs, config, pydml, filename, base_dir):
    config = config or get_default_config()
    t0 = time.perf_counter()
    prog = parse(source, pydml=pydml, filename=filename)
    t1 = time.perf_counter()
    tr = Translator(args or {}, config, base_dir=base_dir or (os.path.dirname(filename) if filename else None))
    input_types = {}
    if isinstance(inputs, dict):
        input_types = {k: value_dt(v) for k, v in inputs.items()}
    cp = tr.compile(prog, inputs=list(inputs), outputs=outputs, input_types=input_types)
    from ..compiler import cost
    shapes = inputs if isinstance(inputs, dict) else None
    if getattr(config, "rewrites", True):
        cost.reorder_chains(cp, shapes)          # size-dependent mm-chain order (needs raw DAGs)
    compile_program(cp, make_impl, config)
    cost.annotate(cp, shapes, config)            # dims, memory estimates, exec types
    t2 = time.perf_counter()
    cs = CompiledScript(cp, config, set(inputs), list(outputs), t1 - t0, t2 - t1)
    cs.source = source
    cs.compile_args = dict(args=args, inputs=inputs, outputs=outputs, pydml=pydml, filename=filename,
                           base_dir=base_dir)
    _tag_loops(cp, source, args, inputs, outputs, config, pydml)
    return cs


def _tag_loops(cp, source, args, inputs, outputs, config, pydml):
    """Key every while loop by what determines its compiled body -- script text, arguments,
    input metadata, configuration and the loop's ordinal: a recompilation of the same script
    (the bench compiles every step) finds the HIP graph its loop was captured into
    (runtime/graphloop.py) instead of capturing again."""
    import hashlib
    from ..compiler.blocks import BasicBlock, WhileBlock
    meta = []
    if isinstance(inputs, dict):
        for k in sorted(inputs):
            v = inputs[k]
            meta.append((k, type(v).__name__, tuple(getattr(v, "shape", ())), str(getattr(v, "dtype", ""))))
    h = hashlib.sha1(repr((source, sorted((args or {}).items(), key=lambda kv: kv[0]), meta, list(outputs),
                           repr(config), pydml)).encode()).hexdigest()
    n = [0]

    def walk(blocks):
        for b in blocks or ():
            if isinstance(b, BasicBlock):
                continue
            if isinstance(b, WhileBlock):
                # + the body's variable names: compiler temporaries (_licm*) are numbered per
                # compilation, and the graph binds them by name
                from ..compiler.translator import _all_writes
                names = (tuple(sorted(getattr(b, "body_live_in", ()) or ())), tuple(sorted(_all_writes(b.body))),
                         tuple(sorted(b.pred.reads)))
                b._gkey = (h, n[0], names)
                n[0] += 1
            for attr in ("body", "then_blocks", "else_blocks"):
                walk(getattr(b, attr, None))
    walk(cp.blocks)
    for k in sorted(cp.functions, key=repr):
        walk(getattr(cp.functions[k], "body", None))


def value_dt(v):
    if isinstance(v, (bool, int, float, str, np.generic)):
        return "S"
    if isinstance(v, FrameBlock):
        return "F"
    if isinstance(v, ListObject):
        return "L"
    try:
        import pandas as pd
        if isinstance(v, pd.DataFrame) and not all(np.issubdtype(t, np.number) for t in v.dtypes):
            return "F"
    except ImportError:
        pass
    return "M"


def convert_input(v, dist=None, config=None):
    """Python/numpy/torch/pandas objects → DML runtime values."""
    if isinstance(v, (bool, int, float, str)):
        return v
    if isinstance(v, np.generic):
        return v.item()
    if isinstance(v, (FrameBlock, ListObject)):
        return v
    from ..parallel import dist as D
    if isinstance(v, D.DistMatrix):
        return v
    try:
        import pandas as pd
        if isinstance(v, pd.DataFrame):
            if all(np.issubdtype(t, np.number) for t in v.dtypes):
                v = v.to_numpy(dtype=np.float64)
            else:
                return FrameBlock([v[c].tolist() for c in v.columns],
                                  ["DOUBLE" if np.issubdtype(t, np.number) else "STRING" for t in v.dtypes],
                                  [str(c) for c in v.columns])
        elif isinstance(v, pd.Series):
            v = v.to_numpy(dtype=np.float64).reshape(-1, 1)
    except ImportError:
        pass
    if hasattr(v, "toarray") and not isinstance(v, np.ndarray):   # scipy sparse
        from ..ops import sparse as SP
        coo = v.tocoo()
        if dist is None and SP.want_sparse(coo.shape[0], coo.shape[1], coo.nnz):
            return SP.from_ijv(coo.row, coo.col, coo.data, coo.shape[0], coo.shape[1], backend.dtype,
                               backend.device)
        v = v.toarray()
    if isinstance(v, (list, tuple)) and v and all(isinstance(x, str) for x in v):
        # lines of CSV text: the no-Spark form of the reference's RDD<String> matrix input
        # (MLContextConversionUtil.javaRDDStringCSVToMatrixObject)
        v = np.asarray([[float(t) for t in ln.split(",")] for ln in v if ln.strip()], dtype=np.float64)
    if isinstance(v, (list, tuple)):
        v = np.asarray(v, dtype=np.float64)
    if isinstance(v, np.ndarray):
        if v.ndim == 1:
            v = v.reshape(-1, 1)
        t = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float64))
    elif isinstance(v, torch.Tensor):
        t = v
        if t.dim() == 1:
            t = t.reshape(-1, 1)
        if t.layout in (torch.sparse_csr, torch.sparse_coo):
            from ..ops import sparse as SP
            t = SP.canonical(t)
    else:
        raise TypeError(f"unsupported input type {type(v).__name__}")
    if dist is not None and config is not None and t.shape[0] >= config.dist_min_rows:
        return D.scatter_rows_from_global(dist, t)
    if t.dtype == torch.bfloat16:
        return t.to(backend.device)
    from ..io.readers import maybe_compress
    return maybe_compress(maybe_bf16(place(t)), config)


def execute(cs: CompiledScript, inputs=None, out=None, stats=None, dist=None):
    config = cs.config
    backend.configure(config)
    if dist is None:
        from ..parallel import dist as D
        dist = D.get_context()
    ctx = ExecutionContext(cs.cp, config, stats=stats, out=out, dist=dist)
    for k, v in (inputs or {}).items():
        ctx.vars[k] = convert_input(v, dist, config)
    if config.explain:
        ctx.print(explain(cs.cp, config.explain))
    t0 = time.perf_counter()
    try:
        exec_blocks(ctx, cs.cp.blocks)
    finally:
        if stats is not None:
            stats.t_exec += time.perf_counter() - t0
            stats.t_parse += cs.t_parse
            stats.t_compile += cs.t_compile
            if ctx.pool is not None:
                for k_, v_ in ctx.pool.stats.items():
                    if isinstance(v_, int) and v_:
                        stats.counters["bufferpool." + k_] = v_
            for k_, v_ in (getattr(cs.cp, "exec_types", None) or {}).items():
                stats.counters[f"compiled exec type {k_}"] = v_
            for k_, v_ in (getattr(cs.cp, "licm_stats", None) or {}).items():
                stats.counters[f"rewrite {k_}"] = v_
            for k_, v_ in (getattr(cs.cp, "rewrite_stats", None) or {}).items():
                stats.counters[f"rewrite {k_}"] = stats.counters.get(f"rewrite {k_}", 0) + v_
            for k_, v_ in (getattr(cs.cp, "chain_stats", None) or {}).items():
                stats.counters[f"mm-chain {k_}"] = v_
    from ..runtime.bufferpool import Evicted
    from ..runtime import scalars as S_
    res = {}
    for k in cs.outputs:
        v = ctx.vars.get(k)
        if isinstance(v, Evicted):
            v = ctx.pool.restore(ctx.vars, k, v)
        res[k] = S_.materialize(v)
    return res, ctx


def run(source, args=None, inputs=None, outputs=(), config=None, pydml=False, filename="", out=None,
        stats=None):
    inputs = inputs or {}
    cs = compile_script(source, args, inputs=inputs, outputs=outputs, config=config, pydml=pydml,
                        filename=filename)
    res, _ = execute(cs, inputs, out=out, stats=stats)
    return res


# ----------------------------------------------------------------------------
def explain(cp, level="hops"):
    lines = ["# EXPLAIN (" + level + "):"]

    def blocks(bl, ind):
        for b in bl:
            if isinstance(b, BasicBlock):
                lines.append(f"{ind}GENERIC (lines {b.pos.line if b.pos else '?'}) [live_out={sorted(b.live_out or [])}]")
                if level.startswith("runtime"):
                    for ins in b.instrs or []:
                        lines.append(f"{ind}  {ins.opcode} {list(ins.ins)} -> {ins.out}")
                else:
                    roots = list(b.roots) + [h for k, h in b.env_out.items()]
                    lines.append(explain_dag(roots, ind + "  "))
            elif isinstance(b, IfBlock):
                lines.append(f"{ind}IF")
                blocks(b.then_blocks, ind + "  ")
                lines.append(f"{ind}ELSE")
                blocks(b.else_blocks, ind + "  ")
            elif isinstance(b, WhileBlock):
                lines.append(f"{ind}WHILE")
                blocks(b.body, ind + "  ")
            elif isinstance(b, ForBlock):
                lines.append(f"{ind}{'PARFOR' if b.parfor else 'FOR'} {b.var}")
                blocks(b.body, ind + "  ")

    for key, fb in cp.functions.items():
        if fb.body is not None:
            lines.append(f"FUNCTION {key[0]}::{key[1]}")
            blocks(fb.body, "  ")
    lines.append("MAIN PROGRAM")
    blocks(cp.blocks, "  ")
    return "\n".join(lines)
