"""AST → statement blocks → HOP DAGs (reference: parser/DMLTranslator.java,
parser/StatementBlock.java, parser/LiveVariableAnalysis.java,
hops/ipa/IPAPassPropagateReplaceLiterals.java,
hops/rewrite/RewriteRemoveUnnecessaryBranches.java,
hops/rewrite/RewriteMergeBlockSequence.java).

Responsibilities:
  * resolve `source(...) as ns` imports into a namespaced function table,
  * substitute command-line parameters ($name / ifdef),
  * split statements into basic blocks at control flow,
  * propagate scalar constants across blocks and remove constant branches
    (the spliced branch merges into the surrounding basic block so that
    operator fusion sees a single DAG),
  * build a HOP DAG per basic block (with on-the-fly constant folding and
    hash-consing CSE),
  * live-variable analysis (transient writes only for live-out variables,
    rmvar for dead ones).
"""
from __future__ import annotations

import os
import math

from ..parser import ast as A
from ..parser.errors import LanguageError, DMLRuntimeError
from ..parser.dml_parser import parse_dml_file
from ..runtime import scalars as S
from . import hops as H
from .hops import Hop, lit
from .blocks import BasicBlock, IfBlock, WhileBlock, ForBlock, FunctionBlock, Predicate, CompiledProgram

DEFAULT_NS = ".defaultNS"

BUILTIN_CONSTANTS = {"NaN": float("nan"), "Inf": float("inf"), "pi": math.pi, "INF": float("inf"),
                     "NAN": float("nan"), "PI": math.pi}

UNARY_MATH = {"abs", "exp", "sqrt", "round", "floor", "ceil", "sign", "sin", "cos", "tan", "asin",
              "acos", "atan", "sinh", "cosh", "tanh", "sigmoid"}
CUMAGG = {"cumsum", "cumprod", "cummin", "cummax"}
FULL_AGG = {"sum": "sum", "prod": "prod", "mean": "mean", "avg": "mean", "var": "var", "sd": "sd",
            "trace": "trace"}
ROWCOL_AGG = {
    "rowSums": ("sum", "row"), "colSums": ("sum", "col"),
    "rowMeans": ("mean", "row"), "colMeans": ("mean", "col"),
    "rowMaxs": ("max", "row"), "colMaxs": ("max", "col"),
    "rowMins": ("min", "row"), "colMins": ("min", "col"),
    "rowVars": ("var", "row"), "colVars": ("var", "col"),
    "rowSds": ("sd", "row"), "colSds": ("sd", "col"),
    "rowProds": ("prod", "row"), "colProds": ("prod", "col"),
    "rowIndexMax": ("imax", "row"), "rowIndexMin": ("imin", "row"),
}
CASTS = {"as.scalar": "cast_scalar", "castAsScalar": "cast_scalar", "as.matrix": "cast_matrix",
         "as.double": "cast_double", "as.integer": "cast_int", "as.logical": "cast_bool",
         "as.frame": "cast_frame", "as.list": "cast_list"}
BINARY_FNS = {"xor": "xor", "bitwAnd": "bitwAnd", "bitwOr": "bitwOr", "bitwXor": "bitwXor",
              "bitwShiftL": "bitwShiftL", "bitwShiftR": "bitwShiftR"}
SCALAR_FOLD_UNARY = UNARY_MATH | {"neg", "not", "cast_double", "cast_int", "cast_bool", "log"}


class FileCtx:
    """Per-source-file namespace context."""

    def __init__(self, key, path, imports):
        self.key = key            # namespace key for this file's functions
        self.path = path
        self.imports = imports    # alias -> namespace key


class Translator:
    def __init__(self, args=None, config=None, base_dir=None):
        self.args = dict(args or {})
        self.config = config
        self.base_dir = base_dir or os.getcwd()
        # validation (reference StatementBlock.validate / Expression.raiseValidateError): reads
        # of never-defined variables and known-dimension mismatches are errors in unconditional
        # code, warnings inside if / loop bodies
        self.cond_depth = 0
        self.warnings = []
        self.inputs = set()
        self.functions = {}       # (nskey, name) -> FunctionBlock
        self.func_defs = {}       # (nskey, name) -> (FunctionDef, FileCtx)
        self.loaded_files = {}    # abs path -> FileCtx

    def validate_error(self, msg):
        """reference Statement.raiseValidateError: error if unconditional, else a warning."""
        if self.cond_depth > 0:
            if msg not in self.warnings:
                self.warnings.append(msg)
            return
        raise LanguageError(msg)

    # ------------------------------------------------------------------ imports
    def _register_file(self, prog: A.Program, key, path):
        ctx = FileCtx(key, path, {})
        base = os.path.dirname(path) if path else self.base_dir
        for st in prog.statements:
            if isinstance(st, A.SetWd):
                base = st.path if os.path.isabs(st.path) else os.path.join(base, st.path)
            if isinstance(st, A.Import):
                ipath = st.path
                cand = [ipath if os.path.isabs(ipath) else os.path.join(base, ipath),
                        os.path.join(self.base_dir, ipath), ipath]
                cand += _package_script_candidates(ipath)
                full = next((c for c in cand if os.path.exists(c)), None)
                if full is None:
                    raise LanguageError(f"{st.pos}: cannot find sourced file '{ipath}'")
                full = os.path.abspath(full)
                if full not in self.loaded_files:
                    sub = parse_dml_file(full) if not full.endswith(".pydml") else _parse_pydml_file(full)
                    self.loaded_files[full] = None   # guard recursion
                    self.loaded_files[full] = self._register_file(sub, full, full)
                ctx.imports[st.namespace] = full
        for name, fd in prog.functions.items():
            self.func_defs[(key, name)] = (fd, ctx)
        return ctx

    # ------------------------------------------------------------------ compile
    def compile(self, prog: A.Program, inputs=(), outputs=(), input_types=None):
        from .parfor_deps import check_program
        check_program(prog)          # parfor loop dependency analysis (ParForStatementBlock.validate)
        main_ctx = self._register_file(prog, DEFAULT_NS, prog.source_path)
        self.inputs = set(inputs)
        self.input_types = dict(input_types or {})
        self.outputs = set(outputs)
        self.main_ctx = main_ctx
        # compile all functions (bodies built lazily with empty const env)
        for (key, name), (fd, ctx) in list(self.func_defs.items()):
            self.functions[(key, name)] = FunctionBlock(name, key, fd.inputs, fd.outputs, None,
                                                        external=fd.external, ext_params=fd.ext_params,
                                                        pos=fd.pos)
        for (key, name), (fd, ctx) in list(self.func_defs.items()):
            fb = self.functions[(key, name)]
            if not fd.external:
                consts = {}
                types = {p.name: p.dtype[0] if p.dtype in ("MATRIX", "SCALAR", "FRAME", "LIST") else "U"
                         for p in fd.inputs}
                fb.body = self.build_stmts(fd.body, ctx, consts, params=fd.inputs, types=types)
                for p in fd.inputs:
                    if p.default is not None:
                        bb = _BBuilder(self, ctx, {})
                        h = bb.expr(p.default)
                        fb.default_preds[p.name] = Predicate(h, bb.reads)
        blocks = self.build_stmts(prog.statements, main_ctx, {}, types=dict(self.input_types))
        cp = CompiledProgram(blocks, self.functions, prog.source_path)
        if self.config is None or getattr(self.config, "rewrites", True):
            from . import ipa
            self._specialise_functions(cp)
            ipa.run(cp, self.config)                # inter-procedural analysis (inlining, ...)
            from .forvec import run as forvec
            fv = forvec(cp, self.config)           # for-loop vectorization (whole-range operations)
            from .splitdag import run as splitdag
            fv.update(splitdag(cp, self.config))   # cut blocks after data-dependent operators
            from .loops import hoist_program
            cp.licm_stats = hoist_program(cp)      # before liveness: adds blocks / variables
            cp.licm_stats.update(fv)
            from .loops import mark_program
            cp.licm_stats.update(mark_program(cp))
            from .speculate import run as speculate
            cp.licm_stats.update(speculate(cp, self.config))
        # liveness
        for fb in self.functions.values():
            if fb.body is not None:
                liveness(fb.body, set(o.name for o in fb.outputs))
        live_in = liveness(blocks, set(outputs) if outputs else None)
        if self.config is None or getattr(self.config, "rewrites", True):
            from .ifconv import run as ifconv
            st = ifconv(cp, self.config)       # needs liveness; changes the block structure
            if st:
                cp.licm_stats.update(st)
                for fb in self.functions.values():
                    if fb.body is not None:
                        liveness(fb.body, set(o.name for o in fb.outputs))
                live_in = liveness(cp.blocks, set(outputs) if outputs else None)
        cp.inputs = live_in
        undefined = live_in - set(inputs)
        if undefined and self.config is not None and getattr(self.config, "strict_undefined", True):
            pass  # reported at runtime with position info (variables may be defined conditionally)
        cp.outputs = set(outputs)
        return cp

    def _specialise_functions(self, cp, rounds=3):
        """Rebuild the body of every function whose scalar parameters are the same literal at
        every call site with those literals as constants (reference
        IPAPassPropagateReplaceLiterals + RewriteRemoveUnnecessaryBranches +
        RewriteMergeBlockSequence): constant branches such as the nn layers'
        `if (mode == "train")` disappear at translation and the remaining statements merge into
        one basic block, so operator fusion sees across them.  Repeated while a rebuilt body
        passes new literals on to its callees."""
        from . import ipa
        applied = {}
        for _ in range(rounds):
            changed = False
            for k, consts in ipa.literal_params(cp).items():
                if k not in self.func_defs or applied.get(k) == consts:
                    continue
                fd, ctx = self.func_defs[k]
                fb = cp.functions[k]
                types = {p.name: p.dtype[0] if p.dtype in ("MATRIX", "SCALAR", "FRAME", "LIST") else "U"
                         for p in fd.inputs}
                fb.body = self.build_stmts(fd.body, ctx, dict(consts), params=fd.inputs, types=types)
                applied[k] = consts
                changed = True
            if not changed:
                break
        cp.specialised = len(applied)

    # ------------------------------------------------------------------ blocks
    def build_stmts(self, stmts, ctx, consts, params=None, types=None):
        """Returns list of blocks. `consts` / `types` are updated in place with the scalar
        constants and data types (M/S/F/L/U) known at exit."""
        blocks = []
        if types is None:
            types = {}
        cur = _BBuilder(self, ctx, consts, types)

        def flush():
            nonlocal cur
            if cur.has_content():
                bb = cur.finish()
                blocks.append(bb)
                consts.clear()
                consts.update(cur.out_consts())
                types.update(cur.out_types())
            cur = _BBuilder(self, ctx, consts, types)

        def process(lst):
            nonlocal cur
            for st in lst:
                if isinstance(st, (A.Assign, A.MultiAssign, A.ExprStmt)):
                    cur.add(st)
                    if isinstance(st, A.Assign) and _reads_unknown_size(st.value):
                        # reference RewriteSplitDagUnknownCSVRead: end the block after a read
                        # of unknown size so the operators using it are recompiled (exec types,
                        # mm-chain order) with the actual dimensions
                        flush()
                elif isinstance(st, (A.Import, A.SetWd)):
                    continue
                elif isinstance(st, A.If):
                    ph = cur.try_const(st.pred)
                    if ph is not None:
                        process(st.then_body if S.as_bool(ph) else st.else_body)
                        continue
                    flush()
                    pb = _BBuilder(self, ctx, consts, types)
                    pred = Predicate(pb.expr(st.pred), pb.reads)
                    c1, c2 = dict(consts), dict(consts)
                    t1, t2 = dict(types), dict(types)
                    self.cond_depth += 1
                    try:
                        tb = self.build_stmts(st.then_body, ctx, c1, types=t1)
                        eb = self.build_stmts(st.else_body, ctx, c2, types=t2)
                    finally:
                        self.cond_depth -= 1
                    blocks.append(IfBlock(pred, tb, eb, pos=st.pos))
                    merged = {k: v for k, v in c1.items() if k in c2 and _same(c2[k], v)}
                    consts.clear()
                    consts.update(merged)
                    for k in set(t1) | set(t2):
                        types[k] = t1.get(k, "U") if t1.get(k, "U") == t2.get(k, "U") else "U"
                    cur = _BBuilder(self, ctx, consts, types)
                elif isinstance(st, A.While):
                    flush()
                    assigned = assigned_vars(st.body)
                    for v in assigned:
                        consts.pop(v, None)
                    self._loop_types(st.body, ctx, consts, types)
                    pb = _BBuilder(self, ctx, consts, types)
                    pred = Predicate(pb.expr(st.pred), pb.reads)
                    self.cond_depth += 1
                    try:
                        body = self.build_stmts(st.body, ctx, dict(consts), types=dict(types))
                    finally:
                        self.cond_depth -= 1
                    blocks.append(WhileBlock(pred, body, pos=st.pos))
                    cur = _BBuilder(self, ctx, consts, types)
                elif isinstance(st, A.For):
                    flush()
                    assigned = assigned_vars(st.body) | {st.var}
                    pb = _BBuilder(self, ctx, consts, types)
                    p_from = Predicate(pb.expr(st.start), pb.reads)
                    pb2 = _BBuilder(self, ctx, consts, types)
                    p_to = Predicate(pb2.expr(st.end), pb2.reads)
                    p_incr = None
                    if st.incr is not None:
                        pb3 = _BBuilder(self, ctx, consts, types)
                        p_incr = Predicate(pb3.expr(st.incr), pb3.reads)
                    params = {}
                    for nm, pr in (("from", p_from), ("to", p_to), ("increment", p_incr)):
                        if pr is not None and pr.root.dt == "M":
                            raise LanguageError(f"{st.pos}: {'parfor' if st.parfor else 'for'} loop {nm} "
                                                f"expression must be a scalar, got a matrix")
                    for k, v in st.params.items():
                        pbk = _BBuilder(self, ctx, consts, types)
                        hv = pbk.expr(v)
                        params[k] = hv.p.get("v") if hv.op == "lit" else None
                        if hv.op == "tread" or (hv.op != "lit" and isinstance(v, A.Ident)):
                            params[k] = v.name if isinstance(v, A.Ident) else None
                    for v in assigned:
                        consts.pop(v, None)
                    types[st.var] = "S"
                    self._loop_types(st.body, ctx, consts, types)
                    self.cond_depth += 1
                    try:
                        body = self.build_stmts(st.body, ctx, dict(consts), types=dict(types))
                    finally:
                        self.cond_depth -= 1
                    fb = ForBlock(st.var, p_from, p_to, p_incr, body, parfor=st.parfor, params=params, pos=st.pos)
                    if st.parfor:
                        from .parfor_deps import loop_accumulators
                        fb.accumulators = loop_accumulators(st, {v for v, d in types.items() if d == "S"})
                    blocks.append(fb)
                    cur = _BBuilder(self, ctx, consts, types)
                else:
                    raise LanguageError(f"unsupported statement {type(st).__name__}")

        process(stmts)
        flush()
        return blocks

    def _loop_types(self, body, ctx, consts, types):
        """Fixpoint of data types over a loop body (types assigned in the body that differ
        from the entry types become unknown)."""
        t = dict(types)
        self.cond_depth += 1
        try:
            self.build_stmts(body, ctx, dict(consts), types=t)
        finally:
            self.cond_depth -= 1
        for k, v in t.items():
            if k in types and types[k] != v:
                types[k] = "U"
            elif k not in types:
                types[k] = v

    def resolve_function(self, ctx: FileCtx, ns, name):
        if ns is not None:
            key = ctx.imports.get(ns)
            if key is None:
                raise LanguageError(f"unknown namespace '{ns}'")
            fb = self.functions.get((key, name))
            if fb is None:
                raise LanguageError(f"function '{ns}::{name}' not found")
            return fb
        return self.functions.get((ctx.key, name))


def _package_script_candidates(path):
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    scripts = os.path.join(here, "scripts")
    p = path
    out = [os.path.join(scripts, p)]
    if p.startswith("scripts/"):
        out.append(os.path.join(here, p))
    # library directories of the shipped scripts (e.g. "scalable_linalg/...", "utils/...")
    out += [os.path.join(scripts, sub, p) for sub in ("staging", "algorithms", "utils")]
    return out


def _parse_pydml_file(path):
    from ..parser.pydml_parser import parse_pydml_file
    return parse_pydml_file(path)


def _same(a, b):
    if isinstance(a, float) and isinstance(b, float) and a != a and b != b:
        return True
    return type(a) == type(b) and a == b


def assigned_vars(stmts):
    out = set()
    for st in stmts:
        if isinstance(st, A.Assign):
            t = st.target
            out.add(t.name)
        elif isinstance(st, A.MultiAssign):
            for t in st.targets:
                out.add(t.name)
        elif isinstance(st, A.If):
            out |= assigned_vars(st.then_body) | assigned_vars(st.else_body)
        elif isinstance(st, A.While):
            out |= assigned_vars(st.body)
        elif isinstance(st, A.For):
            out |= assigned_vars(st.body) | {st.var}
    return out


# ============================================================================
# Basic block builder: statements -> HOP DAG
# ============================================================================
class _BBuilder:
    def __init__(self, tr: Translator, ctx: FileCtx, consts: dict, types=None):
        self.tr = tr
        self.ctx = ctx
        self.consts = dict(consts)
        self.types = dict(types or {})
        self.env = {}            # var -> hop
        self.treads = {}         # var -> tread hop
        self.reads = set()
        self.cse = {}
        self.roots = []          # ordered sink hops (incl. fcalls)
        self.stmt_count = 0
        self.pos = None

    def has_content(self):
        return self.stmt_count > 0

    # -- CSE-aware hop creation --------------------------------------------
    def mk(self, op, inputs=(), p=None, named=None, dt="U", dim1=-1, dim2=-1, pos=None, cse=True):
        h = Hop(op, inputs, p, named, dt, dim1, dim2, pos)
        if cse:
            k = h.key()
            old = self.cse.get(k)
            if old is not None:
                return old
            self.cse[k] = h
        for c in h.inputs:
            c.parents.append(h)
        return h

    def lit(self, v, pos=None):
        h = lit(v, pos)
        k = ("lit", S.vtype_of(v), "NaN" if isinstance(v, float) and v != v else v)
        old = self.cse.get(k)
        if old is not None:
            return old
        self.cse[k] = h
        return h

    # -- statements ----------------------------------------------------------------
    def add(self, st):
        # MLContext/JMLC semantics (reference: RewriteRemovePersistentReadWrite): a persistent
        # read into a bound input variable, or a write of a bound output, becomes a no-op
        if self.ctx is self.tr.main_ctx:
            if isinstance(st, A.Assign) and isinstance(st.target, A.Ident) and st.target.name in self.tr.inputs \
                    and isinstance(st.value, A.Call) and st.value.name == "read" and st.ifdef is None:
                return
            if isinstance(st, A.ExprStmt) and st.call.name == "write" and st.call.args and \
                    isinstance(st.call.args[0].value, A.Ident) and st.call.args[0].value.name in self.tr.outputs:
                return
        self.stmt_count += 1
        if self.pos is None:
            self.pos = st.pos
        if isinstance(st, A.Assign):
            if st.ifdef is not None:
                name = st.ifdef.name
                if name in self.tr.args:
                    val = self.lit(S.parse_literal_arg(self.tr.args[name]))
                else:
                    val = self.expr(st.value)
            else:
                val = self.expr(st.value)
            t = st.target
            if st.accumulate:
                cur = self.var(t.name, st.pos) if isinstance(t, A.Ident) else self.expr(t)
                val = self.binary("+", cur, val, st.pos)
            if isinstance(t, A.Ident):
                self.env[t.name] = val
            elif isinstance(t, A.Indexed):
                target = self.var(t.name, st.pos)
                rl, ru, cl, cu = self.index_bounds(t)
                h = self.mk("lix", [target, val, rl, ru, cl, cu], p={"list": t.cols is None},
                            dt=target.dt, dim1=target.dim1, dim2=target.dim2, pos=st.pos, cse=False)
                self.env[t.name] = h
            elif isinstance(t, A.CmdParam):
                raise LanguageError(f"{st.pos}: cannot assign to command-line parameter ${t.name}")
        elif isinstance(st, A.MultiAssign):
            call = st.value
            fb = self.tr.resolve_function(self.ctx, call.namespace, call.name)
            if fb is None:
                # multi-return builtins (eigen, svd, qr, lu, transformencode, ...)
                h = self.builtin_call(call, multi=True)
            else:
                h = self.fcall(fb, call)
            self.roots.append(h)
            for i, t in enumerate(st.targets):
                if not isinstance(t, A.Ident):
                    raise LanguageError(f"{st.pos}: multi-assignment targets must be identifiers")
                dt = "M" if fb is None else _param_dt(fb.outputs[i] if i < len(fb.outputs) else None)
                self.env[t.name] = self.mk("fout", [h], p={"i": i}, pos=st.pos, cse=False, dt=dt)
        elif isinstance(st, A.ExprStmt):
            h = self.expr(st.call)
            if h.op in ("sink", "fcall"):
                if h not in self.roots:
                    self.roots.append(h)
            else:
                # value discarded; still evaluate builtin calls for errors (cheap ones are DCE'd)
                pass

    def try_const(self, e):
        """Evaluate expression to a constant if possible (without recording reads)."""
        saved = (set(self.reads), dict(self.treads))
        try:
            h = self.expr(e)
        except (LanguageError, DMLRuntimeError):
            h = None
        self.reads, self.treads = saved
        if h is not None and h.op == "lit":
            return h.value
        return None

    def out_consts(self):
        c = dict(self.consts)
        for k, h in self.env.items():
            if h.op == "lit":
                c[k] = h.value
            else:
                c.pop(k, None)
        return c

    def out_types(self):
        return {k: h.dt for k, h in self.env.items()}

    def finish(self) -> BasicBlock:
        bb = BasicBlock()
        bb.pos = self.pos
        bb.cond = self.tr.cond_depth > 0
        bb.roots = list(self.roots)
        bb.env_out = dict(self.env)
        bb.reads = set(self.reads)
        bb.writes = set(self.env.keys())
        return bb

    # -- expressions ---------------------------------------------------------------
    def var(self, name, pos=None):
        if name in self.env:
            return self.env[name]
        if name in self.consts:
            return self.lit(self.consts[name], pos)
        h = self.treads.get(name)
        if h is None:
            if name not in self.types and name not in self.tr.inputs:
                self.tr.validate_error(f"{pos}: Undefined Variable ({name}) used in statement" if pos else
                                       f"Undefined Variable ({name}) used in statement")
            h = Hop("tread", p={"name": name}, pos=pos, dt=self.types.get(name, "U"))
            self.treads[name] = h
        self.reads.add(name)
        return h

    def expr(self, e) -> Hop:
        if isinstance(e, A.Literal):
            v = e.value
            if e.vtype == "DOUBLE":
                v = float(v)
            elif e.vtype == "INT":
                v = int(v)
            return self.lit(v, e.pos)
        if isinstance(e, A.Ident):
            if e.name not in self.env and e.name not in self.consts and e.name in BUILTIN_CONSTANTS \
                    and e.name not in self.tr.inputs:
                return self.lit(BUILTIN_CONSTANTS[e.name], e.pos)
            return self.var(e.name, e.pos)
        if isinstance(e, A.CmdParam):
            if e.name not in self.tr.args:
                raise LanguageError(f"{e.pos}: command-line parameter ${e.name} not specified")
            return self.lit(S.parse_literal_arg(self.tr.args[e.name]), e.pos)
        if isinstance(e, A.BinOp):
            l = self.expr(e.left)
            r = self.expr(e.right)
            if e.op == "%*%":
                return self.mk("mm", [l, r], dt="M", pos=e.pos)
            return self.binary(e.op, l, r, e.pos)
        if isinstance(e, A.UnOp):
            x = self.expr(e.operand)
            if e.op == "+":
                return x
            return self.unary("neg" if e.op == "-" else "not", x, e.pos)
        if isinstance(e, A.Indexed):
            src = self.var(e.name, e.pos)
            rl, ru, cl, cu = self.index_bounds(e)
            dt = src.dt if src.dt in ("M", "F") else "U"
            return self.mk("rix", [src, rl, ru, cl, cu], p={"list": e.cols is None}, pos=e.pos, dt=dt)
        if isinstance(e, A.Call):
            fb = self.tr.resolve_function(self.ctx, e.namespace, e.name)
            if fb is not None:
                h = self.fcall(fb, e)
                self.roots.append(h)
                return self.mk("fout", [h], p={"i": 0}, pos=e.pos, cse=False,
                               dt=_param_dt(fb.outputs[0] if fb.outputs else None))
            return self.builtin_call(e)
        if isinstance(e, A.ExprList):
            return self.mk("bi", [self.expr(x) for x in e.items], p={"name": "list"}, pos=e.pos)
        raise LanguageError(f"unsupported expression {type(e).__name__}")

    def index_bounds(self, e: A.Indexed):
        none = self.lit(None)

        def rng(r):
            if r is None:
                return none, none
            lo = self.expr(r.lower) if r.lower is not None else none
            if r.is_range:
                hi = self.expr(r.upper) if r.upper is not None else none
            else:
                hi = lo
            return lo, hi

        rl, ru = rng(e.rows)
        cl, cu = rng(e.cols)
        return rl, ru, cl, cu

    def binary(self, op, l, r, pos=None):
        if l.op == "lit" and r.op == "lit" and l.value is not None and r.value is not None:
            try:
                return self.lit(S.binary(op, l.value, r.value), pos)
            except DMLRuntimeError:
                pass
        dt = "M" if (l.dt == "M" or r.dt == "M") else ("S" if (l.dt == "S" and r.dt == "S") else "U")
        return self.mk("b", [l, r], p={"o": op}, dt=dt, pos=pos)

    def unary(self, op, x, pos=None):
        if x.op == "lit" and op in SCALAR_FOLD_UNARY and x.value is not None:
            try:
                return self.lit(S.unary(op, x.value), pos)
            except (DMLRuntimeError, TypeError, ValueError):
                pass
        return self.mk("u", [x], p={"o": op}, dt=x.dt, pos=pos)

    def fcall(self, fb: FunctionBlock, call: A.Call):
        names = [p.name for p in fb.inputs]
        pos_args, named = [], {}
        for a in call.args:
            if a.name is None:
                if named:
                    raise LanguageError(f"{call.pos}: positional argument after named argument")
                pos_args.append(self.expr(a.value))
            else:
                named[a.name] = self.expr(a.value)
        if len(pos_args) > len(names):
            raise LanguageError(f"{call.pos}: too many arguments for function {call.name}")
        bound = dict(zip(names, pos_args))
        for k, v in named.items():
            if k not in names:
                raise LanguageError(f"{call.pos}: unknown parameter '{k}' for function {call.name}")
            bound[k] = v
        inputs, given = [], []
        for prm in fb.inputs:
            n = prm.name
            if n in bound:
                # data-type check of the argument against the declared parameter (reference
                # FunctionCallIdentifier.validateExpression)
                want = prm.dtype[0] if prm.dtype in ("MATRIX", "SCALAR", "FRAME", "LIST") else None
                got = bound[n].dt
                if want in ("M", "S") and got in ("M", "S") and want != got:
                    raise LanguageError(f"{call.pos}: data type mismatch for parameter '{n}' of function "
                                        f"{call.name}: expected {prm.dtype.lower()}, got "
                                        f"{'matrix' if got == 'M' else 'scalar'}")
                inputs.append(bound[n])
                given.append(n)
            elif prm.default is None:
                raise LanguageError(f"{call.pos}: missing argument '{n}' in call to function {call.name}")
        return self.mk("fcall", inputs, p={"fkey": (fb.namespace, fb.name), "given": tuple(given)},
                       pos=call.pos, cse=False)

    def builtin_call(self, call: A.Call, multi=False) -> Hop:
        name = call.name
        pos = call.pos
        args = call.args
        if name == "ifdef" and len(args) == 2 and isinstance(args[0].value, A.CmdParam):
            pname = args[0].value.name
            if pname in self.tr.args:
                return self.lit(S.parse_literal_arg(self.tr.args[pname]), pos)
            return self.expr(args[1].value)
        pos_args = [self.expr(a.value) for a in args if a.name is None]
        named = [(a.name, self.expr(a.value)) for a in args if a.name is not None]
        nd = dict(named)

        if name in UNARY_MATH and len(args) == 1:
            return self.unary(name if name != "ceiling" else "ceil", pos_args[0] if pos_args else named[0][1], pos)
        if name == "ceiling":
            return self.unary("ceil", pos_args[0], pos)
        if name == "log":
            if len(pos_args) == 1 and not named:
                return self.unary("log", pos_args[0], pos)
            x = pos_args[0]
            b = pos_args[1] if len(pos_args) > 1 else nd.get("base")
            return self.binary("log", x, b, pos)
        if name in CUMAGG:
            return self.mk("u", [pos_args[0]], p={"o": name}, dt="M", pos=pos)
        if name in FULL_AGG and len(pos_args) == 1 and not named:
            x = pos_args[0]
            if x.dt == "S" and name in ("sum", "mean", "prod"):
                return x
            return self.mk("agg", [x], p={"o": FULL_AGG[name], "dir": "all"}, dt="S", dim1=0, dim2=0, pos=pos)
        if name in ROWCOL_AGG and len(pos_args) == 1:
            o, d = ROWCOL_AGG[name]
            return self.mk("agg", [pos_args[0]], p={"o": o, "dir": d}, dt="M", pos=pos)
        if name in ("min", "max", "pmin", "pmax"):
            o = "min" if name in ("min", "pmin") else "max"
            allargs = pos_args + [h for _, h in named]
            if len(allargs) == 1:
                return self.mk("agg", [allargs[0]], p={"o": o, "dir": "all"}, dt="S", dim1=0, dim2=0, pos=pos)
            h = allargs[0]
            for x in allargs[1:]:
                h = self.binary(o, h, x, pos)
            return h
        if name in ("nrow", "ncol", "length"):
            x = pos_args[0]
            return self.mk("u", [x], p={"o": name}, dt="S", pos=pos)
        if name == "t":
            return self.mk("t", [pos_args[0]], dt="M", pos=pos)
        if name in CASTS:
            x = pos_args[0]
            o = CASTS[name]
            if x.op == "lit" and o in ("cast_double", "cast_int", "cast_bool", "cast_scalar"):
                return self.unary(o, x, pos)
            return self.mk("u", [x], p={"o": o}, dt="S" if o not in ("cast_matrix", "cast_frame", "cast_list") else "M", pos=pos)
        if name in BINARY_FNS and len(pos_args) == 2:
            return self.binary(BINARY_FNS[name], pos_args[0], pos_args[1], pos)
        if name == "ppred":
            opmap = {">": ">", ">=": ">=", "<": "<", "<=": "<=", "==": "==", "!=": "!="}
            o = pos_args[2].value if len(pos_args) > 2 else nd["op"].value
            return self.binary(opmap[o], pos_args[0], pos_args[1], pos)
        if name == "exists":
            # symbol-table probe (reference AggregateUnaryCPInstruction.java:130-136 EXISTS):
            # a variable assigned earlier in this block is defined here; otherwise the frame
            # is probed when the statement runs.  exists("X") names the variable by a string.
            a = args[0].value
            vn = a.name if isinstance(a, A.Ident) else (a.value if isinstance(a, A.Literal) and isinstance(a.value, str) else None)
            if vn is not None:
                if vn in self.env:
                    return H.lit(True, pos)
                return self.mk("bi", [], p={"name": "exists", "var": vn}, dt="S", pos=pos, cse=False)
        if name == "ifelse" and all(h.op == "lit" for h in pos_args) and len(pos_args) == 3:
            return pos_args[1] if S.as_bool(pos_args[0].value) else pos_args[2]
        if name == "time":
            # evaluated where its statement stands: a pure hop would be emitted lazily at its
            # first use (e.g. after a later time() call)
            h = self.mk("bi", [], p={"name": "time"}, dt="S", pos=pos, cse=False)
            self.roots.append(h)
            return h
        if name == "eval":
            # dynamic function call: resolve at runtime in this file context
            return self._eval_call(pos_args, named, pos)
        dt = _BI_DT.get(name, "U")
        if name == "ifelse" and len(pos_args) == 3 and not named:
            # a matrix operand makes the result a matrix; all-scalar operands a scalar
            ds = [h.dt for h in pos_args]
            dt = "M" if "M" in ds else ("S" if all(d == "S" for d in ds) else "U")
        if name in _DIST_FNS:
            tgt = nd.get("target", pos_args[0] if pos_args else None)
            dt = "M" if tgt is not None and tgt.dt == "M" else ("U" if tgt is None or tgt.dt == "U" else "S")
        if name == "read":
            dtn = nd.get("data_type")
            if dtn is not None and dtn.op == "lit":
                dt = {"frame": "F", "scalar": "S", "list": "L"}.get(str(dtn.value), "M")
            else:
                dt = "U"
        side = name in H.SIDE_EFFECT
        nondet = name in H.NONDETERMINISTIC or (name in ("rand", "sample") and
                                               not _has_literal_seed(nd))
        inputs = pos_args + [h for _, h in named]
        h = self.mk("sink" if side else "bi", inputs, p={"name": name, "npos": len(pos_args)},
                    named=[n for n, _ in named], pos=pos, cse=not (side or nondet or multi), dt=dt)
        if side:
            self.roots.append(h)
        return h

    def _eval_call(self, pos_args, named, pos):
        inputs = pos_args + [h for _, h in named]
        return self.mk("bi", inputs, p={"name": "eval", "npos": len(pos_args), "nskey": self.ctx.key,
                                        "imports": tuple(sorted(self.ctx.imports.items()))},
                       named=[n for n, _ in named], pos=pos, cse=False)


def _reads_unknown_size(e):
    """True if the expression reads a matrix without literal rows / cols arguments."""
    if isinstance(e, A.Call):
        if e.name == "read" and not e.namespace:
            named = {a.name for a in e.args if getattr(a, "name", None)}
            return not {"rows", "cols"} <= named
        return any(_reads_unknown_size(a.value) for a in e.args)
    for attr in ("left", "right", "operand", "target"):
        x = getattr(e, attr, None)
        if isinstance(x, A.Expr) and _reads_unknown_size(x):
            return True
    return False


_M_BUILTINS = ("matrix rand Rand seq sample cbind rbind table ctable diag rev removeEmpty replace order solve inv "
               "inverse cholesky outer quantile interQuantile aggregate lower.tri upper.tri conv2d "
               "conv2d_backward_filter conv2d_backward_data max_pool avg_pool max_pool_backward "
               "avg_pool_backward bias_add bias_multiply transformapply transformcolmap transform").split()
_S_BUILTINS = "toString median interQuartileMean moment centralMoment cov cdf invcdf pnorm qnorm pt qt pf qf " \
              "pchisq qchisq pexp qexp exists time".split()
_DIST_FNS = set("cdf invcdf icdf pnorm qnorm pt qt pf qf pchisq qchisq pexp qexp".split())
_BI_DT = {**{n: "M" for n in _M_BUILTINS}, **{n: "S" for n in _S_BUILTINS}, "list": "L",
          "transformdecode": "F", "transformmeta": "F"}


def _param_dt(p):
    if p is None:
        return "U"
    return {"MATRIX": "M", "SCALAR": "S", "FRAME": "F", "LIST": "L"}.get(p.dtype, "U")


def _has_literal_seed(nd):
    s = nd.get("seed")
    return s is not None and s.op == "lit" and s.value is not None and s.value != -1


# ============================================================================
# Live variable analysis (reference: parser/LiveVariableAnalysis.java)
# ============================================================================
def _blocks_gen_kill(blocks):
    """Upward-exposed reads (gen) and definite writes (kill) of a block list."""
    gen, kill = set(), set()
    for b in blocks:
        g, k = _block_gen_kill(b)
        gen |= (g - kill)
        kill |= k
    return gen, kill


def _block_gen_kill(b):
    if isinstance(b, BasicBlock):
        return set(b.reads), set(b.writes)
    if isinstance(b, IfBlock):
        g1, k1 = _blocks_gen_kill(b.then_blocks)
        g2, k2 = _blocks_gen_kill(b.else_blocks)
        return b.pred.reads | g1 | g2, k1 & k2
    if isinstance(b, WhileBlock):
        g, _ = _blocks_gen_kill(b.body)
        return b.pred.reads | g, set()
    if isinstance(b, ForBlock):
        g, _ = _blocks_gen_kill(b.body)
        r = b.start.reads | b.end.reads | (b.incr.reads if b.incr else set())
        return r | (g - {b.var}), set()
    return set(), set()


def liveness(blocks, live_out_final=None):
    """Backward pass setting BasicBlock.live_out / rmvars. Returns live-in set of the list."""
    live = set(live_out_final) if live_out_final is not None else set()
    return _live_list(blocks, live)


def _live_list(blocks, live_after):
    live = set(live_after)
    for b in reversed(blocks):
        live = _live_block(b, live)
    return live


def _live_block(b, live_after):
    if isinstance(b, BasicBlock):
        b.live_out = set(live_after)
        b.rmvars = sorted((b.reads | b.writes) - b.live_out)
        return (b.live_out - b.writes) | b.reads
    if isinstance(b, IfBlock):
        l1 = _live_list(b.then_blocks, live_after)
        l2 = _live_list(b.else_blocks, live_after)
        return l1 | l2 | b.pred.reads
    if isinstance(b, (WhileBlock, ForBlock)):
        if isinstance(b, WhileBlock):
            preds = set(b.pred.reads)
        else:
            preds = b.start.reads | b.end.reads | (b.incr.reads if b.incr else set())
        end = set(live_after) | preds
        for _ in range(10):
            lin = _live_list(b.body, end)
            new_end = set(live_after) | preds | lin
            if isinstance(b, ForBlock) and b.var not in live_after:
                # the iteration variable keeps its last value after the loop
                # (reference ForProgramBlock.java:126), so it stays live when read later
                new_end.discard(b.var)
            if new_end == end:
                break
            end = new_end
        # read before written in one iteration (runtime/graphloop.py); computed before the
        # final pass below, which leaves the body blocks' live_out as they must be
        reads = _live_list(b.body, set())
        lin = _live_list(b.body, end)
        b.iter_live = set(end)          # live after every iteration
        b.body_live_in = set(reads)
        if isinstance(b, ForBlock):
            b.result_vars = sorted(set(live_after) & _all_writes(b.body))
            lin = lin - {b.var}
        return lin | preds | set(live_after)
    return set(live_after)


def _all_writes(blocks):
    out = set()
    for b in blocks:
        if isinstance(b, BasicBlock):
            out |= b.writes
        elif isinstance(b, IfBlock):
            out |= _all_writes(b.then_blocks) | _all_writes(b.else_blocks)
        elif isinstance(b, (WhileBlock, ForBlock)):
            out |= _all_writes(b.body)
            if isinstance(b, ForBlock):
                out.add(b.var)
    return out
