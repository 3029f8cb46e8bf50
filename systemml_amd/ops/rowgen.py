"""Generated Row-template operators (reference: hops/codegen/template/TemplateRow.java for the
fusion candidates, cplan/CNodeRow.java for the generated class and runtime/codegen/
SpoofRowwise.java for its execution; the vector primitives of runtime/codegen/LibSpoofPrimitives
-- vectMult, vectAdd, dotProduct, vectSum, vectMax ... -- become straight-line HIP code here).

A `RowProgram` is one fused DAG whose values are, per row of a tall matrix,
  V  a row vector of length D (an N x D input, a broadcast 1 x D input, or cellwise work on them),
  S  a per-row scalar (an N x 1 input, a row aggregate `rowSums/rowMeans/rowMaxs/rowMins/
     rowSums(^2)` of a V, a matrix-vector product `V %*% v` with a D x 1 side vector, or cellwise
     work on S values),
  C  a constant (scalar / 1 x 1 input).
The program ends in one output:
  row / vec  the root value per row (N x 1 or N x D),
  col        colSums / colMeans / colSums(^2) of a V (1 x D),
  tmv        t(V) %*% S (D x 1: the Row template's t(X) %*% f(X %*% v) shape),
  all        sum / mean / min / max / sum of squares over every value.

On the MI355X the program runs as ONE kernel generated per program and operand signature and
compiled with hipRTC (ops/cell.compile_source, cached by source hash).  L = 4..64 lanes share a
row (L chosen from D so every lane holds several elements); the row's reductions are phases:
phase p streams the row once, evaluates the V expressions its row aggregates / dot products
need and reduces them across the L lanes with `__shfl_xor`; the S values that depend on them
are then available to phase p + 1 (re-reads of the same row come from L1/L2, so HBM sees each
input row once).  Column outputs accumulate in LDS slices per row group (deterministic, no
atomics) and leave one fp64 partial row per workgroup; full aggregates one fp64 partial.

Everywhere else -- CPU backend, sparse / compressed / constant-column / row-partitioned
operands, shapes that do not classify as V / S / C, D = 1 -- the program runs as the original
operators one after the other (`sequential`), so fusion never changes semantics or errors.
"""
from __future__ import annotations

import ctypes

import torch

from . import core as C
from .backend import backend
from .cell import (_C_BIN, _C_UN, _DT, _Tensor, _prelude, _raw_stream, _rtc_lib, _signature, compile_source,
                   gpu_arch)

ROW_AGGS = ("sum", "sumsq", "mean", "min", "max")
COL_AGGS = ("sum", "sumsq", "mean")
ALL_AGGS = ("sum", "sumsq", "mean", "min", "max")
OTYPES = ("row", "vec", "col", "tmv", "all")
MAXIN, MAXOPS, MAXOUT = 8, 64, 6
LDS_BYTES = 65536
stats = {"kernel": 0, "sequential": 0, "compiled": 0}

FULL, ROWV, COLV, HSCALAR, DSCALAR, SIDE = range(6)


class RowProgram:
    """ops: tuple of (kind, op, a, b) over node indices -- inputs are nodes 0..n_in-1, op j is
    node n_in + j; kind 'b' (binary), 'u' (unary, 'sq' = x^2), 'ragg' (row aggregate `op` of
    node a), 'dot' (node a %*% input b: b a D x 1 side vector -> per-row scalar, or a D x K side
    matrix -> a K-wide per-row vector, the reference's vectMatrixMult), 'cbindc' (a K-wide
    vector with node b -- a scalar -- appended: cbind(W, matrix(c, nrow, 1))), 'wcols' (columns
    1..b of a K-wide vector: W[, 1:b]).  out: output node; otype / oagg: output type and its
    aggregate; extra: the S / W node of a 'tmv' output (t(V) %*% S -> D x 1, t(V) %*% W -> D x K).
    more: further outputs (node, otype, oagg, extra) computed by the same pass (multi-output
    Row template): the kernel streams the rows once for all of them."""
    __slots__ = ("n_in", "ops", "out", "otype", "oagg", "extra", "more", "parts")

    def __init__(self, n_in, ops, out, otype, oagg=None, extra=None, more=(), parts=()):
        if otype not in OTYPES or any(m[1] not in OTYPES for m in more):
            raise ValueError(otype)
        self.n_in = n_in
        self.ops = tuple(tuple(x) for x in ops)
        self.out = out
        self.otype = otype
        self.oagg = oagg
        self.extra = extra
        self.more = tuple(tuple(m) for m in more)
        # a merged multi-output program: its source programs and their input positions, run
        # one by one when the merged kernel does not apply to the actual operands
        self.parts = tuple(parts)

    def outputs(self):
        return ((self.out, self.otype, self.oagg, self.extra),) + self.more

    def key(self):
        return (self.n_in, self.ops, self.out, self.otype, self.oagg, self.extra, self.more)

    def __eq__(self, other):
        return isinstance(other, RowProgram) and self.key() == other.key()

    def __hash__(self):
        return hash(self.key())

    def side_inputs(self):
        return {b for kind, _, _, b in self.ops if kind == "dot"}

    def describe(self):
        body = ",".join(("dot" if k == "dot" else (f"r{o}" if k == "ragg" else (k if k in ("cbindc", "wcols", "wcolsv") else o)))
                        for k, o, _, _ in self.ops)
        tails = []
        for _, ot, oagg, _ in self.outputs():
            tails.append({"row": "", "vec": "", "col": f"|col{oagg}", "tmv": "|t(.)%*%", "all": f"|{oagg}"}[ot])
        return f"row[{body}]{''.join(tails)}" + (f"x{len(self.outputs())}" if self.more else "")

    def __repr__(self):
        return self.describe()


def _seq_value(kind, o, va, vb):
    if kind == "b":
        return C.binary(o, va, vb)
    if kind == "u":
        return C.binary("^", va, 2) if o == "sq" else C.unary(o, va)
    if kind == "ragg":
        return C.agg(o, "row", va)
    if kind == "cbindc":
        col = vb if isinstance(vb, torch.Tensor) and vb.dim() == 2 else \
            torch.full((va.shape[0], 1), float(C._num(vb)), dtype=va.dtype, device=va.device)
        return torch.cat([va, col.to(va.dtype).to(va.device).expand(va.shape[0], 1)], 1)
    if kind in ("wcols", "wcolsv"):
        return C.rix(va, None, None, 1, vb)
    return C.mm(va, vb, False)


def _seq_output(vals, node, ot, oagg, extra):
    r = vals[node]
    if ot == "col":
        return C.agg(oagg, "col", r)
    if ot == "all":
        return C.agg(oagg, "all", r)
    if ot == "tmv":
        return C.mm(r, vals[extra], True)
    return r


def sequential(prog: RowProgram, args):
    """The fused DAG's original operators, one after the other."""
    vals = list(args)
    for kind, o, a, b in prog.ops:
        vals.append(_seq_value(kind, o, vals[a], vals[b] if kind in ("b", "dot", "cbindc", "wcolsv") else b))
    outs = tuple(_seq_output(vals, *o) for o in prog.outputs())
    return outs if prog.more else outs[0]


def evaluate(prog: RowProgram, args):
    r = _kernel(prog, args) if backend.use_kernels else None
    if r is not None:
        stats["kernel"] += 1
        return r
    if prog.parts:
        # the merged kernel is out of scope here: each source program on its own
        res = []
        for p, m in prog.parts:
            v = evaluate(p, [args[i] for i in m])
            res.extend(v if p.more else (v,))
        return tuple(res)
    stats["sequential"] += 1
    return sequential(prog, args)


# ----------------------------------------------------------------------------- classification
FULLW, ROWW, SIDEM = 6, 7, 8
MAXW = 16                      # widest per-row vector (K) a program keeps in registers


def classify(prog: RowProgram, shapes):
    """shapes: per input (rows, cols) or None (scalar).  Returns (N, D, leaf modes, node kinds,
    node widths) or None when the operands are outside the kernel's scope.  Kinds: V (a D-wide
    row), W (a narrow per-row vector, width in `widths`), S (per-row scalar), C (constant),
    X / Y (D x 1 side vector / D x K side matrix)."""
    side = prog.side_inputs()
    D = 0
    for k in side:
        s = shapes[k]
        if s is None:
            return None
        if D and s[0] != D:
            return None
        D = s[0]
    if not D:
        # no side operand: the rows are the widest input (narrower ones are K-wide vectors)
        D = max((s[1] for k, s in enumerate(shapes) if s is not None and k not in side), default=0)
    N = 1
    for k, s in enumerate(shapes):
        if s is None or k in side:
            continue
        r, c = s
        if r > 1:
            if N > 1 and r != N:
                return None
            N = r
    if D <= 1:
        return None
    modes, kinds, widths = [], [], []
    for k, s in enumerate(shapes):
        if k in side:
            if s[1] == 1:
                modes.append(SIDE)
                kinds.append("X")
                widths.append(0)
            elif s[1] <= MAXW and s[1] != D:
                modes.append(SIDEM)
                kinds.append("Y")
                widths.append(s[1])
            else:
                return None
            continue
        if s is None:
            modes.append(HSCALAR)
            kinds.append("C")
            widths.append(0)
            continue
        r, c = s
        if c == D and (r == N or r == 1) and (N > 1 or r == 1):
            modes.append(FULL if (r == N and N > 1) else ROWV)
            kinds.append("V")
            widths.append(0)
        elif c == 1 and r == N and N > 1:
            modes.append(COLV)
            kinds.append("S")
            widths.append(0)
        elif r == 1 and c == 1:
            modes.append(DSCALAR)
            kinds.append("C")
            widths.append(0)
        elif 1 < c <= MAXW and c != D and (r == N or r == 1) and N > 1:
            modes.append(FULLW if r == N else ROWW)
            kinds.append("W")
            widths.append(c)
        else:
            return None
    for kind, o, a, b in prog.ops:
        ka, wa = kinds[a], widths[a]
        if kind == "b":
            kb, wb = kinds[b], widths[b]
            if "X" in (ka, kb) or "Y" in (ka, kb) or ("V" in (ka, kb) and "W" in (ka, kb)):
                return None
            if ka == "W" and kb == "W" and wa != wb:
                return None
            if "V" in (ka, kb):
                kinds.append("V")
                widths.append(0)
            elif "W" in (ka, kb):
                kinds.append("W")
                widths.append(wa if ka == "W" else wb)
            else:
                kinds.append("S" if "S" in (ka, kb) else "C")
                widths.append(0)
        elif kind == "u":
            if ka in ("X", "Y"):
                return None
            kinds.append(ka)
            widths.append(wa)
        elif kind == "ragg":
            if ka not in ("V", "S", "W"):
                return None
            kinds.append("S")
            widths.append(0)
        elif kind == "cbindc":
            if ka != "W" or kinds[b] not in ("S", "C") or wa + 1 > MAXW:
                return None
            kinds.append("W")
            widths.append(wa + 1)
        elif kind == "wcols":
            if ka != "W" or not (1 <= b <= wa):
                return None
            kinds.append("W" if b > 1 else "S")
            widths.append(b if b > 1 else 0)
        else:
            if ka != "V" or kinds[b] not in ("X", "Y"):
                return None
            kinds.append("S" if kinds[b] == "X" else "W")
            widths.append(0 if kinds[b] == "X" else widths[b])
    colacc = 0
    for node, ot, oagg, extra in prog.outputs():
        ko = kinds[node]
        if ot in ("row", "vec", "all") and ko not in ("V", "S", "W"):
            return None
        if ot == "col" and ko not in ("V", "W"):
            return None
        if ot == "tmv" and (ko != "V" or kinds[extra] not in ("S", "W")):
            return None
        if ot == "tmv" or (ot == "col" and ko == "V"):
            colacc += 1
        if prog.more and ot == "vec" and ko == "V":
            return None                  # one D-wide written output at most, as the primary
    if colacc > 1:
        return None                      # one LDS column accumulator per kernel
    return N, D, tuple(modes), tuple(kinds), tuple(widths)


def out_shape(prog: RowProgram, shapes, which=0):
    """Result shape of output `which` for input shapes (None: scalar) under the original
    operators' rules; None if an operator would reject its operands or the result is a scalar."""
    from .cell import _bin_ok
    v = list(shapes)
    for kind, o, a, b in prog.ops:
        sa = v[a]
        if kind == "u":
            v.append(sa)
        elif kind == "b":
            sb = v[b]
            if sa is None or sb is None:
                v.append(sb if sa is None else sa)
            elif _bin_ok(sa, sb):
                v.append((max(sa[0], sb[0]), max(sa[1], sb[1])))
            else:
                return None
        elif kind == "ragg":
            if sa is None:
                return None
            v.append((sa[0], 1))
        elif kind == "cbindc":
            if sa is None:
                return None
            v.append((sa[0], sa[1] + 1))
        elif kind == "wcols":
            if sa is None or b > sa[1]:
                return None
            v.append((sa[0], b))
        elif kind == "wcolsv":
            return None                      # width known at run time only
        else:
            sb = v[b]
            if sa is None or sb is None or sa[1] != sb[0]:
                return None
            v.append((sa[0], sb[1]))
    node, ot, _, extra = prog.outputs()[which]
    r = v[node]
    if r is None:
        return None
    if ot == "col":
        return (1, r[1])
    if ot == "tmv":
        e = v[extra]
        return None if e is None or e[0] != r[0] else (r[1], e[1])
    if ot == "all":
        return None
    return r


REG_BUDGET = 96            # cached fp32 values per lane (fp64 count twice)
ACCW_BUDGET = 160          # register accumulators of a t(V) %*% W output per lane


def _colacc_output(prog, kinds):
    """The output accumulated per column in LDS / registers (col of a V, tmv), or None."""
    for o in prog.outputs():
        node, ot, _, extra = o
        if ot == "tmv" or (ot == "col" and kinds[node] == "V"):
            return o
    return None


def plan_registers(prog, modes, kinds, D, L, vec, T, dcap, dts=None, widths=None):
    """(J, cache): J lane-owned column chunks of VEC elements cover a row (0: the row is too
    wide -- strided streaming loops instead); cache holds the input indices kept in registers
    ('acc' for the column accumulators), chosen greedily within REG_BUDGET: the column
    accumulators, then the N x D inputs (each row read from HBM once for every phase), then
    the row-invariant 1 x D / side vectors."""
    dts = dts or tuple(0 for _ in modes)
    J = (D + L * vec - 1) // (L * vec)
    if J * vec > 64:
        return 0, frozenset()
    per = J * vec * (1 if T == torch.float32 else 2)
    used = 0
    cache = []
    ca = _colacc_output(prog, kinds)
    if widths:
        # K-wide per-row vectors live in registers too (their widths, counted once)
        used += sum(w for w in widths[prog.n_in:]) * (1 if T == torch.float32 else 2) // 2
    if ca is not None and ca[1] == "tmv" and kinds[ca[3]] == "W":
        # t(V) %*% W: J x VEC x K register accumulators per lane (merged per workgroup at the
        # end) instead of LDS atomics on every element of every row
        kw = widths[ca[3]] if widths else 1
        if J * vec * kw * (1 if T == torch.float32 else 2) <= ACCW_BUDGET and dcap \
                and dcap * kw * (4 if T == torch.float32 else 8) <= LDS_BYTES:
            cache.append("acc")
            used += per          # its own budget; counted like a one-wide accumulator here
    elif ca is not None and dcap and dcap * (4 if T == torch.float32 else 8) <= LDS_BYTES:
        cache.append("acc")
        used += per
    vecuse = set()
    for kind, o, a, b in prog.ops:
        for x in ((a, b) if kind in ("b", "dot") else (a,)):
            if x < prog.n_in and modes[x] in (FULL, ROWV, SIDE):
                vecuse.add(x)
    for node, _, _, _ in prog.outputs():
        if node < prog.n_in and modes[node] in (FULL, ROWV, SIDE):
            vecuse.add(node)
    full = [k for k in sorted(vecuse) if modes[k] == FULL]
    pipe = bool(full) and used + 2 * per * len(full) <= REG_BUDGET and \
        all(vec in (1, 4) or dts[k] == 2 for k in full)
    for k in full:
        if used + per * (2 if pipe else 1) <= REG_BUDGET:
            cache.append(k)
            used += per * (2 if pipe else 1)
    if pipe and all(k in cache for k in full):
        cache.append("pipe")
    for k in sorted(vecuse):
        if modes[k] in (ROWV, SIDE) and used + per <= REG_BUDGET:
            cache.append(k)
            used += per
    return J, frozenset(cache)


def lanes_for(D):
    L = 4
    while L < 64 and L * 4 < D:
        L *= 2
    return L


def dcap_for(D):
    """LDS columns of a column-aggregate accumulator (D rounded up to 64)."""
    return (D + 63) // 64 * 64 if D <= 16384 else None


def lds_slices(G, dcap, T):
    """Accumulator slices: one per row group (deterministic sums) when they fit in LDS, else
    one slice shared by all groups through LDS atomics; 0 if even that does not fit."""
    sz = 4 if T == torch.float32 else 8
    if G * dcap * sz <= LDS_BYTES:
        return G
    return 1 if dcap * sz <= LDS_BYTES else 0


# ----------------------------------------------------------------------------- code generation
_RAGG_INIT = {"sum": "T(0)", "sumsq": "T(0)", "mean": "T(0)", "min": "(T)__builtin_inf()", "max": "-(T)__builtin_inf()"}


def _acc_step(o, acc, v):
    if o in ("sum", "mean"):
        return f"{acc} += {v};"
    if o == "sumsq":
        return f"{acc} += {v} * {v};"
    return f"{acc} = sysml_{o}<T>({acc}, {v});"


def _comb(o, a, b):
    if o in ("sum", "mean", "sumsq"):
        return f"{a} + {b}"
    return f"sysml_{o}<T>({a}, {b})"


def generate(prog: RowProgram, T, modes, dts, kinds, L, dcap, vec=1, slices=None, J=0, cache=frozenset(),
             widths=None):
    """HIP source of the fused row kernel (see the module docstring for the phase structure).
    K-wide per-row vectors (W nodes) are register arrays every lane of the row's group holds in
    full: a product with a D x K side matrix accumulates K partial dot products per lane over
    the lane's columns and reduces them across the L lanes like a row aggregate; cellwise work
    and row aggregates on W values then run redundantly in every lane (K is small)."""
    ct = "float" if T == torch.float32 else "double"
    n_in = prog.n_in
    G = 256 // L
    widths = widths or tuple(0 for _ in kinds)
    nodes = [("in", None, k, None) for k in range(n_in)] + list(prog.ops)
    outs = prog.outputs()
    # phase availability: a reduction over a V runs in the phase its input is complete in and
    # its result is available from the next phase on
    avail, red_phase = [], {}
    for i, (kind, o, a, b) in enumerate(nodes):
        if kind == "in":
            avail.append(0)
        elif kind in ("ragg", "dot") and kinds[a] == "V":
            red_phase[i] = avail[a]
            avail.append(avail[a] + 1)
        elif kind in ("b", "cbindc"):
            avail.append(max(avail[a], avail[b]))
        else:
            avail.append(avail[a])

    def out_phase(o):
        node, ot, _, extra = o
        return avail[node] if ot != "tmv" else max(avail[node], avail[extra])
    finals = [out_phase(o) for o in outs]
    ca = _colacc_output(prog, kinds)
    ca_w = ca is not None and ca[1] == "tmv" and kinds[ca[3]] == "W"     # t(V) %*% W: D x K
    KW = widths[ca[3]] if ca_w else 1

    def op_expr(i, ref):
        kind, o, a, b = nodes[i]
        if kind == "b":
            return _C_BIN[o].format(a=ref(a), b=ref(b))
        if kind == "u":
            return _C_UN[o].format(a=ref(a), b="")
        if kind == "ragg":                 # of an S value
            return f"({ref(a)} * {ref(a)})" if o == "sumsq" else ref(a)
        raise AssertionError(kind)

    out = []
    w = out.append
    w(f"// generated: {prog.describe()}")
    w(f"struct SysmlRowArgs {{ const void* in[8]; double s[8]; sysml_i64 rows, cols; void* out[{MAXOUT}]; "
      f"double* part[{MAXOUT}]; }};")
    w(f"extern \"C\" __global__ void __launch_bounds__(256) sysml_row_k(const SysmlRowArgs A) {{")
    w(f"  typedef {ct} T;")
    w(f"  constexpr int L = {L}, G = {G};")
    w("  const int tid = threadIdx.x, lane = tid % L, grp = tid / L;")
    w("  const sysml_i64 N = A.rows, D = A.cols;")
    w("  (void)lane; (void)D;")
    # constants
    cname = {}
    for k in range(n_in):
        if kinds[k] == "C":
            if modes[k] == HSCALAR:
                w(f"  const T c{k} = (T)A.s[{k}];")
            else:
                w(f"  const T c{k} = sysml_ld<T>(A.in[{k}], {dts[k]}, 0);")
            cname[k] = f"c{k}"
    for i in range(n_in, len(nodes)):
        if kinds[i] == "C":
            w(f"  const T c{i} = {op_expr(i, lambda j: cname[j])};")
            cname[i] = f"c{i}"
    # D x K side matrices: staged in LDS once per workgroup when small, else read through L1/L2
    smat = {}
    for k in range(n_in):
        if modes[k] == SIDEM:
            K = widths[k]
            if dcap and dcap * K * (4 if T == torch.float32 else 8) <= 32768:
                # column-major in LDS ([K][dcap]): a lane's VEC consecutive d of one column are
                # adjacent words (vector LDS reads; the row-major [d][K] layout put the lanes'
                # d, VEC apart, on one bank)
                w(f"  __shared__ T sm{k}[{dcap * K}];")
                w(f"  for (int q = tid; q < D * {K}; q += 256) sm{k}[(q % {K}) * {dcap} + q / {K}] = "
                  f"sysml_ld<T>(A.in[{k}], {dts[k]}, q);")
                smat[k] = lambda d, kk, k=k, dc=dcap: f"sm{k}[({kk}) * {dc} + ({d})]"
            else:
                smat[k] = lambda d, kk, k=k, K=K: f"sysml_ld<T>(A.in[{k}], {dts[k]}, ({d}) * {K} + {kk})"
    colacc = ca is not None
    S = G if slices is None else slices
    if ca_w:
        S = 1
    structured = J > 0
    creg = colacc and structured and "acc" in cache
    if creg and ca_w:
        w(f"  T racc[{J}][{vec}][{KW}];")
        w("  #pragma unroll")
        w(f"  for (int jj = 0; jj < {J}; ++jj)")
        w("    #pragma unroll")
        w(f"    for (int u = 0; u < {vec}; ++u)")
        w("      #pragma unroll")
        w(f"      for (int kk = 0; kk < {KW}; ++kk) racc[jj][u][kk] = T(0);")
    elif creg:
        w(f"  T racc[{J}][{vec}];")
        w("  #pragma unroll")
        w(f"  for (int jj = 0; jj < {J}; ++jj)")
        w("    #pragma unroll")
        w(f"    for (int u = 0; u < {vec}; ++u) racc[jj][u] = T(0);")
    elif colacc:
        w(f"  __shared__ T acc[{S}][{dcap * KW}];")
        w(f"  for (int q = tid; q < {S} * {dcap * KW}; q += 256) (&acc[0][0])[q] = T(0);")
    if smat or (colacc and not creg):
        w("  __syncthreads();")

    def col_add(ind, val, kk=None):
        idx = "d" if kk is None else f"d * {KW} + {kk}"
        if S == G and kk is None:
            w(f"{ind}acc[grp][{idx}] += {val};")
        else:
            w(f"{ind}atomicAdd(&acc[0][{idx}], {val});")

    def load_cached(k, base, indent, name=None, declare=True, cond="d0 < D"):
        name = name or f"xr{k}"
        if declare:
            w(f"{indent}T {name}[{J}][{vec}];")
        w(f"{indent}#pragma unroll")
        w(f"{indent}for (int jj = 0; jj < {J}; ++jj) {{")
        w(f"{indent}  const sysml_i64 d0 = ((sysml_i64)lane + (sysml_i64)jj * L) * {vec};")
        w(f"{indent}  if ({cond}) sysml_ldv{vec}<T>(A.in[{k}], {dts[k]}, {base}, {name}[jj]);")
        w(f"{indent}}}")

    # software pipelining of the cached row: the next row of the group is loaded (xn) while the
    # current one (xr) is reduced, so every lane keeps its loads in flight across the phases
    piped = [k for k in range(n_in) if modes[k] == FULL and k in cache and "pipe" in cache]

    w("  const sysml_i64 first = (sysml_i64)blockIdx.x * G + grp;")
    w("  (void)first;")

    def load_raw(k, rowexpr, indent, declare):
        if declare:
            w(f"{indent}SysmlRaw<{dts[k]}, {vec}> rn{k}[{J}];")
        w(f"{indent}#pragma unroll")
        w(f"{indent}for (int jj = 0; jj < {J}; ++jj) {{")
        w(f"{indent}  const sysml_i64 d0 = ((sysml_i64)lane + (sysml_i64)jj * L) * {vec};")
        w(f"{indent}  if ({rowexpr} < N && d0 < D) rn{k}[jj].load(A.in[{k}], {rowexpr} * D + d0);")
        w(f"{indent}}}")
    for k in piped:
        load_raw(k, "first", "  ", True)
    # row-invariant vectors (1 x D inputs, side vectors of products) cached once per kernel
    for k in range(n_in):
        if modes[k] in (ROWV, SIDE) and k in cache:
            load_cached(k, "d0", "  ")
    # 1 x K inputs: once per kernel
    for k in range(n_in):
        if modes[k] == ROWW:
            K = widths[k]
            w(f"  T w{k}[{K}];")
            w(f"  for (int kk = 0; kk < {K}; ++kk) w{k}[kk] = sysml_ld<T>(A.in[{k}], {dts[k]}, kk);")
    # per-output accumulators of full aggregates / W column sums
    for q, (node, ot, oagg, extra) in enumerate(outs):
        if ot == "all":
            w(f"  T tot{q} = {_RAGG_INIT[oagg]};")
        elif ot == "col" and kinds[node] == "W":
            w(f"  T cw{q}[{widths[node]}];")
            w(f"  for (int kk = 0; kk < {widths[node]}; ++kk) cw{q}[kk] = T(0);")
    w("  for (sysml_i64 row = (sysml_i64)blockIdx.x * G + grp; row < N; row += (sysml_i64)gridDim.x * G) {")
    w("    const sysml_i64 rowoff = row * D;")
    w("    (void)rowoff;")
    if piped:
        w("    const sysml_i64 nxt = row + (sysml_i64)gridDim.x * G;")
        for k in piped:
            w(f"    T xr{k}[{J}][{vec}];")
            w("    #pragma unroll")
            w(f"    for (int jj = 0; jj < {J}; ++jj) rn{k}[jj].template get<T>(xr{k}[jj]);")
            load_raw(k, "nxt", "    ", False)
    sname = dict(cname)
    wname = {}
    for k in range(n_in):
        if kinds[k] == "S":
            w(f"    const T s{k} = sysml_ld<T>(A.in[{k}], {dts[k]}, row);")
            sname[k] = f"s{k}"
        elif modes[k] == FULLW:
            K = widths[k]
            w(f"    T w{k}[{K}];")
            w("    #pragma unroll")
            w(f"    for (int kk = 0; kk < {K}; ++kk) w{k}[kk] = sysml_ld<T>(A.in[{k}], {dts[k]}, row * {K} + kk);")
            wname[k] = f"w{k}"
        elif modes[k] == ROWW:
            wname[k] = f"w{k}"
    # the row itself: every N x D input read ONCE from HBM into registers, reused by all phases
    for k in range(n_in):
        if modes[k] == FULL and k in cache and k not in piped:
            load_cached(k, "rowoff + d0", "    ")

    def sref(j):
        return sname[j]

    def wref(j):
        """Element kk of node j in a W context (S / C values broadcast)."""
        if kinds[j] == "W":
            return f"{wname[j]}[kk]"
        return sname[j]

    emitted = set(range(n_in)) | set(cname)

    def emit_values(p):
        """S and W nodes computable by phase p (outside the element loops)."""
        for i in range(n_in, len(nodes)):
            if i in emitted or kinds[i] not in ("S", "W") or i in red_phase or avail[i] > p:
                continue
            kind, o, a, b = nodes[i]
            if kinds[i] == "S" and kind == "ragg" and kinds[a] == "W":
                K = widths[a]
                w(f"    T s{i} = {_RAGG_INIT[o]};")
                w("    #pragma unroll")
                w(f"    for (int kk = 0; kk < {K}; ++kk) {{ {_acc_step(o, f's{i}', f'{wname[a]}[kk]')} }}")
                if o == "mean":
                    w(f"    s{i} /= (T){K};")
                sname[i] = f"s{i}"
            elif kinds[i] == "S" and kind == "wcols":
                w(f"    const T s{i} = {wname[a]}[0];")
                sname[i] = f"s{i}"
            elif kinds[i] == "S":
                w(f"    const T s{i} = {op_expr(i, sref)};")
                sname[i] = f"s{i}"
            else:
                K = widths[i]
                w(f"    T w{i}[{K}];")
                if kind == "cbindc":
                    w("    #pragma unroll")
                    w(f"    for (int kk = 0; kk < {K - 1}; ++kk) w{i}[kk] = {wname[a]}[kk];")
                    w(f"    w{i}[{K - 1}] = {sname[b]};")
                elif kind == "wcols":
                    w("    #pragma unroll")
                    w(f"    for (int kk = 0; kk < {K}; ++kk) w{i}[kk] = {wname[a]}[kk];")
                else:
                    w("    #pragma unroll")
                    w(f"    for (int kk = 0; kk < {K}; ++kk) w{i}[kk] = {op_expr(i, wref)};")
                wname[i] = f"w{i}"
            emitted.add(i)

    def vector_body(targets, indent, extra=()):
        """Opens the element loop (lane-owned column chunks jj when structured, a strided
        stream otherwise) and emits the statements for the V nodes `targets` need; returns
        (name map, indent of the loop body)."""
        need = set()
        stack = list(targets)
        while stack:
            j = stack.pop()
            if j in need or kinds[j] != "V":
                continue
            need.add(j)
            kind, o, a, b = nodes[j]
            if kind != "in":
                stack.extend([a] if kind == "u" else [a, b])
        names = dict(sname)
        if structured:
            w(f"{indent}#pragma unroll")
            w(f"{indent}for (int jj = 0; jj < {J}; ++jj) {{")
            w(f"{indent}  const sysml_i64 d0 = ((sysml_i64)lane + (sysml_i64)jj * L) * {vec};")
            w(f"{indent}  if (d0 < D) {{")
        else:
            w(f"{indent}{{")
            w(f"{indent}  for (sysml_i64 d0 = (sysml_i64)lane * {vec}; d0 < D; d0 += (sysml_i64)L * {vec}) {{")
        for k in sorted({j for j in need if j < n_in} | set(extra)):
            if modes[k] == SIDEM:
                continue
            if k in cache and structured:
                names[k] = f"xr{k}[jj][u]"
                continue
            base = "rowoff + d0" if modes[k] == FULL else "d0"
            w(f"{indent}    T x{k}[{vec}]; sysml_ldv{vec}<T>(A.in[{k}], {dts[k]}, {base}, x{k});")
            names[k] = f"x{k}[u]"
        w(f"{indent}    #pragma unroll")
        w(f"{indent}    for (int u = 0; u < {vec}; ++u) {{")
        w(f"{indent}      const sysml_i64 d = d0 + u; (void)d;")
        ind = indent + "      "
        for j in sorted(need):
            kind, o, a, b = nodes[j]
            if kind == "in":
                continue
            w(f"{ind}const T e{j} = {op_expr(j, lambda x: names[x])};")
            names[j] = f"e{j}"
        return names, ind

    def close_loop(indent):
        w(f"{indent}    }}")
        w(f"{indent}  }}")
        w(f"{indent}}}")

    pending = set(range(len(outs)))
    nphase = max(finals + [p + 1 for p in red_phase.values()])
    for p in range(nphase + 1):
        emit_values(p)
        reds = [i for i, q in red_phase.items() if q == p]
        if reds:
            for i in reds:
                kind, o, a, b = nodes[i]
                if kinds[i] == "W":
                    w(f"    T a{i}[{widths[i]}];")
                    w(f"    for (int kk = 0; kk < {widths[i]}; ++kk) a{i}[kk] = T(0);")
                else:
                    w(f"    T a{i} = {_RAGG_INIT[o] if kind == 'ragg' else 'T(0)'};")
            names, ind = vector_body([nodes[i][2] for i in reds], "    ",
                                     sorted({nodes[i][3] for i in reds if nodes[i][0] == "dot"}))
            for i in reds:
                kind, o, a, b = nodes[i]
                if kind == "dot" and kinds[i] == "W":
                    w(f"{ind}#pragma unroll")
                    w(f"{ind}for (int kk = 0; kk < {widths[i]}; ++kk) a{i}[kk] += {names[a]} * {smat[b]('d', 'kk')};")
                elif kind == "dot":
                    w(f"{ind}a{i} += {names[a]} * {names[b]};")
                else:
                    w(ind + _acc_step(o, f"a{i}", names[a]))
            close_loop("    ")
            for i in reds:
                kind, o, a, b = nodes[i]
                if kinds[i] == "W":
                    w("    #pragma unroll")
                    w(f"    for (int kk = 0; kk < {widths[i]}; ++kk)")
                    w(f"      for (int off = L / 2; off >= 1; off >>= 1) a{i}[kk] += __shfl_xor(a{i}[kk], off, L);")
                    wname[i] = f"a{i}"
                else:
                    oo = "sum" if kind == "dot" else o
                    w(f"    for (int off = L / 2; off >= 1; off >>= 1) a{i} = {_comb(oo, f'a{i}', f'__shfl_xor(a{i}, off, L)')};")
                    if kind == "ragg" and o == "mean":
                        w(f"    a{i} /= (T)D;")
                    sname[i] = f"a{i}"
                emitted.add(i)
        now = [q for q in sorted(pending) if finals[q] == p]
        if not now:
            continue
        emit_values(p)
        vtargets, vextra = [], []
        for q in now:
            node, ot, oagg, extra = outs[q]
            ko = kinds[node]
            if ko == "S":
                if ot in ("row", "vec"):
                    w(f"    if (lane == 0) static_cast<T*>(A.out[{q}])[row] = {sname[node]};")
                else:            # all
                    w(f"    if (lane == 0) {{ {_acc_step(oagg, f'tot{q}', sname[node])} }}")
            elif ko == "W":
                K = widths[node]
                if ot in ("row", "vec"):
                    w("    #pragma unroll")
                    w(f"    for (int kk = 0; kk < {K}; ++kk)")
                    w(f"      if ((kk % L) == lane) static_cast<T*>(A.out[{q}])[row * {K} + kk] = {wname[node]}[kk];")
                elif ot == "all":
                    w("    if (lane == 0) {")
                    w("      #pragma unroll")
                    w(f"      for (int kk = 0; kk < {K}; ++kk) {{ {_acc_step(oagg, f'tot{q}', f'{wname[node]}[kk]')} }}")
                    w("    }")
                else:            # col of a W
                    step = f"{wname[node]}[kk]" + (f" * {wname[node]}[kk]" if oagg == "sumsq" else "")
                    w("    if (lane == 0) {")
                    w("      #pragma unroll")
                    w(f"      for (int kk = 0; kk < {K}; ++kk) cw{q}[kk] += {step};")
                    w("    }")
            else:
                vtargets.append(q)
                if ot == "tmv":
                    vextra.append(extra)
            pending.discard(q)
        if vtargets:
            names, ind = vector_body([outs[q][0] for q in vtargets], "    ")
            for q in vtargets:
                node, ot, oagg, extra = outs[q]
                v = names[node]
                if ot == "vec" or ot == "row":
                    w(f"{ind}static_cast<T*>(A.out[{q}])[rowoff + d] = {v};")
                elif ot == "all":
                    w(ind + _acc_step(oagg, f"tot{q}", v))
                elif ot == "col":
                    cval = f"{v}{(' * ' + v) if oagg == 'sumsq' else ''}"
                    if creg:
                        w(f"{ind}racc[jj][u] += {cval};")
                    else:
                        col_add(ind, cval)
                elif kinds[extra] == "W":
                    w(f"{ind}#pragma unroll")
                    w(f"{ind}for (int kk = 0; kk < {KW}; ++kk)")
                    if creg:
                        w(f"{ind}  racc[jj][u][kk] += {v} * {wname[extra]}[kk];")
                    else:
                        col_add(ind + "  ", f"{v} * {wname[extra]}[kk]", "kk")
                else:
                    cval = f"{v} * {sname[extra]}"
                    if creg:
                        w(f"{ind}racc[jj][u] += {cval};")
                    else:
                        col_add(ind, cval)
            close_loop("    ")
        if not pending:
            break
    w("  }")
    # ---- per-workgroup partials of the aggregated outputs
    if ca is not None:
        q = outs.index(ca)
        if creg and ca_w:
            w(f"  __shared__ T acc[1][{dcap * KW}];")
            w(f"  for (int q = tid; q < {dcap * KW}; q += 256) acc[0][q] = T(0);")
            w("  __syncthreads();")
            w("  for (int g = 0; g < G; ++g) {")
            w("    if (grp == g) {")
            w("      #pragma unroll")
            w(f"      for (int jj = 0; jj < {J}; ++jj)")
            w("      #pragma unroll")
            w(f"      for (int u = 0; u < {vec}; ++u) {{")
            w(f"        const sysml_i64 d = ((sysml_i64)lane + (sysml_i64)jj * L) * {vec} + u;")
            w("        #pragma unroll")
            w(f"        for (int kk = 0; kk < {KW}; ++kk)")
            w(f"          if (d < D) acc[0][d * {KW} + kk] += racc[jj][u][kk];")
            w("      }")
            w("    }")
            w("    __syncthreads();")
            w("  }")
            w(f"  for (sysml_i64 d = tid; d < D * {KW}; d += 256) A.part[{q}][(sysml_i64)blockIdx.x * D * {KW} + d] = (double)acc[0][d];")
        elif creg:
            # merge the row groups' register accumulators in a fixed order (deterministic)
            w(f"  __shared__ T acc[1][{dcap}];")
            w(f"  for (int q = tid; q < {dcap}; q += 256) acc[0][q] = T(0);")
            w("  __syncthreads();")
            w("  for (int g = 0; g < G; ++g) {")
            w("    if (grp == g) {")
            w("      #pragma unroll")
            w(f"      for (int jj = 0; jj < {J}; ++jj)")
            w("      #pragma unroll")
            w(f"      for (int u = 0; u < {vec}; ++u) {{")
            w(f"        const sysml_i64 d = ((sysml_i64)lane + (sysml_i64)jj * L) * {vec} + u;")
            w("        if (d < D) acc[0][d] += racc[jj][u];")
            w("      }")
            w("    }")
            w("    __syncthreads();")
            w("  }")
            w(f"  for (sysml_i64 d = tid; d < D; d += 256) A.part[{q}][(sysml_i64)blockIdx.x * D + d] = (double)acc[0][d];")
        else:
            w("  __syncthreads();")
            w(f"  for (sysml_i64 d = tid; d < D * {KW}; d += 256) {{")
            w("    double s = 0.0;")
            w(f"    for (int g = 0; g < {S}; ++g) s += (double)acc[g][d];")
            w(f"    A.part[{q}][(sysml_i64)blockIdx.x * D * {KW} + d] = s;")
            w("  }")
    nred = sum(1 for o in outs if o[1] == "all" or (o[1] == "col" and kinds[o[0]] == "W"))
    if nred:
        w("  __shared__ double red[4];")
    for q, (node, ot, oagg, extra) in enumerate(outs):
        if ot == "all":
            w("  {")
            w(f"    double t = (double)tot{q};")
            w(f"    for (int off = 32; off >= 1; off >>= 1) t = sysml_acc_comb({_AGGC[oagg]}, t, __shfl_xor(t, off, 64));")
            w("    __syncthreads();")
            w("    if ((tid & 63) == 0) red[tid >> 6] = t;")
            w("    __syncthreads();")
            w("    if (tid == 0) {")
            w("      double r = red[0];")
            w(f"      for (int q = 1; q < 4; ++q) r = sysml_acc_comb({_AGGC[oagg]}, r, red[q]);")
            w(f"      A.part[{q}][blockIdx.x] = r;")
            w("    }")
            w("  }")
        elif ot == "col" and kinds[node] == "W":
            K = widths[node]
            w("  #pragma unroll")
            w(f"  for (int kk = 0; kk < {K}; ++kk) {{")
            w(f"    double t = (double)cw{q}[kk];")
            w("    for (int off = 32; off >= 1; off >>= 1) t += __shfl_xor(t, off, 64);")
            w("    __syncthreads();")
            w("    if ((tid & 63) == 0) red[tid >> 6] = t;")
            w("    __syncthreads();")
            w(f"    if (tid == 0) A.part[{q}][(sysml_i64)blockIdx.x * {K} + kk] = red[0] + red[1] + red[2] + red[3];")
            w("  }")
    w("}")
    return _prelude() + _ROW_PRELUDE + "\n".join(out) + "\n"


_ROW_PRELUDE = r"""
template <typename T>
__device__ __forceinline__ void sysml_ldv1(const void* p, int dt, sysml_i64 off, T (&o)[1]) {
  o[0] = sysml_ld<T>(p, dt, off);
}
// vector loads of VEC adjacent elements (off a multiple of VEC, base 16-byte aligned)
template <typename T>
__device__ __forceinline__ void sysml_ldv4(const void* p, int dt, sysml_i64 off, T (&o)[4]) {
  if (dt == 0) {
    const float4 q = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + off);
    o[0] = (T)q.x; o[1] = (T)q.y; o[2] = (T)q.z; o[3] = (T)q.w;
  } else if (dt == 1) {
    const double2 a = *reinterpret_cast<const double2*>(static_cast<const double*>(p) + off);
    const double2 b = *reinterpret_cast<const double2*>(static_cast<const double*>(p) + off + 2);
    o[0] = (T)a.x; o[1] = (T)a.y; o[2] = (T)b.x; o[3] = (T)b.y;
  } else {
    const uint2 q = *reinterpret_cast<const uint2*>(static_cast<const unsigned short*>(p) + off);
    o[0] = (T)sysml_bf2f(q.x & 0xffff); o[1] = (T)sysml_bf2f(q.x >> 16);
    o[2] = (T)sysml_bf2f(q.y & 0xffff); o[3] = (T)sysml_bf2f(q.y >> 16);
  }
}
template <typename T>
__device__ __forceinline__ void sysml_ldv8(const void* p, int dt, sysml_i64 off, T (&o)[8]) {
  if (dt == 2) {
    const uint4 q = *reinterpret_cast<const uint4*>(static_cast<const unsigned short*>(p) + off);
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[2 * i] = (T)sysml_bf2f(w[i] & 0xffff); o[2 * i + 1] = (T)sysml_bf2f(w[i] >> 16); }
  } else {
    T a[4], b[4];
    sysml_ldv4<T>(p, dt, off, a);
    sysml_ldv4<T>(p, dt, off + 4, b);
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[i] = a[i]; o[4 + i] = b[i]; }
  }
}
"""

_ROW_PRELUDE += r"""
// raw (unconverted) vector chunks: the next row's loads stay in flight in these registers and
// are converted only when the row is reached (a conversion right after the load would wait)
template <int DT, int V> struct SysmlRaw;
template <> struct SysmlRaw<2, 8> {
  uint4 q;
  __device__ __forceinline__ void load(const void* p, sysml_i64 off) {
    q = *reinterpret_cast<const uint4*>(static_cast<const unsigned short*>(p) + off);
  }
  template <typename T> __device__ __forceinline__ void get(T (&o)[8]) const {
    const unsigned w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) { o[2 * i] = (T)sysml_bf2f(w[i] & 0xffff); o[2 * i + 1] = (T)sysml_bf2f(w[i] >> 16); }
  }
};
template <> struct SysmlRaw<2, 4> {
  uint2 q;
  __device__ __forceinline__ void load(const void* p, sysml_i64 off) {
    q = *reinterpret_cast<const uint2*>(static_cast<const unsigned short*>(p) + off);
  }
  template <typename T> __device__ __forceinline__ void get(T (&o)[4]) const {
    o[0] = (T)sysml_bf2f(q.x & 0xffff); o[1] = (T)sysml_bf2f(q.x >> 16);
    o[2] = (T)sysml_bf2f(q.y & 0xffff); o[3] = (T)sysml_bf2f(q.y >> 16);
  }
};
template <> struct SysmlRaw<2, 1> {
  unsigned short q;
  __device__ __forceinline__ void load(const void* p, sysml_i64 off) { q = static_cast<const unsigned short*>(p)[off]; }
  template <typename T> __device__ __forceinline__ void get(T (&o)[1]) const { o[0] = (T)sysml_bf2f(q); }
};
template <> struct SysmlRaw<0, 4> {
  float4 q;
  __device__ __forceinline__ void load(const void* p, sysml_i64 off) {
    q = *reinterpret_cast<const float4*>(static_cast<const float*>(p) + off);
  }
  template <typename T> __device__ __forceinline__ void get(T (&o)[4]) const {
    o[0] = (T)q.x; o[1] = (T)q.y; o[2] = (T)q.z; o[3] = (T)q.w;
  }
};
template <> struct SysmlRaw<0, 1> {
  float q;
  __device__ __forceinline__ void load(const void* p, sysml_i64 off) { q = static_cast<const float*>(p)[off]; }
  template <typename T> __device__ __forceinline__ void get(T (&o)[1]) const { o[0] = (T)q; }
};
template <> struct SysmlRaw<1, 4> {
  double2 a, b;
  __device__ __forceinline__ void load(const void* p, sysml_i64 off) {
    a = *reinterpret_cast<const double2*>(static_cast<const double*>(p) + off);
    b = *reinterpret_cast<const double2*>(static_cast<const double*>(p) + off + 2);
  }
  template <typename T> __device__ __forceinline__ void get(T (&o)[4]) const {
    o[0] = (T)a.x; o[1] = (T)a.y; o[2] = (T)b.x; o[3] = (T)b.y;
  }
};
template <> struct SysmlRaw<1, 1> {
  double q;
  __device__ __forceinline__ void load(const void* p, sysml_i64 off) { q = static_cast<const double*>(p)[off]; }
  template <typename T> __device__ __forceinline__ void get(T (&o)[1]) const { o[0] = (T)q; }
};
"""

_AGGC = {"sum": 0, "mean": 0, "sumsq": 0, "min": 2, "max": 3}   # partials of sumsq are already squared


class _RowArgs(ctypes.Structure):
    _fields_ = [("inp", ctypes.c_void_p * MAXIN), ("s", ctypes.c_double * MAXIN), ("rows", ctypes.c_int64),
                ("cols", ctypes.c_int64), ("out", ctypes.c_void_p * MAXOUT), ("part", ctypes.c_void_p * MAXOUT)]


_funcs = {}


def _func(prog, T, modes, dts, kinds, L, dcap, vec, slices, J, cache, dev, widths):
    key = (prog.key(), T, modes, dts, L, dcap, vec, slices, J, cache, str(dev), widths)
    f = _funcs.get(key, False)
    if f is not False:
        return f
    src = generate(prog, T, modes, dts, kinds, L, dcap, vec, slices, J, cache, widths)
    code = compile_source(src, gpu_arch(dev))        # raises on a compile error: a generator bug
    fn = ctypes.c_void_p()
    cbuf = ctypes.create_string_buffer(code, len(code))
    rc = _rtc_lib().sysml_rtc_load(cbuf, b"sysml_row_k", ctypes.byref(fn))
    if rc != 0:
        raise RuntimeError(f"hipModuleLoadData failed ({rc})")
    stats["compiled"] += 1
    f = (fn, cbuf)
    _funcs[key] = f
    return f


class _Plan:
    __slots__ = ("prog", "fn", "kinds", "N", "D", "T", "nblk", "outs", "dev", "dev_index", "launch", "count")


MIN_LANES = 32768          # fewer lanes in flight than this on a large input: torch's reductions win


def _make_plan(prog: RowProgram, args):
    from ..runtime.scalars import DevScalar
    if len(args) != prog.n_in or prog.n_in > MAXIN or len(prog.ops) > MAXOPS or len(prog.outputs()) > MAXOUT:
        return None
    dev = None
    shapes = []
    f64 = bf16 = False
    for x in args:
        tx = type(x)
        if tx is _Tensor:
            if not x.is_cuda or x.layout is not torch.strided or x.dim() != 2 or x.dtype not in _DT:
                return None
            if dev is None:
                dev = x.device
            elif x.device != dev:
                return None
            f64 = f64 or x.dtype == torch.float64
            bf16 = bf16 or x.dtype == torch.bfloat16
            shapes.append(tuple(x.shape))
        elif tx is DevScalar:
            if not x.t.is_cuda or x.t.dtype not in _DT:
                return None
            shapes.append(None)
        else:
            shapes.append(None)
    if dev is None:
        return None
    cl = classify(prog, shapes)
    if cl is None:
        return None
    N, D, modes, kinds, widths = cl
    # DevScalar inputs are device-resident 1 x 1 values
    modes = tuple(DSCALAR if type(x) is DevScalar else m for x, m in zip(args, modes))
    T = torch.float64 if (f64 or (bf16 and backend.dtype == torch.float64)) else torch.float32
    outs = prog.outputs()
    ca = _colacc_output(prog, kinds)
    dcap = dcap_for(D) if (ca is not None or any(m == SIDEM for m in modes)) else 0
    if (ca is not None or any(m == SIDEM for m in modes)) and dcap is None:
        return None
    if ca is not None and ca[1] == "tmv" and kinds[ca[3]] == "W" and \
            dcap * widths[ca[3]] * (4 if T == torch.float32 else 8) > LDS_BYTES:
        return None
    dts, akinds, aligned = [], [], True
    for k, x in enumerate(args):
        tx = type(x)
        if tx is _Tensor:
            dts.append(_DT[x.dtype])
            akinds.append("t")
            if modes[k] in (FULL, ROWV, SIDE) and not (x.is_contiguous() and x.data_ptr() % 16 == 0):
                aligned = False
        elif tx is DevScalar:
            dts.append(_DT[x.t.dtype])
            akinds.append("d")
        else:
            dts.append(0)
            akinds.append("s")
    dts = tuple(dts)
    vec = 1
    vleaves = [k for k, m in enumerate(modes) if m in (FULL, ROWV, SIDE)]
    if aligned:
        if D % 8 == 0 and any(dts[k] == 2 and modes[k] == FULL for k in vleaves) and \
                all(dts[k] == 2 for k in vleaves if modes[k] == FULL):
            vec = 8          # bf16 rows: 16-byte loads (other vectors as two 16-byte loads)
        elif D % 4 == 0:
            vec = 4
    L = lanes_for((D + vec - 1) // vec)
    G = 256 // L
    if N * L < MIN_LANES and N * D >= (1 << 20):
        return None                     # a few very long rows: too little parallelism per row
    slices = G
    J, cache = plan_registers(prog, modes, kinds, D, L, vec, T, dcap, dts, widths)
    if ca is not None and "acc" not in cache:
        kw = widths[ca[3]] if (ca[1] == "tmv" and kinds[ca[3]] == "W") else 1
        slices = lds_slices(G, dcap * kw, T) if kw == 1 else 1
        if slices == 0:
            return None
    f = _func(prog, T, modes, dts, kinds, L, dcap, vec, slices, J, cache, dev, widths)
    ngrp = (N + G - 1) // G
    pl = _Plan()
    pl.prog, pl.fn, pl.kinds, pl.N, pl.D, pl.T, pl.dev = prog, f[0], akinds, N, D, T, dev
    pl.dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
    agg_out = any(o[1] in ("col", "tmv", "all") for o in outs)
    pl.nblk = max(1, min(ngrp, 1024 if ca is not None else (2048 if agg_out else 16384)))
    # per output: (type, kind, width, aggregate, extra width)
    pl.outs = tuple((ot, kinds[node], widths[node], oagg, widths[extra] if ot == "tmv" and kinds[extra] == "W" else 0)
                    for node, ot, oagg, extra in outs)
    pl.launch = _rtc_lib().sysml_rtc_launch
    from . import kernels
    pl.count = kernels._count
    return pl


_plans = {}


_spec = {}


def _specialise(prog, args):
    """prog with every run-time column bound (wcolsv: X[, 1:k], k a scalar operand) replaced by
    its value, or None when a bound is not a host integer in range."""
    if not any(k == "wcolsv" for k, _, _, _ in prog.ops):
        return prog, ()
    bounds = []
    for kind, _, _, b in prog.ops:
        if kind == "wcolsv":
            v = args[b] if b < prog.n_in else None
            if type(v) not in (int, float) or v != int(v) or not 1 <= int(v) <= MAXW:
                return None, None
            bounds.append(int(v))
    key = (id(prog), tuple(bounds))
    sp = _spec.get(key)
    if sp is None or sp[0] is not prog:
        it = iter(bounds)
        ops = [("wcols", None, a, next(it)) if k == "wcolsv" else (k, o, a, b) for k, o, a, b in prog.ops]
        sp = _spec[key] = (prog, RowProgram(prog.n_in, ops, prog.out, prog.otype, prog.oagg, prog.extra, prog.more))
    return sp[1], tuple(bounds)


def _kernel(prog: RowProgram, args):
    """One launch of the generated row kernel, or None when the operands are outside its scope
    (launch plans cached per program and operand signature)."""
    sig = _signature(args)
    if sig is None:
        return None
    prog, bounds = _specialise(prog, args)
    if prog is None:
        return None
    key = (id(prog), sig, bounds)
    pl = _plans.get(key, False)
    if pl is False or (pl is not None and pl.prog is not prog):
        pl = _make_plan(prog, args)
        _plans[key] = pl
    if pl is None:
        return None
    N, D, T, dev, nblk = pl.N, pl.D, pl.T, pl.dev, pl.nblk
    A = _RowArgs()
    keep = []
    for k, (x, kd) in enumerate(zip(args, pl.kinds)):
        if kd == "t":
            if not x.is_contiguous():
                x = x.contiguous()
                keep.append(x)
            A.inp[k] = x.data_ptr()
        elif kd == "d":
            t = x.t.reshape(1)
            keep.append(t)
            A.inp[k] = t.data_ptr()
        else:
            A.s[k] = float(x)
    bufs = []
    for q, (ot, kind, width, oagg, xw) in enumerate(pl.outs):
        out = part = None
        if ot in ("row", "vec"):
            out = torch.empty((N, D) if kind == "V" else ((N, width) if kind == "W" else (N, 1)), dtype=T, device=dev)
        elif ot == "col":
            part = torch.empty((nblk, D if kind == "V" else width), dtype=torch.float64, device=dev)
        elif ot == "tmv":
            part = torch.empty((nblk, D * max(xw, 1)), dtype=torch.float64, device=dev)
        else:
            part = torch.empty(nblk, dtype=torch.float64, device=dev)
        A.out[q] = out.data_ptr() if out is not None else 0
        A.part[q] = part.data_ptr() if part is not None else 0
        bufs.append((out, part))
    A.rows, A.cols = N, D
    st = _raw_stream(pl.dev_index) if _raw_stream is not None else torch.cuda.current_stream(dev).cuda_stream
    rc = pl.launch(pl.fn, nblk, 1, 256, ctypes.byref(A), ctypes.sizeof(A), st)
    if rc != 0:
        raise RuntimeError(f"generated row kernel launch failed: {rc}")
    pl.count("row")
    del keep
    res = []
    for (ot, kind, width, oagg, xw), (out, part) in zip(pl.outs, bufs):
        if out is not None:
            res.append(out)
        elif ot == "col":
            r = part.sum(0, keepdim=True).to(T)
            if oagg == "mean":
                r = r / N
            res.append(r)
        elif ot == "tmv":
            res.append(part.sum(0).to(T).reshape(D, max(xw, 1)))
        else:
            r = part.sum() if oagg in ("sum", "sumsq", "mean") else (part.min() if oagg == "min" else part.max())
            if oagg == "mean":
                r = r / (N * (D if kind == "V" else (width if kind == "W" else 1)))
            res.append(C._lazy_out(r))
    return tuple(res) if prog.more else res[0]
