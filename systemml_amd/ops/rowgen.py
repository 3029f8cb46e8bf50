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
MAXIN, MAXOPS = 8, 48
LDS_BYTES = 65536
stats = {"kernel": 0, "sequential": 0, "compiled": 0}

FULL, ROWV, COLV, HSCALAR, DSCALAR, SIDE = range(6)


class RowProgram:
    """ops: tuple of (kind, op, a, b) over node indices -- inputs are nodes 0..n_in-1, op j is
    node n_in + j; kind 'b' (binary), 'u' (unary, 'sq' = x^2), 'ragg' (row aggregate `op` of
    node a), 'dot' (node a %*% input b, b a D x 1 side vector).  out: output node; otype / oagg:
    output type and its aggregate; extra: the S node of a 'tmv' output."""
    __slots__ = ("n_in", "ops", "out", "otype", "oagg", "extra")

    def __init__(self, n_in, ops, out, otype, oagg=None, extra=None):
        if otype not in OTYPES:
            raise ValueError(otype)
        self.n_in = n_in
        self.ops = tuple(tuple(x) for x in ops)
        self.out = out
        self.otype = otype
        self.oagg = oagg
        self.extra = extra

    def key(self):
        return (self.n_in, self.ops, self.out, self.otype, self.oagg, self.extra)

    def __eq__(self, other):
        return isinstance(other, RowProgram) and self.key() == other.key()

    def __hash__(self):
        return hash(self.key())

    def side_inputs(self):
        return {b for kind, _, _, b in self.ops if kind == "dot"}

    def describe(self):
        body = ",".join(("dot" if k == "dot" else (f"r{o}" if k == "ragg" else o)) for k, o, _, _ in self.ops)
        tail = {"row": "", "vec": "", "col": f"|col{self.oagg}", "tmv": "|t(.)%*%", "all": f"|{self.oagg}"}[self.otype]
        return f"row[{body}]{tail}"

    def __repr__(self):
        return self.describe()


def sequential(prog: RowProgram, args):
    """The fused DAG's original operators, one after the other."""
    vals = list(args)
    for kind, o, a, b in prog.ops:
        if kind == "b":
            v = C.binary(o, vals[a], vals[b])
        elif kind == "u":
            v = C.binary("^", vals[a], 2) if o == "sq" else C.unary(o, vals[a])
        elif kind == "ragg":
            v = C.agg(o, "row", vals[a])
        else:
            v = C.mm(vals[a], vals[b], False)
        vals.append(v)
    r = vals[prog.out]
    ot = prog.otype
    if ot == "col":
        return C.agg(prog.oagg, "col", r)
    if ot == "all":
        return C.agg(prog.oagg, "all", r)
    if ot == "tmv":
        return C.mm(r, vals[prog.extra], True)
    return r


def evaluate(prog: RowProgram, args):
    r = _kernel(prog, args) if backend.use_kernels else None
    if r is not None:
        stats["kernel"] += 1
        return r
    stats["sequential"] += 1
    return sequential(prog, args)


# ----------------------------------------------------------------------------- classification
def classify(prog: RowProgram, shapes):
    """shapes: per input (rows, cols) or None (scalar).  Returns (N, D, leaf modes, node kinds)
    or None when the operands are outside the kernel's scope."""
    side = prog.side_inputs()
    D = 0
    N = 1
    for k, s in enumerate(shapes):
        if s is None or k in side:
            continue
        r, c = s
        if c > 1:
            if D and c != D:
                return None
            D = c
        if r > 1:
            if N > 1 and r != N:
                return None
            N = r
    if D <= 1:
        return None
    modes = []
    for k, s in enumerate(shapes):
        if k in side:
            if s is None or s != (D, 1):
                return None
            modes.append(SIDE)
            continue
        if s is None:
            modes.append(HSCALAR)
            continue
        r, c = s
        if (r, c) == (N, D) and N > 1:
            modes.append(FULL)
        elif r == 1 and c == D:
            modes.append(ROWV)
        elif c == 1 and r == N and N > 1:
            modes.append(COLV)
        elif r == 1 and c == 1:
            modes.append(DSCALAR)
        else:
            return None
    kinds = []
    for m in modes:
        kinds.append("V" if m in (FULL, ROWV) else ("S" if m == COLV else ("X" if m == SIDE else "C")))
    for kind, o, a, b in prog.ops:
        ka = kinds[a]
        if kind == "b":
            kb = kinds[b]
            if "X" in (ka, kb):
                return None
            kinds.append("V" if "V" in (ka, kb) else ("S" if "S" in (ka, kb) else "C"))
        elif kind == "u":
            if ka == "X":
                return None
            kinds.append(ka)
        elif kind == "ragg":
            if ka not in ("V", "S"):
                return None
            kinds.append("S")
        else:
            if ka != "V" or kinds[b] != "X":
                return None
            kinds.append("S")
    ko = kinds[prog.out]
    ot = prog.otype
    if ot in ("row", "vec") and ko not in ("V", "S"):
        return None
    if ot == "col" and ko != "V":
        return None
    if ot == "tmv" and (ko != "V" or kinds[prog.extra] != "S"):
        return None
    if ot == "all" and ko not in ("V", "S"):
        return None
    return N, D, tuple(modes), tuple(kinds)


def out_shape(prog: RowProgram, shapes):
    """Result shape for input shapes (None: scalar) under the original operators' rules; None
    if an operator would reject its operands or the result is a scalar."""
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
        else:
            sb = v[b]
            if sa is None or sb is None or sa[1] != sb[0]:
                return None
            v.append((sa[0], sb[1]))
    r = v[prog.out]
    if r is None:
        return None
    ot = prog.otype
    if ot == "col":
        return (1, r[1])
    if ot == "tmv":
        e = v[prog.extra]
        return None if e is None or e[0] != r[0] else (r[1], e[1])
    return r


REG_BUDGET = 96            # cached fp32 values per lane (fp64 count twice)


def plan_registers(prog, modes, kinds, D, L, vec, T, dcap, dts=None):
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
    if prog.otype in ("col", "tmv") and dcap and dcap * (4 if T == torch.float32 else 8) <= LDS_BYTES:
        cache.append("acc")
        used += per
    vecuse = set()
    for kind, o, a, b in prog.ops:
        for x in ((a, b) if kind in ("b", "dot") else (a,)):
            if x < prog.n_in and modes[x] in (FULL, ROWV, SIDE):
                vecuse.add(x)
    if prog.out < prog.n_in and modes[prog.out] in (FULL, ROWV, SIDE):
        vecuse.add(prog.out)
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


def generate(prog: RowProgram, T, modes, dts, kinds, L, dcap, vec=1, slices=None, J=0, cache=frozenset()):
    """HIP source of the fused row kernel (see the module docstring for the phase structure)."""
    ct = "float" if T == torch.float32 else "double"
    n_in = prog.n_in
    G = 256 // L
    nodes = [("in", None, k, None) for k in range(n_in)] + list(prog.ops)
    # phase availability: a reduction over a V runs in the phase its input is complete in and
    # its result is available from the next phase on
    avail, red_phase = [], {}
    for i, (kind, o, a, b) in enumerate(nodes):
        if kind == "in":
            avail.append(0)
        elif kind in ("ragg", "dot") and kinds[a] == "V":
            red_phase[i] = avail[a]
            avail.append(avail[a] + 1)
        elif kind == "b":
            avail.append(max(avail[a], avail[b]))
        else:
            avail.append(avail[a])
    ot = prog.otype
    vec_out = kinds[prog.out] == "V"
    final = avail[prog.out] if ot != "tmv" else max(avail[prog.out], avail[prog.extra])

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
    w("struct SysmlRowArgs { const void* in[8]; double s[8]; sysml_i64 rows, cols; void* out; double* part; };")
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
    colacc = ot in ("col", "tmv")
    S = G if slices is None else slices
    structured = J > 0
    creg = colacc and structured and "acc" in cache
    if creg:
        w(f"  T racc[{J}][{vec}];")
        w("  #pragma unroll")
        w(f"  for (int jj = 0; jj < {J}; ++jj)")
        w("    #pragma unroll")
        w(f"    for (int u = 0; u < {vec}; ++u) racc[jj][u] = T(0);")
    elif colacc:
        w(f"  __shared__ T acc[{S}][{dcap}];")
        w(f"  for (int q = tid; q < {S} * {dcap}; q += 256) (&acc[0][0])[q] = T(0);")
        w("  __syncthreads();")

    def col_add(ind, val):
        if S == G:
            w(f"{ind}acc[grp][d] += {val};")
        else:
            w(f"{ind}atomicAdd(&acc[0][d], {val});")

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
    if ot == "all":
        w(f"  T tot = {_RAGG_INIT[prog.oagg]};")
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
    for k in range(n_in):
        if kinds[k] == "S":
            w(f"    const T s{k} = sysml_ld<T>(A.in[{k}], {dts[k]}, row);")
            sname[k] = f"s{k}"
    # the row itself: every N x D input read ONCE from HBM into registers, reused by all phases
    for k in range(n_in):
        if modes[k] == FULL and k in cache and k not in piped:
            load_cached(k, "rowoff + d0", "    ")

    def sref(j):
        return sname[j]

    emitted = set(range(n_in)) | set(cname)

    def emit_scalars(p):
        for i in range(n_in, len(nodes)):
            if i in emitted or kinds[i] != "S" or i in red_phase or avail[i] > p:
                continue
            w(f"    const T s{i} = {op_expr(i, sref)};")
            sname[i] = f"s{i}"
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

    nphase = max([final] + [p + 1 for p in red_phase.values()])
    for p in range(nphase + 1):
        emit_scalars(p)
        reds = [i for i, q in red_phase.items() if q == p]
        if reds:
            for i in reds:
                kind, o, a, b = nodes[i]
                w(f"    T a{i} = {_RAGG_INIT[o] if kind == 'ragg' else 'T(0)'};")
            names, ind = vector_body([nodes[i][2] for i in reds], "    ",
                                     sorted({nodes[i][3] for i in reds if nodes[i][0] == "dot"}))
            for i in reds:
                kind, o, a, b = nodes[i]
                if kind == "dot":
                    w(f"{ind}a{i} += {names[a]} * {names[b]};")
                else:
                    w(ind + _acc_step(o, f"a{i}", names[a]))
            close_loop("    ")
            for i in reds:
                kind, o, a, b = nodes[i]
                oo = "sum" if kind == "dot" else o
                w(f"    for (int off = L / 2; off >= 1; off >>= 1) a{i} = {_comb(oo, f'a{i}', f'__shfl_xor(a{i}, off, L)')};")
                if kind == "ragg" and o == "mean":
                    w(f"    a{i} /= (T)D;")
                sname[i] = f"a{i}"
                emitted.add(i)
        if p == final:
            emit_scalars(p)
            if ot in ("row", "vec") and not vec_out:
                w(f"    if (lane == 0) static_cast<T*>(A.out)[row] = {sname[prog.out]};")
            elif ot == "all" and not vec_out:
                w(f"    if (lane == 0) {{ {_acc_step(prog.oagg, 'tot', sname[prog.out])} }}")
            else:
                names, ind = vector_body([prog.out], "    ")
                v = names[prog.out]
                cval = f"{v}{(' * ' + v) if prog.oagg == 'sumsq' else ''}" if ot == "col" else \
                    (f"{v} * {sname[prog.extra]}" if ot == "tmv" else None)
                if creg:
                    w(f"{ind}racc[jj][u] += {cval};")
                elif colacc:
                    col_add(ind, cval)
                elif ot == "vec":
                    w(f"{ind}static_cast<T*>(A.out)[rowoff + d] = {v};")
                else:
                    w(ind + _acc_step(prog.oagg, "tot", v))
                close_loop("    ")
            break
    w("  }")
    if creg:
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
        w("  for (sysml_i64 d = tid; d < D; d += 256) A.part[(sysml_i64)blockIdx.x * D + d] = (double)acc[0][d];")
    elif colacc:
        w("  __syncthreads();")
        w("  for (sysml_i64 d = tid; d < D; d += 256) {")
        w("    double s = 0.0;")
        w(f"    for (int g = 0; g < {S}; ++g) s += (double)acc[g][d];")
        w("    A.part[(sysml_i64)blockIdx.x * D + d] = s;")
        w("  }")
    elif ot == "all":
        o = prog.oagg
        w("  double t = (double)tot;")
        w(f"  for (int off = 32; off >= 1; off >>= 1) t = sysml_acc_comb({_AGGC[o]}, t, __shfl_xor(t, off, 64));")
        w("  __shared__ double red[4];")
        w("  if ((tid & 63) == 0) red[tid >> 6] = t;")
        w("  __syncthreads();")
        w("  if (tid == 0) {")
        w(f"    double r = red[0];")
        w(f"    for (int q = 1; q < 4; ++q) r = sysml_acc_comb({_AGGC[o]}, r, red[q]);")
        w("    A.part[blockIdx.x] = r;")
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
                ("cols", ctypes.c_int64), ("out", ctypes.c_void_p), ("part", ctypes.c_void_p)]


_funcs = {}


def _func(prog, T, modes, dts, kinds, L, dcap, vec, slices, J, cache, dev):
    key = (prog.key(), T, modes, dts, L, dcap, vec, slices, J, cache, str(dev))
    f = _funcs.get(key, False)
    if f is not False:
        return f
    src = generate(prog, T, modes, dts, kinds, L, dcap, vec, slices, J, cache)
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
    __slots__ = ("prog", "fn", "kinds", "N", "D", "T", "nblk", "ot", "vec_out", "dev", "dev_index", "launch",
                 "count")


MIN_LANES = 32768          # fewer lanes in flight than this on a large input: torch's reductions win


def _make_plan(prog: RowProgram, args):
    from ..runtime.scalars import DevScalar
    if len(args) != prog.n_in or prog.n_in > MAXIN or len(prog.ops) > MAXOPS:
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
    N, D, modes, kinds = cl
    # DevScalar inputs are device-resident 1 x 1 values
    modes = tuple(DSCALAR if type(x) is DevScalar else m for x, m in zip(args, modes))
    T = torch.float64 if (f64 or (bf16 and backend.dtype == torch.float64)) else torch.float32
    ot = prog.otype
    dcap = 0
    if ot in ("col", "tmv"):
        dcap = dcap_for(D)
        if dcap is None:
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
    J, cache = plan_registers(prog, modes, kinds, D, L, vec, T, dcap, dts)
    if ot in ("col", "tmv") and "acc" not in cache:
        slices = lds_slices(G, dcap, T)
        if slices == 0:
            return None
    f = _func(prog, T, modes, dts, kinds, L, dcap, vec, slices, J, cache, dev)
    ngrp = (N + G - 1) // G
    pl = _Plan()
    pl.prog, pl.fn, pl.kinds, pl.N, pl.D, pl.T, pl.ot, pl.dev = prog, f[0], akinds, N, D, T, ot, dev
    pl.dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
    pl.nblk = max(1, min(ngrp, 1024 if ot in ("col", "tmv") else (2048 if ot == "all" else 16384)))
    pl.vec_out = kinds[prog.out] == "V"
    pl.launch = _rtc_lib().sysml_rtc_launch
    from . import kernels
    pl.count = kernels._count
    return pl


_plans = {}


def _kernel(prog: RowProgram, args):
    """One launch of the generated row kernel, or None when the operands are outside its scope
    (launch plans cached per program and operand signature)."""
    sig = _signature(args)
    if sig is None:
        return None
    key = (id(prog), sig)
    pl = _plans.get(key, False)
    if pl is False or (pl is not None and pl.prog is not prog):
        pl = _make_plan(prog, args)
        _plans[key] = pl
    if pl is None:
        return None
    N, D, T, ot, dev, nblk = pl.N, pl.D, pl.T, pl.ot, pl.dev, pl.nblk
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
    out = part = None
    if ot in ("row", "vec"):
        out = torch.empty((N, D) if pl.vec_out else (N, 1), dtype=T, device=dev)
    elif ot in ("col", "tmv"):
        part = torch.empty((nblk, D), dtype=torch.float64, device=dev)
    else:
        part = torch.empty(nblk, dtype=torch.float64, device=dev)
    A.rows, A.cols = N, D
    A.out = out.data_ptr() if out is not None else 0
    A.part = part.data_ptr() if part is not None else 0
    st = _raw_stream(pl.dev_index) if _raw_stream is not None else torch.cuda.current_stream(dev).cuda_stream
    rc = pl.launch(pl.fn, nblk, 1, 256, ctypes.byref(A), ctypes.sizeof(A), st)
    if rc != 0:
        raise RuntimeError(f"generated row kernel launch failed: {rc}")
    pl.count("row")
    del keep
    if out is not None:
        return out
    if ot in ("col", "tmv"):
        r = part.sum(0, keepdim=True).to(T)
        if ot == "col" and prog.oagg == "mean":
            r = r / N
        return r if ot == "col" else r.reshape(D, 1)
    o = prog.oagg
    r = part.sum() if o in ("sum", "sumsq", "mean") else (part.min() if o == "min" else part.max())
    if o == "mean":
        r = r / (N * (D if pl.vec_out else 1))
    return C._lazy_out(r)
