"""Vector programs: a basic block's small-matrix and scalar algebra as ONE single-workgroup
kernel (the "Vector" template of compiler/vecgen.py).

Iterative solvers spend their inner loop in two kinds of work: one or two passes over the
big data matrix (fused row-streaming / MFMA kernels) and a tail of updates on D x K solver
state and scalars -- in conjugate gradient `q += lambda * p; alpha = rr / sum(p * q);
beta += alpha * p; r += alpha * q; rr = sum(r ^ 2); p = -r + (rr / rr_old) * p` and the
convergence test.  Run operator by operator, that tail is a dozen launches and several
device round trips per iteration (reference: the per-instruction CP/GPU dispatch of
runtime/instructions/{cp,gpu}); with the state on the host it serialises the GPU behind
the host.  A VProgram runs the whole tail in one launch of 1024 threads (16 wave64s, one
CU): each thread owns a fixed set of cells, cellwise operators are straight-line code per
cell, every full aggregate is a per-thread partial + one LDS block reduction, and the
scalar algebra between reductions is evaluated (uniformly) by every thread.  Values that
cross a reduction barrier go through a scratch buffer the same thread re-reads (L2
resident), so register use does not grow with the matrix size.  All scalar results leave
the device in ONE copy at the end -- the single synchronisation an iterative loop needs
for its predicate.

The kernel source is generated per program and operand signature and compiled by hipRTC
(ops/hip/rtc.hip, cached by source hash like the Cell template's kernels).  Outside the
kernel's scope -- CPU backend, sparse / distributed / constant-column operands, shapes
that are not one common R x C (<= VMAX cells) plus scalars, string scalars, mixed-type
selects -- the program's original operators run one by one (with Cell-template fusion),
so semantics and error behaviour never change.
"""
from __future__ import annotations

import ctypes
import weakref

import torch

from .backend import backend
from ..utils import hosttrace as _HT
from .cell import (_C_BIN, _C_UN, BIN_CODES, UN_CODES, _prelude, compile_source, gpu_arch, _rtc_lib, RTC)

VMAX = 65536            # largest common cell count run as one workgroup
REG = __import__("os").environ.get("SYSML_VPROG_REG", "1") != "0"   # register-resident variant for small n
NT = 1024               # threads of the workgroup (16 wave64s)
REDS = ("sum", "sumsq", "min", "max", "mean", "dot", "dot3")

stats = {"kernel": 0, "fallback": 0, "compiled": 0}
_Tensor = torch.Tensor
_DT = {torch.float32: 0, torch.float64: 1}


class VProgram:
    """n_in leaves (dt 'M' | 'S'); instrs[k] = (kind, op, srcs) defines value n_in + k:
      kind 'm'  cellwise matrix operator (op in BIN_CODES / UN_CODES or 'sel' = cond ? a : b)
      kind 's'  scalar operator (same operator set)
      kind 'r'  full aggregate of matrix operands (sum / sumsq / min / max / mean over one,
                'dot' = sum(a * b), 'dot3' = sum(a * b * c))
    outs: the value ids the block reads afterwards, in output order."""

    def __init__(self, leaf_dts, instrs, outs, fallback_dag=None):
        self.leaf_dts = tuple(leaf_dts)
        self.instrs = tuple((k, o, tuple(s)) for k, o, s in instrs)
        self.outs = tuple(outs)
        self.fallback_dag = fallback_dag     # (placeholder names, clone output hops) -- ops run one by one
        self._fallback = None
        self._plans = {}
        n = len(self.leaf_dts)
        self.cls = list(self.leaf_dts) + ["S" if k in ("s", "r") else "M" for k, _, _ in self.instrs]
        # stages: a cellwise operator runs in the loop of the latest stage its inputs are
        # available in; a reduction's result is available one stage later (after the barrier)
        avail = [0] * (n + len(self.instrs))
        stage = [0] * (n + len(self.instrs))
        for k, (kind, o, srcs) in enumerate(self.instrs):
            v = n + k
            a = max((avail[s] for s in srcs), default=0)
            if kind == "r":
                stage[v] = a
                avail[v] = a + 1
            else:
                stage[v] = a
                avail[v] = a
        self.avail = avail
        self.stage = stage
        self.nstages = max([stage[n + k] + (1 if kind == "r" else 0) for k, (kind, _, _) in enumerate(self.instrs)],
                           default=0) + 1

    def describe(self):
        return "vprog[" + ",".join(o for _, o, _ in self.instrs) + "]"

    def __repr__(self):
        return self.describe()


# ----------------------------------------------------------------------------- typing
def _scalar_types(vp, leaf_types):
    """DML value types ('i' | 'd' | 'b') of every scalar value for the leaves' Python types
    (runtime/scalars.binary: INT op INT stays INT except '/' and '^'); None when an operator
    would leave the supported set (strings, mixed-type selects)."""
    t = list(leaf_types) + [None] * len(vp.instrs)
    n = len(vp.leaf_dts)
    for k, (kind, o, srcs) in enumerate(vp.instrs):
        if kind == "m":
            t[n + k] = "M"
            continue
        if kind == "r":
            t[n + k] = "d"
            continue
        ts = [t[s] for s in srcs]
        if any(x not in ("i", "d", "b") for x in ts):
            return None
        if o == "sel":
            if ts[1] != ts[2]:
                return None
            r = ts[1]
        elif o in ("==", "!=", "<", "<=", ">", ">=", "&", "|", "xor", "not"):
            r = "b"
        elif o in ("+", "-", "*", "min", "max"):
            r = "i" if all(x in ("i", "b") for x in ts) else "d"
        elif o in ("neg", "abs"):
            r = "i" if ts[0] in ("i", "b") else "d"
        elif o in BIN_CODES or o in UN_CODES:
            r = "d"
        else:
            return None
        t[n + k] = r
    return t


# ----------------------------------------------------------------------------- code generation
_SCALAR_BIN = {"/": "sysml_vdiv({a}, {b})", "^": "sysml_vpow({a}, {b})", "log": "sysml_vlogb({a}, {b})"}
_SCALAR_UN = {"sqrt": "sysml_vsqrt({a})", "log": "sysml_vlog({a})", "round": "sysml_vround({a})",
              "exp": "exp({a})"}


def _dbl(tmpl):
    """A cell-template operator expression over double scalars instead of T cells."""
    return tmpl.replace("<T>", "<double>").replace("(T)", "(double)").replace("T(", "double(")


def _expr(o, args, scalar):
    if o == "sel":
        return f"(({args[0]}) != 0 ? ({args[1]}) : ({args[2]}))"
    if len(args) == 2:
        if scalar and o in _SCALAR_BIN:
            return _SCALAR_BIN[o].format(a=args[0], b=args[1])
        t = _C_BIN[o]
        return (_dbl(t) if scalar else t).format(a=args[0], b=args[1])
    if scalar and o in _SCALAR_UN:
        return _SCALAR_UN[o].format(a=args[0])
    t = _C_UN[o]
    return (_dbl(t) if scalar else t).format(a=args[0])


_VPRELUDE = r"""
// scalar semantics of runtime/scalars.py (Java / R rules) for the uniform scalar algebra
__device__ __forceinline__ double sysml_vdiv(double a, double b) { return a / b; }
__device__ __forceinline__ double sysml_vpow(double a, double b) { return pow(a, b); }
__device__ __forceinline__ double sysml_vsqrt(double a) { return a >= 0.0 ? sqrt(a) : __builtin_nan(""); }
__device__ __forceinline__ double sysml_vlog(double a) {
  return (a < 0.0 || a != a) ? __builtin_nan("") : (a == 0.0 ? -__builtin_inf() : log(a)); }
__device__ __forceinline__ double sysml_vlogb(double a, double b) { return sysml_vlog(a) / log(b); }
__device__ __forceinline__ double sysml_vround(double a) {
  return (a != a || a == __builtin_inf() || a == -__builtin_inf()) ? a : floor(a + 0.5); }
__device__ __forceinline__ double sysml_red_comb(int op, double a, double b) {
  if (op == 0) return a + b;
  if (a != a) return a;
  if (b != b) return b;
  return op == 1 ? (a < b ? a : b) : (a > b ? a : b);
}
"""


def generate(vp, T, dts, kinds, n_out_m, n_out_s):
    """HIP source of the program for a signature: T compute type of the cells, dts[k] storage
    type of matrix / device-scalar leaf k, kinds[k] in 'm' (matrix), 'h' (host scalar),
    'd' (device scalar)."""
    ct = "float" if T == torch.float32 else "double"
    n = len(vp.leaf_dts)
    nv = n + len(vp.instrs)
    cls = vp.cls
    # consumers' stages: a matrix value read in a later stage than the one computing it goes
    # through scratch
    uses = [[] for _ in range(nv)]
    for k, (kind, o, srcs) in enumerate(vp.instrs):
        for s in srcs:
            uses[s].append(n + k)
    out_m = [v for v in vp.outs if cls[v] == "M"]
    out_s = [v for v in vp.outs if cls[v] == "S"]
    scratch = {}
    for v in range(n, nv):
        if cls[v] == "M" and any(vp.stage[u] > vp.stage[v] for u in uses[v]):
            scratch[v] = len(scratch)
    lines = []
    A = lines.append
    A("  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;")
    A("  const sysml_i64 n = P.n;")
    for k in range(n):
        if kinds[k] == "h":
            A(f"  const double v{k} = P.s[{k}];")
        elif kinds[k] == "d":
            A(f"  const double v{k} = sysml_ld<double>(P.in[{k}], {dts[k]}, 0);")
    # scalar ops by availability stage; reductions per stage
    by_stage_scalar = {}
    by_stage_loop = {}
    for k, (kind, o, srcs) in enumerate(vp.instrs):
        v = n + k
        if kind == "s":
            by_stage_scalar.setdefault(vp.avail[v], []).append(v)
        else:
            by_stage_loop.setdefault(vp.stage[v], []).append(v)
    kred = max([sum(1 for v in by_stage_loop.get(s, []) if vp.instrs[v - n][0] == "r")
                for s in range(vp.nstages)] + [1])
    for st in range(vp.nstages):
        for v in by_stage_scalar.get(st, []):
            kind, o, srcs = vp.instrs[v - n]
            A(f"  const double v{v} = (double){_expr(o, [f'v{s}' for s in srcs], True)};")
        loop = by_stage_loop.get(st, [])
        if not loop:
            continue
        reds = [v for v in loop if vp.instrs[v - n][0] == "r"]
        for v in reds:
            o = vp.instrs[v - n][1]
            init = "__builtin_inf()" if o == "min" else ("-__builtin_inf()" if o == "max" else "0.0")
            A(f"  double r{v} = {init};")
        A("  for (sysml_i64 i = tid; i < n; i += %d) {" % NT)
        loaded = set()

        def mref(s):
            # expression of matrix-or-scalar value s inside the stage loop
            if cls[s] == "S":
                return f"(T)v{s}"
            if s < n:
                if s not in loaded:
                    A(f"    const T x{s} = sysml_ld<T>(P.in[{s}], {dts[s]}, i);")
                    loaded.add(s)
                return f"x{s}"
            if vp.stage[s] < st:
                if s not in loaded:
                    A(f"    const T x{s} = P.scratch[(sysml_i64){scratch[s]} * n + i];")
                    loaded.add(s)
                return f"x{s}"
            return f"m{s}"

        for v in loop:
            kind, o, srcs = vp.instrs[v - n]
            args = [mref(s) for s in srcs]
            if kind == "m":
                A(f"    const T m{v} = (T){_expr(o, args, False)};")
                if v in scratch:
                    A(f"    P.scratch[(sysml_i64){scratch[v]} * n + i] = m{v};")
                if v in out_m:
                    A(f"    static_cast<T*>(P.out[{out_m.index(v)}])[i] = m{v};")
            else:
                if o == "dot":
                    x = f"(double){args[0]} * (double){args[1]}"
                elif o == "dot3":
                    x = f"(double){args[0]} * (double){args[1]} * (double){args[2]}"
                else:
                    x = f"(double){args[0]}"
                if o in ("sum", "mean", "dot", "dot3"):
                    A(f"    r{v} += {x};")
                elif o == "sumsq":
                    A(f"    {{ const double t = {x}; r{v} += t * t; }}")
                elif o == "min":
                    A(f"    {{ const double t = {x}; r{v} = (t != t || t < r{v}) ? t : r{v}; }}")
                else:
                    A(f"    {{ const double t = {x}; r{v} = (t != t || t > r{v}) ? t : r{v}; }}")
        A("  }")
        # one block reduction for all of this stage's aggregates
        for j, v in enumerate(reds):
            o = vp.instrs[v - n][1]
            cop = 1 if o == "min" else (2 if o == "max" else 0)
            A(f"  for (int off = 32; off > 0; off >>= 1) r{v} = sysml_red_comb({cop}, r{v}, __shfl_xor(r{v}, off));")
            A(f"  if (lane == 0) red[wid * {kred} + {j}] = r{v};")
        A("  __syncthreads();")
        for j, v in enumerate(reds):
            o = vp.instrs[v - n][1]
            cop = 1 if o == "min" else (2 if o == "max" else 0)
            A(f"  double v{v} = red[{j}];")
            A(f"  for (int w = 1; w < {NT // 64}; ++w) v{v} = sysml_red_comb({cop}, v{v}, red[w * {kred} + {j}]);")
            if o == "mean":
                A(f"  v{v} = v{v} / (double)n;")
        A("  __syncthreads();")
    if out_s:
        A("  if (tid == 0) {")
        for j, v in enumerate(out_s):
            A(f"    P.sout[{j}] = (double)v{v};")
        A("  }")
    body = "\n".join(lines)
    return (_prelude() + _VPRELUDE + f"""
// generated: {vp.describe()}
typedef {ct} T;
struct VArgs {{
  const void* in[{max(n, 1)}];
  double s[{max(n, 1)}];
  void* out[{max(n_out_m, 1)}];
  double* sout;
  T* scratch;
  sysml_i64 n;
  const double* live;
}};
extern "C" __global__ void __launch_bounds__({NT}) sysml_vprog_k(const VArgs P) {{
  {{  // dead run-ahead iteration (runtime/program.py; bit 0 of the address inverts the sense)
    const unsigned long long la = (unsigned long long)P.live;
    if (la != 0ull && ((*(const double*)(la & ~1ull) == 0.0) != ((la & 1ull) != 0ull))) return;
  }}
  __shared__ double red[{NT // 64} * {kred}];
{body}
}}
"""), len(scratch)


REG_CPT = (1, 2, 4, 8, 16)   # cells per thread of the register-resident variant (n <= 16 * NTR)
NTR = 512                    # its workgroup: 8 wave64s, 256 VGPRs per lane


def _reg_cpt(n):
    for c in REG_CPT:
        if n <= c * NTR:
            return c
    return 0


def generate_reg(vp, T, dts, kinds, n_out_m, n_out_s, cpt):
    """Register-resident variant for n <= cpt * NT cells: every thread owns cells
    tid + c * NTR (c < cpt); all matrix operands are loaded once, up front (every load in
    flight together), and each value stays in VGPRs for the whole program -- the stages
    between aggregates cost one LDS block reduction each and no memory traffic."""
    ct = "float" if T == torch.float32 else "double"
    n = len(vp.leaf_dts)
    nv = n + len(vp.instrs)
    cls = vp.cls
    out_m = [v for v in vp.outs if cls[v] == "M"]
    out_s = [v for v in vp.outs if cls[v] == "S"]
    lines = []
    A = lines.append
    A("  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;")
    A("  const sysml_i64 n = P.n;")
    for k in range(n):
        if kinds[k] == "h":
            A(f"  const double v{k} = P.s[{k}];")
        elif kinds[k] == "d":
            A(f"  const double v{k} = sysml_ld<double>(P.in[{k}], {dts[k]}, 0);")
        else:
            A(f"  T x{k}[{cpt}];")
    mats = [k for k in range(n) if kinds[k] == "m"]
    if mats:
        A(f"  #pragma unroll")
        A(f"  for (int c = 0; c < {cpt}; ++c) {{")
        A(f"    const sysml_i64 i = tid + (sysml_i64)c * {NTR};")
        A(f"    const sysml_i64 ic = i < n ? i : n - 1;")
        for k in mats:
            A(f"    x{k}[c] = sysml_ld<T>(P.in[{k}], {dts[k]}, ic);")
        A("  }")
    for v in range(n, nv):
        if cls[v] == "M":
            A(f"  T m{v}[{cpt}];")
    by_stage_scalar, by_stage_loop = {}, {}
    for k, (kind, o, srcs) in enumerate(vp.instrs):
        v = n + k
        if kind == "s":
            by_stage_scalar.setdefault(vp.avail[v], []).append(v)
        else:
            by_stage_loop.setdefault(vp.stage[v], []).append(v)
    kred = max([sum(1 for v in by_stage_loop.get(st, []) if vp.instrs[v - n][0] == "r")
                for st in range(vp.nstages)] + [1])

    def ref(sv):
        if cls[sv] == "S":
            return f"(T)v{sv}"
        return f"x{sv}[c]" if sv < n else f"m{sv}[c]"

    for st in range(vp.nstages):
        for v in by_stage_scalar.get(st, []):
            kind, o, srcs = vp.instrs[v - n]
            A(f"  const double v{v} = (double){_expr(o, [f'v{x}' for x in srcs], True)};")
        loop = by_stage_loop.get(st, [])
        if not loop:
            continue
        reds = [v for v in loop if vp.instrs[v - n][0] == "r"]
        for v in reds:
            o = vp.instrs[v - n][1]
            init = "__builtin_inf()" if o == "min" else ("-__builtin_inf()" if o == "max" else "0.0")
            A(f"  double r{v} = {init};")
        A("  #pragma unroll")
        A(f"  for (int c = 0; c < {cpt}; ++c) {{")
        A(f"    const sysml_i64 i = tid + (sysml_i64)c * {NTR};")
        A("    const bool ok = i < n;")
        for v in loop:
            kind, o, srcs = vp.instrs[v - n]
            args = [ref(x) for x in srcs]
            if kind == "m":
                A(f"    m{v}[c] = (T){_expr(o, args, False)};")
                if v in out_m:
                    A(f"    if (ok) static_cast<T*>(P.out[{out_m.index(v)}])[i] = m{v}[c];")
            else:
                if o == "dot":
                    x = f"(double){args[0]} * (double){args[1]}"
                elif o == "dot3":
                    x = f"(double){args[0]} * (double){args[1]} * (double){args[2]}"
                else:
                    x = f"(double){args[0]}"
                if o in ("sum", "mean", "dot", "dot3"):
                    A(f"    if (ok) r{v} += {x};")
                elif o == "sumsq":
                    A(f"    if (ok) {{ const double t = {x}; r{v} += t * t; }}")
                elif o == "min":
                    A(f"    if (ok) {{ const double t = {x}; r{v} = (t != t || t < r{v}) ? t : r{v}; }}")
                else:
                    A(f"    if (ok) {{ const double t = {x}; r{v} = (t != t || t > r{v}) ? t : r{v}; }}")
        A("  }")
        for j, v in enumerate(reds):
            o = vp.instrs[v - n][1]
            cop = 1 if o == "min" else (2 if o == "max" else 0)
            A(f"  for (int off = 32; off > 0; off >>= 1) r{v} = sysml_red_comb({cop}, r{v}, __shfl_xor(r{v}, off));")
            A(f"  if (lane == 0) red[wid * {kred} + {j}] = r{v};")
        if reds:
            A("  __syncthreads();")
        for j, v in enumerate(reds):
            o = vp.instrs[v - n][1]
            cop = 1 if o == "min" else (2 if o == "max" else 0)
            A(f"  double v{v} = red[{j}];")
            A(f"  for (int w = 1; w < {NTR // 64}; ++w) v{v} = sysml_red_comb({cop}, v{v}, red[w * {kred} + {j}]);")
            if o == "mean":
                A(f"  v{v} = v{v} / (double)n;")
        if reds:
            A("  __syncthreads();")
    if out_s:
        A("  if (tid == 0) {")
        for j, v in enumerate(out_s):
            A(f"    P.sout[{j}] = (double)v{v};")
        A("  }")
    body = "\n".join(lines)
    return (_prelude() + _VPRELUDE + f"""
// generated (register-resident, {cpt} cells / thread): {vp.describe()}
typedef {ct} T;
struct VArgs {{
  const void* in[{max(n, 1)}];
  double s[{max(n, 1)}];
  void* out[{max(n_out_m, 1)}];
  double* sout;
  T* scratch;
  sysml_i64 n;
  const double* live;
}};
extern "C" __global__ void __launch_bounds__({NTR}) sysml_vprog_k(const VArgs P) {{
  {{  // dead run-ahead iteration (runtime/program.py; bit 0 of the address inverts the sense)
    const unsigned long long la = (unsigned long long)P.live;
    if (la != 0ull && ((*(const double*)(la & ~1ull) == 0.0) != ((la & 1ull) != 0ull))) return;
  }}
  __shared__ double red[{NTR // 64} * {kred}];
{body}
}}
"""), 0


def _args_struct(n_in, n_out_m):
    class VArgs(ctypes.Structure):
        _fields_ = [("inp", ctypes.c_void_p * max(n_in, 1)), ("s", ctypes.c_double * max(n_in, 1)),
                    ("out", ctypes.c_void_p * max(n_out_m, 1)), ("sout", ctypes.c_void_p),
                    ("scratch", ctypes.c_void_p), ("n", ctypes.c_int64), ("live", ctypes.c_void_p)]
    return VArgs


# ----------------------------------------------------------------------------- host uploads
class _Uploads:
    """Device copies of small host tensors read by vector programs (loop constants such as a
    regularisation matrix), keyed by tensor identity and version, dropped with the tensor."""

    def __init__(self):
        self._d = {}

    def get(self, t, device):
        k = id(t)
        e = self._d.get(k)
        if e is not None and e[0]() is t and e[1] == t._version and e[2].device == device:
            return e[2]
        d = t.to(device, non_blocking=True)
        dd = self._d
        ref = weakref.ref(t, lambda _r, k=k: dd.pop(k, None) if dd.get(k, (None,))[0] is _r else None)
        self._d[k] = (ref, t._version, d)
        return d


_uploads = _Uploads()


# ----------------------------------------------------------------------------- evaluation
def evaluate(vp, ctx, args):
    r = _kernel(vp, args) if backend.use_kernels and RTC else None
    if r is not None:
        stats["kernel"] += 1
        return r
    stats["fallback"] += 1
    return fallback(vp, ctx, args)


def fallback(vp, ctx, args):
    """The region's original operators one by one (Cell-fused), as before fusion."""
    fb = vp._fallback
    if fb is None:
        from ..compiler.lops import _linearize
        from ..compiler.blocks import BasicBlock
        from ..compiler.codegen import fuse_cells
        from ..runtime.instructions import make_impl
        names, outs = vp.fallback_dag
        tmp = BasicBlock()
        tmp.env_out = {f"__vp_o{k}": h for k, h in enumerate(outs)}
        tmp.live_out = None
        fuse_cells(tmp, single=backend.use_kernels)     # on the GPU every operator a generated kernel
        instrs, writes, nslots = _linearize([], list(tmp.env_out.items()), make_impl)
        argpos = {nm: k for k, nm in enumerate(names)}
        reads = [(ins.out, argpos[ins.hop.p["name"]]) for ins in instrs if ins.opcode == "tread"]
        rest = [ins for ins in instrs if ins.opcode != "tread"]
        fb = vp._fallback = (reads, rest, [s for _, s in writes], nslots)
    reads, rest, outslots, nslots = fb
    slots = [None] * nslots
    for s, k in reads:
        slots[s] = args[k]
    for ins in rest:
        slots[ins.out] = ins.fn(ctx, [slots[i] for i in ins.ins])
    return tuple(slots[s] for s in outslots)


_DevScalar = []


def _signature(vp, args):
    if not _DevScalar:
        from ..runtime.scalars import DevScalar
        _DevScalar.append(DevScalar)
    DevScalar = _DevScalar[0]
    sig = []
    shape = None
    dev = None
    for x, dt in zip(args, vp.leaf_dts):
        tx = type(x)
        if dt == "M":
            if tx is not _Tensor or x.layout is not torch.strided or x.dim() != 2 or x.dtype not in _DT:
                return None
            s = (x.shape[0], x.shape[1])
            if shape is None:
                shape = s
            elif s != shape:
                return None
            if x.is_cuda:
                if dev is None:
                    dev = x.device
                elif x.device != dev:
                    return None
            sig.append(("m", x.dtype, x.is_cuda))
        elif tx is float:
            sig.append(("h", "d"))
        elif tx is bool:
            sig.append(("h", "b"))
        elif tx is int:
            sig.append(("h", "i"))
        elif tx is DevScalar:
            if not x.t.is_cuda or x.t.dtype not in _DT:
                return None
            sig.append(("d", x.vt, x.t.dtype))
        else:
            return None
    if shape is None or shape[0] * shape[1] < 1 or shape[0] * shape[1] > VMAX:
        return None
    return tuple(sig), shape, dev


class _Plan:
    __slots__ = ("fn", "T", "kinds", "types", "Args", "nscr", "out_m", "out_s", "dev", "cpt")


def _make_plan(vp, sig, dev, cpt=0):
    kinds, dts, ltypes = [], [], []
    f64 = False
    for e in sig:
        if e[0] == "m":
            kinds.append("m")
            dts.append(_DT[e[1]])
            ltypes.append("M")
            f64 = f64 or e[1] == torch.float64
        elif e[0] == "h":
            kinds.append("h")
            dts.append(0)
            ltypes.append(e[1])
        else:
            kinds.append("d")
            dts.append(_DT[e[2]])
            ltypes.append(e[1])
    types = _scalar_types(vp, ltypes)
    if types is None:
        return None
    # a select of matrices needs a scalar (or matrix) condition; a scalar program value used as
    # a matrix is fine (broadcast); matrix values never flow into scalar operators (by construction)
    T = torch.float64 if (f64 or backend.dtype == torch.float64) else torch.float32
    out_m = [v for v in vp.outs if vp.cls[v] == "M"]
    out_s = [v for v in vp.outs if vp.cls[v] == "S"]
    if cpt:
        src, nscr = generate_reg(vp, T, dts, kinds, len(out_m), len(out_s), cpt)
    else:
        src, nscr = generate(vp, T, dts, kinds, len(out_m), len(out_s))
    code = compile_source(src, gpu_arch(dev))
    L = _rtc_lib()
    fn = ctypes.c_void_p()
    cbuf = ctypes.create_string_buffer(code, len(code))
    rc = L.sysml_rtc_load(cbuf, b"sysml_vprog_k", ctypes.byref(fn))
    if rc != 0:
        raise RuntimeError(f"hipModuleLoadData failed ({rc})")
    stats["compiled"] += 1
    pl = _Plan()
    pl.fn = (fn, cbuf)
    pl.T, pl.kinds, pl.types, pl.nscr = T, kinds, types, nscr
    pl.Args = _args_struct(len(vp.leaf_dts), len(out_m))
    pl.out_m, pl.out_s = out_m, out_s
    pl.dev = dev
    pl.cpt = cpt
    return pl


_raw_stream = torch._C._cuda_getCurrentRawStream if hasattr(torch._C, "_cuda_getCurrentRawStream") else None
# SYSML_VPROG_DEFER=1: scalar results read back through an event-tracked pinned copy and
# materialised on first use.  Off by default -- measured slower (1.25M rows: 87-93 vs 74 ms/step,
# 10M: 419 vs 397): the deferred values turn the solvers' host scalar algebra into device launches
DEFER_READS = __import__("os").environ.get("SYSML_VPROG_DEFER", "0") == "1"


_PLANS = {}      # structural program key + signature + device -> plan: programs of recompiled scripts share


def _kernel(vp, args):
    s = _signature(vp, args)
    if s is None:
        return None
    sig, (R, Cc), dev = s
    if dev is None:
        dev = backend.device
    if dev is None or getattr(dev, "type", None) != "cuda":
        return None
    cpt = _reg_cpt(R * Cc) if REG else 0
    key = (sig, str(dev), cpt)
    pl = vp._plans.get(key, False)
    if pl is False:
        gkey = (vp.leaf_dts, vp.instrs, vp.outs, sig, str(dev), backend.dtype, cpt)
        pl = _PLANS.get(gkey, False)
        if pl is False:
            try:
                pl = _make_plan(vp, sig, dev, cpt)
            except RuntimeError as e:
                import warnings
                warnings.warn(f"vector program not compiled, running its operators one by one: {e}")
                pl = None
            _PLANS[gkey] = pl
        vp._plans[key] = pl
    if pl is None:
        return None
    n = R * Cc
    T = pl.T
    P = pl.Args()
    keep = []
    for k, (x, kd) in enumerate(zip(args, pl.kinds)):
        if kd == "m":
            if not x.is_cuda:
                x = _uploads.get(x, dev)
            if not x.is_contiguous():
                x = x.contiguous()
            keep.append(x)
            P.inp[k] = x.data_ptr()
        elif kd == "d":
            t = x.t.reshape(1)
            keep.append(t)
            P.inp[k] = t.data_ptr()
        else:
            P.s[k] = float(x)
    outs_m = [torch.empty((R, Cc), dtype=T, device=dev) for _ in pl.out_m]
    for j, o in enumerate(outs_m):
        P.out[j] = o.data_ptr()
    sout = torch.empty(max(1, len(pl.out_s)), dtype=torch.float64, device=dev) if pl.out_s else None
    P.sout = sout.data_ptr() if sout is not None else 0
    scr = torch.empty(pl.nscr * n, dtype=T, device=dev) if pl.nscr else None
    P.scratch = scr.data_ptr() if scr is not None else 0
    P.n = n
    P.live = backend.live
    di = dev.index if dev.index is not None else torch.cuda.current_device()
    st = _raw_stream(di) if _raw_stream is not None else torch.cuda.current_stream(dev).cuda_stream
    rc = _rtc_lib().sysml_rtc_launch(pl.fn[0], 1, 1, NTR if pl.cpt else NT, ctypes.byref(P), ctypes.sizeof(P), st)
    if rc != 0:
        raise RuntimeError(f"vector program launch failed: {rc}")
    from . import kernels
    kernels._count("vprog")
    types = pl.types
    res = []
    im = iter(outs_m)
    si = 0
    if backend.defer and sout is not None:
        # run-ahead loop: the scalars stay in HBM (the next iteration's kernels read them
        # there); the loop reads its predicate one iteration late
        DS = _DevScalar[0]
        for v in vp.outs:
            if vp.cls[v] == "M":
                res.append(next(im))
            else:
                t = types[v]
                res.append(DS(sout[si], t if t in ("b", "i") else "d"))
                si += 1
        return tuple(res)
    if DEFER_READS and sout is not None:
        # the scalars are copied to pinned host memory behind the kernel and returned as device
        # scalars that share that copy's event: the host goes on queueing the block's device
        # work and waits (for this kernel only, not for work queued after it) where a value is
        # first needed on the host -- a print, a branch -- instead of draining the queue here
        DS = _DevScalar[0]
        hb = torch.empty(sout.numel(), dtype=torch.float64, pin_memory=True)
        hb.copy_(sout, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        for v in vp.outs:
            if vp.cls[v] == "M":
                res.append(next(im))
            else:
                t = types[v]
                d = DS(sout[si], t if t in ("b", "i") else "d")
                d._hb, d._ev = hb[si:si + 1], ev
                res.append(d)
                si += 1
        return tuple(res)
    svals = sout.cpu().tolist() if sout is not None else ()     # the one device synchronisation (GIL released)
    _HT.mark("vprog-sync")
    del keep
    for v in vp.outs:
        if vp.cls[v] == "M":
            res.append(next(im))
        else:
            x = svals[si]
            si += 1
            t = types[v]
            res.append((x != 0.0) if t == "b" else (int(x) if t == "i" else x))
    return tuple(res)
