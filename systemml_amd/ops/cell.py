"""Fused cellwise operators at run time (reference: runtime/codegen/SpoofCellwise.java and the
SpoofOperator / SpoofCUDA instructions that execute the classes the codegen compiler emits).

A `CellProgram` is the lowered form of one fused DAG (compiler/codegen.py): the DAG's leaves
are its inputs, preloaded into registers 0..n_in-1, and every fused binary / unary operator is
one instruction (kind, op, dst, a, b) over at most 16 registers; an optional aggregate
(sum / sumsq / mean / min / max over all cells, rows or columns) consumes the output register.

On the MI355X the whole program runs as ONE pass over the output cells: every input is read
once, intermediates stay in VGPRs, and only the result (or the aggregate) is written.  The
kernel is GENERATED per program and operand signature (`generate`: the DAG as straight-line
HIP code in a `Spec` struct over the templates of ops/hip/cell_rtc.inc), compiled once by
hipRTC for the device's gfx target (ops/hip/rtc.hip) and cached in memory and on disk by the
source hash -- the reference compiles its generated operator classes the same way.  When the
run-time compiler is unavailable (or SYSML_CELL_RTC=0) the prebuilt register-program
interpreter of ops/hip/cell.hip runs the same program.  Everywhere else -- CPU backend, sparse / compressed / constant-column /
row-partitioned operands, shapes outside the broadcast modes the kernel supports -- the program
runs instruction by instruction through ops/core.binary / unary / agg, i.e. exactly the
operators the DAG had before fusion, so fusion never changes semantics or error behaviour.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import tempfile
import time

import torch

from . import core as C
from .augmented import ConstCol as _ConstCol
from .backend import backend

BIN_CODES = {"+": 1, "-": 2, "*": 3, "/": 4, "^": 5, "%%": 6, "%/%": 7, "==": 8, "!=": 9, "<": 10,
             "<=": 11, ">": 12, ">=": 13, "&": 14, "|": 15, "xor": 16, "min": 17, "max": 18, "log": 19}
UN_CODES = {"sq": 20,               # x ^ 2 (binary '^' with the literal 2, lowered to one multiply)
            "neg": 32, "not": 33, "abs": 34, "exp": 35, "log": 36, "sqrt": 37, "round": 38, "floor": 39,
            "ceil": 40, "sign": 41, "sin": 42, "cos": 43, "tan": 44, "asin": 45, "acos": 46, "atan": 47,
            "sinh": 48, "cosh": 49, "tanh": 50, "sigmoid": 51}
AGG_CODES = {"sum": 0, "sumsq": 1, "mean": 0, "min": 2, "max": 3}
AGG_DIRS = {"all": 1, "row": 2, "col": 3}
MAXIN, MAXOPS, NR = 12, 40, 16
COL4 = 1000           # column-aggregate variant offset: 4 adjacent columns per lane (sysml_cell_col4)
# row aggregates over 4-cell groups with vector loads (sysml_cell_row4); SYSML_CELL_ROW4=0: one cell
# per lane (sysml_cell_row)
ROW4 = os.environ.get("SYSML_CELL_ROW4", "1") != "0"
FULL, ROWV, COLV, HSCALAR, DSCALAR, CHAN = range(6)
# per-channel broadcast operators (bias_add / bias_multiply: a C x 1 vector over the H*W columns
# of each channel of an N x (C*H*W) operand); generated kernels only (mode CHAN)
BIAS_OPS = {"bias+": "+", "bias*": "*"}

stats = {"kernel": 0, "sequential": 0, "rtc_compiled": 0, "rtc_cache_hits": 0, "rtc_launches": 0,
         "interpreter_launches": 0}
RTC = os.environ.get("SYSML_CELL_RTC", "1") != "0"
TRACE = os.environ.get("SYSML_CELL_TRACE", "0") == "1"
fallbacks = {}
RTC_DIR = os.environ.get("SYSML_RTC_CACHE", os.path.join(tempfile.gettempdir(), "systemml_amd_rtc"))

# C expressions of the operators ({a}, {b}: operand expressions of type T)
_C_BIN = {"+": "({a} + {b})", "-": "({a} - {b})", "*": "({a} * {b})", "/": "({a} / {b})", "^": "pow({a}, {b})",
          "%%": "sysml_rem<T>({a}, {b})", "%/%": "floor({a} / {b})", "==": "sysml_b<T>({a} == {b})",
          "!=": "sysml_b<T>({a} != {b})", "<": "sysml_b<T>({a} < {b})", "<=": "sysml_b<T>({a} <= {b})",
          ">": "sysml_b<T>({a} > {b})", ">=": "sysml_b<T>({a} >= {b})",
          "&": "sysml_b<T>({a} != T(0) && {b} != T(0))", "|": "sysml_b<T>({a} != T(0) || {b} != T(0))",
          "xor": "sysml_b<T>(({a} != T(0)) != ({b} != T(0)))", "min": "sysml_min<T>({a}, {b})",
          "max": "sysml_max<T>({a}, {b})", "log": "(log({a}) / log({b}))", "bias+": "({a} + {b})",
          "bias*": "({a} * {b})"}
_C_UN = {"sq": "({a} * {a})", "neg": "(-{a})", "not": "sysml_b<T>({a} == T(0))", "abs": "fabs({a})",
         "exp": "exp({a})", "log": "log({a})", "sqrt": "sqrt({a})", "round": "floor({a} + T(0.5))",
         "floor": "floor({a})", "ceil": "ceil({a})", "sign": "(T)(({a} > T(0)) - ({a} < T(0)))",
         "sin": "sin({a})", "cos": "cos({a})", "tan": "tan({a})", "asin": "asin({a})", "acos": "acos({a})",
         "atan": "atan({a})", "sinh": "sinh({a})", "cosh": "cosh({a})", "tanh": "tanh({a})",
         "sigmoid": "(T(1) / (T(1) + exp(-{a})))"}


class CellProgram:
    """ops: tuple of (kind 'b' | 'u', op, dst, a, b) register instructions; n_in: inputs in
    registers 0..n_in-1; out: result register; agg: None or (op, 'all' | 'row' | 'col')."""
    __slots__ = ("ops", "n_in", "out", "agg", "_code")

    def __init__(self, ops, n_in, out, agg=None):
        self.ops = tuple(tuple(x) for x in ops)
        self.n_in = n_in
        self.out = out
        self.agg = tuple(agg) if agg else None
        self._code = {}

    def key(self):
        return (self.ops, self.n_in, self.out, self.agg)

    def __eq__(self, other):
        return isinstance(other, CellProgram) and self.key() == other.key()

    def __hash__(self):
        return hash(self.key())

    def describe(self):
        body = ",".join(o for _, o, _, _, _ in self.ops)
        return f"cell[{body}]" + (f"|{self.agg[0]}-{self.agg[1]}" if self.agg else "")

    def __repr__(self):
        return self.describe()

    def device_code(self, device):
        """The instructions as an int32 (n_ops x 4) HBM array, uploaded once per device."""
        t = self._code.get(device)
        if t is None:
            rows = []
            for kind, o, d, a, b in self.ops:
                if o in BIAS_OPS:
                    raise ValueError("per-channel operators run in generated kernels only")
                op = BIN_CODES[o] if kind == "b" else UN_CODES[o]
                for r in (d, a, b):
                    if not 0 <= r < NR:
                        raise ValueError(f"cell program register {r} out of range")
                rows.append([op, d, a, b])
            t = torch.tensor(rows or [[0, 0, 0, 0]], dtype=torch.int32).to(device)
            self._code[device] = t
        return t


# ----------------------------------------------------------------------------- evaluation
def evaluate(prog: CellProgram, args):
    r = _kernel(prog, args) if backend.use_kernels else None
    if r is not None:
        stats["kernel"] += 1
        return r
    if backend.use_kernels and any(type(x) is _ConstCol for x in args):
        r = _split_cc(prog, args)
        if r is not None:
            stats["kernel"] += 1
            return r
    stats["sequential"] += 1
    if TRACE and backend.use_kernels:
        # SYSML_CELL_TRACE=1: which programs miss the generated kernels, on which operands
        k = (prog.describe(), tuple((tuple(x.shape), str(x.dtype), x.device.type) if type(x) is _Tensor
                                    else type(x).__name__ for x in args))
        fallbacks[k] = fallbacks.get(k, 0) + 1
    return sequential(prog, args)


def _axpy_form(prog):
    """(y, p, q, sign) when the program is y +/- p * q (or p * q + y) over its inputs, else None:
    with one of p, q a host scalar the host runs it as ONE torch.add(y, x, alpha=+-s) -- the CG
    update shape of iterative solvers (S + a * V, R - a * HV), where per-call dispatch dominates
    on D x K matrices."""
    f = prog._code.get("axpy", False)
    if f is not False:
        return f
    f = None
    if len(prog.ops) == 2 and not prog.agg:
        (k1, o1, t, a1, b1), (k2, o2, d, a2, b2) = prog.ops
        n = prog.n_in
        if k1 == "b" and o1 == "*" and a1 < n and b1 < n and k2 == "b" and d == prog.out:
            if o2 in ("+", "-") and b2 == t and a2 != t and a2 < n:
                f = (a2, a1, b1, 1.0 if o2 == "+" else -1.0)
            elif o2 == "+" and a2 == t and b2 != t and b2 < n:
                f = (b2, a1, b1, 1.0)
    prog._code["axpy"] = f
    return f


def _split_cc(prog, args):
    """The program over constant-column-augmented operands (cbind(X, c), ops/augmented.py) --
    e.g. MultiLogReg's icpt=2 `rowSums(X ^ 2 * t(sc ^ 2))` on cbind(X, 1): the generated kernel
    runs over X itself (bf16 as stored, the aggregation fused) and the constant column's value
    follows on the host, instead of materialising f(cbind(X, c)) (a full-size pass and a
    full-size write).  Matrix operands: augmented ones over one shape, and row vectors over all
    D + 1 columns (split into their first D entries and the last); scalars must be host
    values.  None when that or the aggregation does not fit (or for a bare aggregate, which
    ops/augmented.agg serves)."""
    from . import augmented as AUG
    if not prog.ops:
        return None
    shape = None
    for x in args:
        if AUG.is_cc(x):
            if shape is None:
                shape = tuple(x.X.shape)
            elif tuple(x.X.shape) != shape:
                return None
    xs, cs = [], []
    for x in args:
        if AUG.is_cc(x):
            xs.append(x.X)
            cs.append(torch.full((1, 1), x.c, dtype=torch.float64))
        elif type(x) in (float, int, bool):
            xs.append(x)
            cs.append(x)
        elif type(x) is _Tensor and x.dim() == 2 and x.shape[0] == 1 and x.shape[1] == shape[1] + 1 \
                and x.layout is torch.strided:
            xs.append(x[:, :shape[1]])
            cs.append(x[:, shape[1]:].detach().to("cpu", torch.float64))
        else:
            return None
    agg = prog.agg
    if agg is not None and agg[0] not in ("sum", "min", "max"):
        return None
    r = _kernel(prog, xs)
    if r is None:
        return None
    elem = CellProgram(prog.ops, prog.n_in, prog.out)
    fc = float(sequential(elem, cs).reshape(-1)[0])        # the constant column's value, on the host
    n = shape[0]
    if agg is None:
        return AUG.ConstCol(r, fc)
    o, d = agg
    if d == "col":
        rc = C.cvt(r)
        v = n * fc if o == "sum" else fc
        return torch.cat([rc, torch.full((1, 1), v, dtype=rc.dtype, device=rc.device)], 1)
    if d == "row":
        return C.binary("+" if o == "sum" else o, r, fc)
    return C.binary("+", r, n * fc) if o == "sum" else C.binary(o, r, fc)


def sequential(prog: CellProgram, args):
    """The fused DAG's original operators, one after the other."""
    ax = _axpy_form(prog)
    if ax is not None:
        y, p, q = args[ax[0]], args[ax[1]], args[ax[2]]
        x, sc = (q, p) if (type(p) is float or type(p) is int) else (p, q)
        if type(y) is _Tensor and type(x) is _Tensor and (type(sc) is float or type(sc) is int) and \
                not y.is_cuda and y.layout is torch.strided and x.layout is torch.strided and \
                y.dtype is torch.float64 and x.dtype is torch.float64 and y.shape == x.shape:
            return torch.add(y, x, alpha=ax[3] * sc)
    regs = list(args) + [None] * (NR - len(args))
    for kind, o, d, a, b in prog.ops:
        if kind == "b" and o in BIAS_OPS:
            from ..runtime import builtins as B
            regs[d] = (B.b_bias_mult if o == "bias*" else B.b_bias_add)(None, regs[a], regs[b])
        elif kind == "b":
            regs[d] = C.binary(o, regs[a], regs[b])
        elif o == "sq":
            regs[d] = C.binary("^", regs[a], 2)
        else:
            regs[d] = C.unary(o, regs[a])
    r = regs[prog.out]
    if prog.agg:
        r = C.agg(prog.agg[0], prog.agg[1], r)
    return r


def _bin_ok(sa, sb):
    """ops/core._check_bin_dims: the operand shapes a cellwise binary operator accepts."""
    if sa == sb:
        return True
    (ra, ca), (rb, cb) = sa, sb
    return ((ra == rb and (ca == 1 or cb == 1)) or (ca == cb and (ra == 1 or rb == 1)) or
            (ra == 1 and ca == 1) or (rb == 1 and cb == 1) or (ca == 1 and rb == 1) or (ra == 1 and cb == 1))


def out_shape(prog: CellProgram, shapes):
    """Result shape of the program for input shapes (None: scalar); None if an operator would
    reject its operands (the sequential path then raises the operator's own error)."""
    regs = list(shapes) + [None] * (NR - len(shapes))
    for kind, o, d, a, b in prog.ops:
        if kind == "u":
            regs[d] = regs[a]
            continue
        sa, sb = regs[a], regs[b]
        if o in BIAS_OPS:
            if sa is None or sb is None or sb[1] != 1 or sb[0] <= 0 or sa[1] % sb[0]:
                return None
            regs[d] = sa
            continue
        if sa is None:
            regs[d] = sb
        elif sb is None:
            regs[d] = sa
        elif _bin_ok(sa, sb):
            regs[d] = (max(sa[0], sb[0]), max(sa[1], sb[1]))
        else:
            return None
    return regs[prog.out]


def chan_inputs(prog: CellProgram):
    """Input registers read as per-channel operands of bias+ / bias*, or None when the program
    is outside the generated kernels' scope: a channel operand that is an intermediate, or an
    input read both per channel and cellwise.  Registers are reused once their value is dead,
    so a register number names an input only until the first instruction writing it."""
    f = prog._code.get("chan", False)
    if f is not False:
        return f
    inputs = set(range(prog.n_in))            # registers still holding their input
    chan, cellwise = set(), set()
    ok = True
    for kind, o, d, a, b in prog.ops:
        if o in BIAS_OPS:
            if b not in inputs:
                ok = False
            chan.add(b)
            reads = (a,)
        else:
            reads = (a, b) if kind == "b" else (a,)
        cellwise.update(r for r in reads if r in inputs)
        inputs.discard(d)
    if chan & cellwise:
        ok = False
    f = frozenset(chan) if ok else None
    prog._code["chan"] = f
    return f


class _In(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("s", ctypes.c_double), ("mode", ctypes.c_int), ("dtype", ctypes.c_int),
                ("vec", ctypes.c_int), ("pad", ctypes.c_int)]


class _Prog(ctypes.Structure):
    _fields_ = [("inp", _In * MAXIN), ("rows", ctypes.c_int64), ("cols", ctypes.c_int64), ("total", ctypes.c_int64),
                ("n_in", ctypes.c_int), ("n_ops", ctypes.c_int), ("out", ctypes.c_int), ("aggop", ctypes.c_int),
                ("need_ij", ctypes.c_int), ("pad", ctypes.c_int)]


_DT = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2}
_Tensor = torch.Tensor
_checked = []


def _lib():
    from . import kernels
    L = kernels.load(required=True)
    if not _checked:
        L.sysml_cell.restype = ctypes.c_int
        L.sysml_cell.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                 ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p]
        L.sysml_cell_blocks.restype = ctypes.c_int64
        L.sysml_cell_blocks.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_int64]
        L.sysml_cell_prog_size.restype = ctypes.c_int
        if L.sysml_cell_prog_size() != ctypes.sizeof(_Prog):
            raise RuntimeError("cell.hip Prog layout does not match ops/cell.py")
        _checked.append(True)
    return L


# ----------------------------------------------------------------------------- code generation
def _cases(vals):
    expr = str(vals[-1])
    for k in range(len(vals) - 2, -1, -1):
        expr = f"(k == {k}) ? {vals[k]} : {expr}"
    return expr


def generate(prog: CellProgram, T, modes, dts, vecs, mode, variant, idx32=False, outbf=False, ch4=False):
    """HIP source of the fused kernel: the program as straight-line code over the cell values
    of its inputs, instantiated into the flat / row / column kernel template.  idx32: the
    operand has < 2^31 cells (32-bit row / column arithmetic); outbf: the (unaggregated)
    result is stored as bf16; ch4: every per-channel operand's H*W and the column count are
    multiples of 4 (a 4-cell group lies in one channel: one load instead of four)."""
    ct = "float" if T == torch.float32 else "double"
    var = [f"x[{k}]" for k in range(prog.n_in)] + [None] * (NR - prog.n_in)
    body = []
    for q, (kind, o, d, a, b) in enumerate(prog.ops):
        e = (_C_BIN[o] if kind == "b" else _C_UN[o]).format(a=var[a], b=var[b] if kind == "b" else "")
        body.append(f"    const T v{q} = {e};")
        var[d] = f"v{q}"
    aggop = AGG_CODES[prog.agg[0]] if prog.agg else 0
    need_ij = int(any(m in (ROWV, COLV, CHAN) for m in modes))
    if mode == 0:
        call = "sysml_cell_flat<Spec, 0>(A);"
    elif mode == 1:
        call = "sysml_cell_flat<Spec, 1>(A);"
    elif mode == 2:
        call = (f"sysml_cell_row4<Spec, {variant - COL4}>(A);" if variant >= COL4
                else f"sysml_cell_row<Spec, {variant}>(A);")
    elif variant >= COL4:
        call = f"sysml_cell_col4<Spec, {variant - COL4}>(A);"
    else:
        call = f"sysml_cell_col<Spec, {variant}>(A);"
    return (_prelude() + f"""
// generated: {prog.describe()}
struct Spec {{
  typedef {ct} T;
  static constexpr int NIN = {prog.n_in};
  static constexpr int AGGOP = {aggop};
  static constexpr int NEED_IJ = {need_ij};
  static constexpr int IDX32 = {int(bool(idx32))};
  static constexpr int OUTBF = {int(bool(outbf))};
  static constexpr int CH4 = {int(bool(ch4))};
  static constexpr int mode(int k) {{ return {_cases(modes)}; }}
  static constexpr int dt(int k) {{ return {_cases(dts)}; }}
  static constexpr int vec(int k) {{ return {_cases(vecs)}; }}
  static __device__ __forceinline__ T f(const T (&x)[NIN]) {{
{chr(10).join(body)}
    return {var[prog.out]};
  }}
}};

extern "C" __global__ void __launch_bounds__(256) {kernel_name(prog, mode, outbf)}(const SysmlCellArgs A) {{ {call} }}
""")


_OPNAME = {"+": "add", "-": "sub", "*": "mul", "/": "div", "^": "pow", "%%": "mod", "%/%": "idiv", "==": "eq",
           "!=": "ne", "<": "lt", "<=": "le", ">": "gt", ">=": "ge", "&": "and", "|": "or", "bias+": "badd",
           "bias*": "bmul"}


def kernel_name(prog, mode, outbf=False):
    """Symbol of a generated kernel: its operators, aggregate and output type, so rocprofv3's
    per-kernel statistics tell the fused programs apart (sysml_cell_<ops>[_<agg>][_bf])."""
    ops = "_".join(_OPNAME.get(o, o) for _, o, _, _, _ in prog.ops)[:80] or "copy"
    agg = f"_{prog.agg[0]}{prog.agg[1]}" if prog.agg else ""
    return f"sysml_cell_{ops}{agg}{'_bf' if outbf else ''}"


_PRELUDE = []


def _prelude():
    if not _PRELUDE:
        here = os.path.dirname(os.path.abspath(__file__))
        with open(os.path.join(here, "hip", "cell_rtc.inc")) as f:
            _PRELUDE.append("#pragma clang fp contract(off)\n" + f.read())
    return _PRELUDE[0]


class _RtcArgs(ctypes.Structure):
    _fields_ = [("inp", ctypes.c_void_p * MAXIN), ("s", ctypes.c_double * MAXIN), ("rows", ctypes.c_int64),
                ("cols", ctypes.c_int64), ("total", ctypes.c_int64), ("chunk", ctypes.c_int64),
                ("out", ctypes.c_void_p), ("part", ctypes.c_void_p)]


_rtc_funcs = {}
_rtc_bound = []
_arch = {}


def _rtc_lib():
    from . import kernels
    L = kernels.load(required=True)
    if not _rtc_bound:
        L.sysml_rtc_compile.restype = ctypes.c_int
        L.sysml_rtc_compile.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                        ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t),
                                        ctypes.c_char_p, ctypes.c_size_t]
        L.sysml_rtc_code.restype = ctypes.c_int
        L.sysml_rtc_code.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.sysml_rtc_load.restype = ctypes.c_int
        L.sysml_rtc_load.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
        L.sysml_rtc_launch.restype = ctypes.c_int
        L.sysml_rtc_launch.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint, ctypes.c_uint, ctypes.c_void_p,
                                       ctypes.c_size_t, ctypes.c_void_p]
        _rtc_bound.append(True)
    return L


def gpu_arch(dev=None):
    """gfx target of the device (e.g. 'gfx950'); the code objects are built for it."""
    k = str(dev)
    a = _arch.get(k)
    if a is None:
        try:
            a = torch.cuda.get_device_properties(dev).gcnArchName.split(":")[0] or "gfx950"
        except Exception:
            a = "gfx950"
        _arch[k] = a
    return a


def compile_source(src, arch):
    """Code object bytes of `src` (hipRTC), through the on-disk cache keyed by source + arch."""
    L = _rtc_lib()
    h = hashlib.sha1((arch + "\0" + src).encode()).hexdigest()
    path = os.path.join(RTC_DIR, f"cell-{h}.co")
    try:
        with open(path, "rb") as f:
            stats["rtc_cache_hits"] += 1
            return f.read()
    except OSError:
        pass
    t0 = time.perf_counter()
    handle, size = ctypes.c_void_p(), ctypes.c_size_t()
    log = ctypes.create_string_buffer(8192)
    rc = L.sysml_rtc_compile(src.encode(), b"sysml_cell.hip", arch.encode(), ctypes.byref(handle),
                             ctypes.byref(size), log, len(log))
    if rc != 0:
        raise RuntimeError(f"hipRTC compilation failed ({rc}): {log.value.decode(errors='replace')[:2000]}")
    buf = ctypes.create_string_buffer(size.value)
    rc = L.sysml_rtc_code(handle, buf)
    if rc != 0:
        raise RuntimeError(f"hipRTC code retrieval failed ({rc})")
    code = buf.raw
    stats["rtc_compiled"] += 1
    stats["rtc_compile_s"] = stats.get("rtc_compile_s", 0.0) + time.perf_counter() - t0
    try:
        os.makedirs(RTC_DIR, exist_ok=True)
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as f:
            f.write(code)
        os.replace(tmp, path)
    except OSError:
        pass
    return code


def _rtc_func(prog, T, modes, dts, vecs, mode, variant, dev, idx32=False, outbf=False, ch4=False):
    key = (prog.key(), T, modes, dts, vecs, mode, variant, str(dev), idx32, outbf, ch4)
    f = _rtc_funcs.get(key, False)
    if f is not False:
        return f
    try:
        code = compile_source(generate(prog, T, modes, dts, vecs, mode, variant, idx32, outbf, ch4), gpu_arch(dev))
        L = _rtc_lib()
        fn = ctypes.c_void_p()
        cbuf = ctypes.create_string_buffer(code, len(code))
        rc = L.sysml_rtc_load(cbuf, kernel_name(prog, mode, outbf).encode(), ctypes.byref(fn))
        if rc != 0:
            raise RuntimeError(f"hipModuleLoadData failed ({rc})")
        f = (fn, cbuf)
    except RuntimeError as e:                 # interpreter kernel instead, once per signature
        import warnings
        warnings.warn(f"fused cell kernel not compiled, using the interpreter: {e}")
        f = None
    _rtc_funcs[key] = f
    return f


_S = "s"
_plans = {}


_DevScalar = []


def _signature(args):
    """Hashable operand signature (shapes, dtypes, devices, layout, alignment) or None."""
    if not _DevScalar:
        from ..runtime.scalars import DevScalar as _D
        _DevScalar.append(_D)
    DevScalar = _DevScalar[0]
    sig = []
    for x in args:
        tx = type(x)
        if tx is _Tensor:
            if x.layout is not torch.strided:
                return None               # sparse operands: the sequential operators' sparse paths
            sig.append((x.shape, x.dtype, x.device, x.layout, x.is_contiguous(), x.data_ptr() & 15))
        elif tx is DevScalar:
            sig.append(("d", x.t.dtype, x.t.device))
        elif tx is float or tx is int or tx is bool:
            sig.append(_S)
        else:
            return None
    return tuple(sig)


class _Plan:
    """Everything a launch of one program on one operand signature needs but the pointers."""
    __slots__ = ("prog", "fn", "interp", "mode", "nblk", "gx", "gy", "R", "Cc", "T", "odt", "out_shape",
                 "part_shape", "kinds", "P", "dev", "dev_index", "launch", "count", "hws")


def _make_plan(prog, args):
    from ..runtime.scalars import DevScalar
    if len(args) != prog.n_in or len(prog.ops) > MAXOPS or prog.n_in > MAXIN:
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
    shp = out_shape(prog, shapes)
    if shp is None:
        return None
    R, Cc = shp
    if R <= 0 or Cc <= 0:
        return None
    T = torch.float64 if (f64 or (bf16 and backend.dtype == torch.float64)) else torch.float32
    chan = chan_inputs(prog)
    if chan is None or (chan and not RTC):
        return None                   # per-channel operands: generated kernels only, inputs only
    P = _Prog()
    kinds = []
    need_ij = 0
    hws = {}
    for k, x in enumerate(args):
        e = P.inp[k]
        tx = type(x)
        if k in chan:
            if tx is not _Tensor or x.shape[1] != 1 or Cc % x.shape[0]:
                return None
            e.dtype = _DT[x.dtype]
            e.mode = CHAN
            hws[k] = Cc // x.shape[0]
            need_ij = 1
            kinds.append("c")
            continue
        if tx is _Tensor:
            r, c = x.shape
            e.dtype = _DT[x.dtype]
            if (r, c) == (R, Cc):
                e.mode = FULL
                e.vec = int(x.is_contiguous() and x.data_ptr() % 16 == 0)
            elif r == 1 and c == 1:
                e.mode = DSCALAR
            elif r == 1 and c == Cc:
                e.mode = ROWV
                need_ij = 1
            elif c == 1 and r == R:
                e.mode = COLV
                need_ij = 1
            else:
                return None
            kinds.append("t")
        elif tx is DevScalar:
            e.dtype = _DT[x.t.dtype]
            e.mode = DSCALAR
            kinds.append("d")
        else:
            e.mode = HSCALAR
            kinds.append("s")
    P.rows, P.cols, P.total = R, Cc, R * Cc
    P.n_in, P.n_ops, P.out = prog.n_in, len(prog.ops), prog.out
    P.need_ij = need_ij
    agg = prog.agg
    mode = 0
    if agg:
        P.aggop = AGG_CODES[agg[0]]
        mode = AGG_DIRS[agg[1]]
    L = _lib()
    nblk = L.sysml_cell_blocks(mode, R, Cc)
    pl = _Plan()
    pl.prog, pl.mode, pl.nblk, pl.R, pl.Cc, pl.T, pl.kinds, pl.P, pl.dev = prog, mode, nblk, R, Cc, T, kinds, P, dev
    pl.dev_index = dev.index if dev.index is not None else torch.cuda.current_device()
    pl.out_shape = (R, Cc) if mode == 0 else ((R, 1) if mode == 2 else None)
    pl.part_shape = (nblk,) if mode == 1 else ((nblk, Cc) if mode == 3 else None)
    pl.fn = None
    pl.odt = T
    pl.gx, pl.gy = nblk, 1
    if RTC:
        modes = tuple(P.inp[k].mode for k in range(prog.n_in))
        dts = tuple(P.inp[k].dtype for k in range(prog.n_in))
        vecs = tuple(P.inp[k].vec for k in range(prog.n_in))
        if mode == 2:
            variant = 1 if Cc <= 8 else (4 if Cc <= 32 else (16 if Cc <= 128 else 64))
            if ROW4 and Cc % 4 == 0 and Cc >= 64:
                g4 = Cc // 4
                variant = COL4 + (64 if g4 >= 64 else (16 if g4 >= 16 else 4))   # 4 cells per lane
        elif mode == 3:
            variant = 8 if Cc <= 8 else 64
            if Cc % 4 == 0 and Cc >= 1024:
                variant = COL4 + 64           # 4 adjacent columns per lane, vector loads
        else:
            variant = 0
        outbf = mode == 0 and T == torch.float32 and 0 < backend.act_bf16_min_cells <= R * Cc
        ch4 = bool(hws) and Cc % 4 == 0 and all(h % 4 == 0 for h in hws.values())
        f = _rtc_func(prog, T, modes, dts, vecs, mode, variant, dev, R * Cc < 2 ** 31, outbf, ch4)
        if f is not None:
            pl.fn = f[0]
            if outbf:
                pl.odt = torch.bfloat16
            if mode == 3:
                cols_per_block = 4 * (variant - COL4) if variant >= COL4 else variant
                pl.gx, pl.gy = (Cc + cols_per_block - 1) // cols_per_block, nblk
                if nblk == 1:                 # one row block writes the column aggregate itself
                    pl.out_shape, pl.part_shape = (1, Cc), None
    pl.interp = pl.fn is None
    pl.hws = hws
    if chan and pl.interp:
        return None
    pl.launch = _rtc_lib().sysml_rtc_launch
    from . import kernels
    pl.count = kernels._count
    return pl


_raw_stream = torch._C._cuda_getCurrentRawStream if hasattr(torch._C, "_cuda_getCurrentRawStream") else None


def _kernel(prog: CellProgram, args):
    """One launch of the cell kernel, or None when the operands are outside its scope.  The
    launch plan (generated kernel, grid, modes) is cached per program and operand signature,
    so a repeated call only fills the pointers and launches."""
    sig = _signature(args)
    if sig is None:
        return None
    key = (id(prog), sig, RTC, backend.act_bf16_min_cells)
    pl = _plans.get(key, False)
    if pl is False or (pl is not None and pl.prog is not prog):
        pl = _make_plan(prog, args)
        _plans[key] = pl
    if pl is None:
        return None
    dev, T, mode = pl.dev, pl.T, pl.mode
    out = torch.empty(pl.out_shape, dtype=pl.odt, device=dev) if pl.out_shape is not None else None
    part = torch.empty(pl.part_shape, dtype=torch.float64, device=dev) if pl.part_shape is not None else None
    st = _raw_stream(pl.dev_index) if _raw_stream is not None else torch.cuda.current_stream(dev).cuda_stream
    keep = []
    if not pl.interp:
        A = _RtcArgs()
        for k, (x, kd) in enumerate(zip(args, pl.kinds)):
            if kd == "t" or kd == "c":
                if not x.is_contiguous():
                    x = x.contiguous()
                    keep.append(x)
                A.inp[k] = x.data_ptr()
                if kd == "c":
                    A.s[k] = pl.hws[k]
            elif kd == "d":
                t = x.t.reshape(1)
                keep.append(t)
                A.inp[k] = t.data_ptr()
            else:
                A.s[k] = float(x)
        A.rows, A.cols, A.total = pl.R, pl.Cc, pl.R * pl.Cc
        A.chunk = (pl.R + pl.nblk - 1) // pl.nblk
        A.out = out.data_ptr() if out is not None else 0
        A.part = part.data_ptr() if part is not None else 0
        rc = pl.launch(pl.fn, pl.gx, pl.gy, 256, ctypes.byref(A), ctypes.sizeof(A), st)
        if rc != 0:
            raise RuntimeError(f"fused cell kernel launch failed: {rc}")
        stats["rtc_launches"] += 1
    else:
        P = _Prog()
        ctypes.memmove(ctypes.byref(P), ctypes.byref(pl.P), ctypes.sizeof(P))
        for k, (x, kd) in enumerate(zip(args, pl.kinds)):
            e = P.inp[k]
            if kd == "t":
                if not x.is_contiguous():
                    x = x.contiguous()
                keep.append(x)
                e.p = x.data_ptr()
            elif kd == "d":
                t = x.t.reshape(1)
                keep.append(t)
                e.p = t.data_ptr()
            else:
                e.s = float(x)
        code = prog.device_code(dev)
        dt = 0 if T == torch.float32 else 1
        rc = _lib().sysml_cell(dt, mode, ctypes.byref(P), code.data_ptr(), out.data_ptr() if out is not None else 0,
                               part.data_ptr() if part is not None else 0, pl.nblk, st)
        if rc != 0:
            raise RuntimeError(f"sysml_cell failed: {rc}")
        stats["interpreter_launches"] += 1
    pl.count("cell")
    del keep
    if mode == 0:
        return out
    agg = prog.agg
    o = agg[0]
    R, Cc = pl.R, pl.Cc
    if mode == 1:
        r = part.sum() if AGG_CODES[o] <= 1 else (part.min() if o == "min" else part.max())
        if o == "mean":
            r = r / (R * Cc)
        return C._lazy_out(r)
    if mode == 2:
        return out / Cc if o == "mean" else out
    if part is None:
        r = out
    else:
        # row-block partials folded on agg.hip (fp64 in, T out): no ATen reduce + cast
        from . import kernels
        ko = "sum" if AGG_CODES[o] <= 1 or o == "mean" else o
        r = kernels.fold_rows(part, ko, T)
        if r is None:
            r = part.sum(0, keepdim=True) if AGG_CODES[o] <= 1 else (part.amin(0, keepdim=True) if o == "min"
                                                                     else part.amax(0, keepdim=True))
            r = r.to(T)
    return r / R if o == "mean" else r


# ----------------------------------------------------------------------------- horizontal batches
class _HTab(ctypes.Structure):
    """One operand set of a batched Cell launch (mirrors SysmlHT of generate_batch)."""
    _fields_ = [("inp", ctypes.c_void_p * MAXIN), ("s", ctypes.c_double * MAXIN), ("out", ctypes.c_void_p),
                ("total", ctypes.c_int64), ("b0", ctypes.c_int64)]


class _HArgs(ctypes.Structure):
    _fields_ = [("tab", ctypes.c_void_p), ("nt", ctypes.c_int), ("pad", ctypes.c_int)]


BATCH_CELLS = 4 * 256                  # cells per workgroup of the batched kernel
_hpinned = []                          # pinned host tables in flight (kept until reused)


def generate_batch(prog: CellProgram, T, modes, dts):
    """HIP source of the batched kernel: workgroup b finds its operand set t (the last table entry
    with b0 <= b) and computes 4 cells per lane of that set's output."""
    ct = "float" if T == torch.float32 else "double"
    var = [f"x[{k}]" for k in range(prog.n_in)] + [None] * (NR - prog.n_in)
    body = []
    for q, (kind, o, d, a, b) in enumerate(prog.ops):
        e = (_C_BIN[o] if kind == "b" else _C_UN[o]).format(a=var[a], b=var[b] if kind == "b" else "")
        body.append(f"    const T v{q} = {e};")
        var[d] = f"v{q}"
    loads = []
    for k in range(prog.n_in):
        if modes[k] == FULL:
            loads.append(f"        x[{k}] = sysml_ld<T>(A.in[{k}], {dts[k]}, e);")
        elif modes[k] == DSCALAR:
            loads.append(f"        x[{k}] = sysml_ld<T>(A.in[{k}], {dts[k]}, 0);")
        else:
            loads.append(f"        x[{k}] = (T)A.s[{k}];")
    name = "sysml_hcell_" + kernel_name(prog, 0)[len("sysml_cell_"):]
    return (_prelude() + f"""
// generated (batched): {prog.describe()}
struct SysmlHT {{ const void* in[{MAXIN}]; double s[{MAXIN}]; void* out; long long total; long long b0; }};
struct Spec {{
  typedef {ct} T;
  static constexpr int NIN = {prog.n_in};
  static __device__ __forceinline__ T f(const T (&x)[NIN]) {{
{chr(10).join(body)}
    return {var[prog.out]};
  }}
}};

extern "C" __global__ void __launch_bounds__(256) {name}(const SysmlHT* __restrict__ tab, const int nt) {{
  typedef Spec::T T;
  int lo = 0, hi = nt - 1;
  while (lo < hi) {{
    const int mid = (lo + hi + 1) >> 1;
    if (tab[mid].b0 <= (long long)blockIdx.x) lo = mid; else hi = mid - 1;
  }}
  const SysmlHT& A = tab[lo];
  const long long e0 = ((long long)blockIdx.x - A.b0) * {BATCH_CELLS} + threadIdx.x;
#pragma unroll
  for (int v = 0; v < 4; ++v) {{
    const long long e = e0 + v * 256;
    if (e < A.total) {{
      T x[Spec::NIN];
{chr(10).join(loads)}
      static_cast<T*>(A.out)[e] = Spec::f(x);
    }}
  }}
}}
"""), name


def evaluate_batch(prog: CellProgram, n, args):
    """n evaluations of one unaggregated Cell program (compiler/codegen.batch_cells), args the n
    operand lists concatenated; returns the tuple of results.  On the MI355X one launch of a
    generated batched kernel covers all of them when they agree in operand kinds and dtypes;
    otherwise each runs on its own."""
    k = prog.n_in
    sets = [list(args[i * k:(i + 1) * k]) for i in range(n)]
    if backend.use_kernels:
        r = _batch_kernel(prog, sets)
        if r is not None:
            stats["batched"] = stats.get("batched", 0) + n
            return r
    return tuple(evaluate(prog, a) for a in sets)


def _batch_kernel(prog, sets):
    from ..runtime.scalars import DevScalar
    first = sets[0]
    modes, dts, shapes = [], [], []
    dev = None
    f64 = False
    for x in first:
        if type(x) is _Tensor:
            if not x.is_cuda or x.layout is not torch.strided or x.dtype not in _DT:
                return None
            dev = x.device
            modes.append(FULL if x.numel() > 1 or x.dim() == 2 and x.shape != (1, 1) else DSCALAR)
            dts.append(_DT[x.dtype])
            f64 |= x.dtype == torch.float64
        elif type(x) is DevScalar:
            modes.append(DSCALAR)
            dts.append(_DT[torch.float64])
        elif isinstance(x, (int, float, bool)):
            modes.append(HSCALAR)
            dts.append(0)
        else:
            return None
    if dev is None:
        return None
    T = torch.float64 if (f64 or backend.dtype == torch.float64) else torch.float32
    n = len(sets)
    tabs = (_HTab * n)()
    outs = []
    keep = []
    b0 = 0
    for i, a in enumerate(sets):
        e = tabs[i]
        shape = None
        for q, x in enumerate(a):
            tx = type(x)
            if modes[q] == FULL:
                if tx is not _Tensor or x.dtype not in _DT or _DT[x.dtype] != dts[q] or x.device != dev \
                        or x.layout is not torch.strided:
                    return None
                if shape is None:
                    shape = tuple(x.shape)
                elif tuple(x.shape) != shape:
                    return None
                if not x.is_contiguous():
                    x = x.contiguous()
                keep.append(x)
                e.inp[q] = x.data_ptr()
            elif modes[q] == DSCALAR:
                t = x.t.reshape(1) if tx is DevScalar else \
                    (x.reshape(1) if tx is _Tensor and x.numel() == 1 else None)
                if t is None or not t.is_cuda or t.dtype not in _DT or _DT[t.dtype] != dts[q]:
                    return None
                keep.append(t)
                e.inp[q] = t.data_ptr()
            else:
                if not isinstance(x, (int, float, bool)):
                    return None
                e.s[q] = float(x)
        if shape is None:
            return None
        if 0 < backend.act_bf16_min_cells <= shape[0] * shape[1]:
            return None                         # the single-operand plan would store this one bf16
        y = torch.empty(shape, dtype=T, device=dev)
        outs.append(y)
        e.out = y.data_ptr()
        e.total = y.numel()
        e.b0 = b0
        b0 += (y.numel() + BATCH_CELLS - 1) // BATCH_CELLS
    if b0 == 0 or b0 >= 2 ** 31:
        return None
    key = ("hcell", prog.key(), T, tuple(modes), tuple(dts), str(dev))
    f = _rtc_funcs.get(key, False)
    if f is False:
        try:
            src, name = generate_batch(prog, T, tuple(modes), tuple(dts))
            code = compile_source(src, gpu_arch(dev))
            fn = ctypes.c_void_p()
            cbuf = ctypes.create_string_buffer(code, len(code))
            rc = _rtc_lib().sysml_rtc_load(cbuf, name.encode(), ctypes.byref(fn))
            if rc != 0:
                raise RuntimeError(f"hipModuleLoadData failed ({rc})")
            f = (fn, cbuf)
        except RuntimeError as ex:
            import warnings
            warnings.warn(f"batched cell kernel not compiled, the updates run one by one: {ex}")
            f = None
        _rtc_funcs[key] = f
    if f is None:
        return None
    nb = ctypes.sizeof(tabs)
    host = torch.empty((nb,), dtype=torch.uint8, pin_memory=True)
    ctypes.memmove(host.data_ptr(), ctypes.addressof(tabs), nb)
    dtab = host.to(dev, non_blocking=True)
    _hpinned.append(host)                       # alive until the copy has run (a short ring)
    if len(_hpinned) > 64:
        del _hpinned[:32]
    A = _HArgs()
    A.tab = dtab.data_ptr()
    A.nt = n
    st = torch.cuda.current_stream(dev).cuda_stream
    rc = _rtc_lib().sysml_rtc_launch(f[0], b0, 1, 256, ctypes.byref(A), ctypes.sizeof(A), st)
    if rc != 0:
        raise RuntimeError(f"batched cell kernel launch failed: {rc}")
    stats["rtc_launches"] += 1
    from . import kernels
    kernels._count("hcell")
    del keep
    return tuple(outs)


# ----------------------------------------------------------------------------- multi-aggregate
MAGG_COL_CW = 64           # column groups (of 4 columns) per workgroup of the column MAgg kernel


class MultiAggProgram:
    """MAgg template (reference: hops/codegen/template/TemplateMultiAgg.java, runtime
    SpoofMultiAggregate): several full aggregates of cellwise programs over the same output
    cells, evaluated in ONE pass over their shared inputs.  progs[k] reads its registers
    0..n_in-1 from the union inputs maps[k][0..n_in-1]."""
    __slots__ = ("progs", "maps", "n_in")

    def __init__(self, progs, maps, n_in):
        self.progs = tuple(progs)
        self.maps = tuple(tuple(m) for m in maps)
        self.n_in = n_in

    def key(self):
        return (tuple(p.key() for p in self.progs), self.maps, self.n_in)

    def describe(self):
        return "magg[" + ";".join(p.describe() for p in self.progs) + "]"

    def __repr__(self):
        return self.describe()


def evaluate_multi(m: MultiAggProgram, args):
    """Tuple of the aggregates: one fused kernel on the MI355X, else each program alone."""
    r = _kernel_multi(m, args) if backend.use_kernels and RTC else None
    if r is not None:
        stats["magg_kernel"] = stats.get("magg_kernel", 0) + 1
        return r
    stats["magg_split"] = stats.get("magg_split", 0) + 1
    return tuple(evaluate(p, [args[i] for i in mp]) for p, mp in zip(m.progs, m.maps))


def generate_multi(m: MultiAggProgram, T, modes, dts, vecs, col=False, ch4=False):
    ct = "float" if T == torch.float32 else "double"
    body, outs = [], []
    q = 0
    for k, (prog, mp) in enumerate(zip(m.progs, m.maps)):
        var = [f"x[{mp[r]}]" for r in range(prog.n_in)] + [None] * (NR - prog.n_in)
        for kind, o, d, a, b in prog.ops:
            e = (_C_BIN[o] if kind == "b" else _C_UN[o]).format(a=var[a], b=var[b] if kind == "b" else "")
            body.append(f"    const T v{q} = {e};")
            var[d] = f"v{q}"
            q += 1
        outs.append(f"    o[{k}] = {var[prog.out]};")
    aggs = [AGG_CODES[p.agg[0]] for p in m.progs]
    need_ij = int(any(x in (ROWV, COLV, CHAN) for x in modes))
    call = f"sysml_cell_magg_col4<Spec, {MAGG_COL_CW}>(A);" if col else "sysml_cell_magg<Spec>(A);"
    return (_prelude() + f"""
// generated: {m.describe()}
struct Spec {{
  typedef {ct} T;
  static constexpr int NIN = {m.n_in};
  static constexpr int NOUT = {len(m.progs)};
  static constexpr int NEED_IJ = {need_ij};
  static constexpr int IDX32 = 0;
  static constexpr int CH4 = {int(ch4)};
  static constexpr int mode(int k) {{ return {_cases(modes)}; }}
  static constexpr int dt(int k) {{ return {_cases(dts)}; }}
  static constexpr int vec(int k) {{ return {_cases(vecs)}; }}
  static constexpr int aggop(int k) {{ return {_cases(aggs)}; }}
  static __device__ __forceinline__ void f(const T (&x)[NIN], T (&o)[NOUT]) {{
{chr(10).join(body)}
{chr(10).join(outs)}
  }}
}};

extern "C" __global__ void __launch_bounds__(256) sysml_cell_k(const SysmlCellArgs A) {{ {call} }}
""")


def _kernel_multi(m: MultiAggProgram, args):
    from ..runtime.scalars import DevScalar
    if len(args) != m.n_in or m.n_in > MAXIN:
        return None
    dev, shapes, f64, bf16 = None, [], False, False
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
        elif tx is float or tx is int or tx is bool:
            shapes.append(None)
        else:
            return None
    if dev is None:
        return None
    outs = {out_shape(p, [shapes[i] for i in mp]) for p, mp in zip(m.progs, m.maps)}
    if len(outs) != 1:
        return None                      # different cell domains: evaluated one by one
    shp = outs.pop()
    if shp is None or shp[0] <= 0 or shp[1] <= 0:
        return None
    R, Cc = shp
    dirs = {p.agg[1] for p in m.progs}
    if len(dirs) != 1:
        return None
    col = dirs.pop() == "col"
    if col and (Cc % 4 or any(p.agg[0] not in ("sum", "sumsq", "mean") for p in m.progs)):
        return None
    # per-channel operands (bias_add / bias_multiply inside the programs): union positions
    chan = set()
    for p, mp in zip(m.progs, m.maps):
        ci = chan_inputs(p)
        if ci is None:
            return None
        chan |= {mp[i] for i in ci}
    T = torch.float64 if (f64 or (bf16 and backend.dtype == torch.float64)) else torch.float32
    A = _RtcArgs()
    keep, modes, dts, vecs = [], [], [], []
    hws = []
    for k, x in enumerate(args):
        tx = type(x)
        mode, dt, vec = HSCALAR, 0, 0
        if k in chan:
            if tx is not _Tensor or x.dim() != 2 or x.shape[1] != 1 or Cc % x.shape[0]:
                return None
            if not x.is_contiguous():
                x = x.contiguous()
            keep.append(x)
            A.inp[k] = x.data_ptr()
            A.s[k] = Cc // x.shape[0]
            hws.append(Cc // x.shape[0])
            modes.append(CHAN)
            dts.append(_DT[x.dtype])
            vecs.append(0)
            continue
        if tx is _Tensor:
            if not x.is_contiguous():
                x = x.contiguous()
            keep.append(x)
            r, c = x.shape
            A.inp[k] = x.data_ptr()
            dt = _DT[x.dtype]
            if (r, c) == (R, Cc):
                mode, vec = FULL, int(x.data_ptr() % 16 == 0)
            elif r == 1 and c == 1:
                mode = DSCALAR
            elif r == 1 and c == Cc:
                mode = ROWV
            elif c == 1 and r == R:
                mode = COLV
            else:
                return None
        elif tx is DevScalar:
            t = x.t.reshape(1)
            keep.append(t)
            A.inp[k] = t.data_ptr()
            dt, mode = _DT[t.dtype], DSCALAR
        else:
            A.s[k] = float(x)
        modes.append(mode)
        dts.append(dt)
        vecs.append(vec)
    ch4 = bool(hws) and Cc % 4 == 0 and all(h % 4 == 0 for h in hws)
    if hws and not col:
        return None                      # per-channel operands: column form only
    key = ("magg", m.key(), T, tuple(modes), tuple(dts), tuple(vecs), str(dev), col, ch4)
    f = _rtc_funcs.get(key, False)
    if f is False:
        try:
            code = compile_source(generate_multi(m, T, tuple(modes), tuple(dts), tuple(vecs), col, ch4),
                                  gpu_arch(dev))
            fn = ctypes.c_void_p()
            cbuf = ctypes.create_string_buffer(code, len(code))
            rc = _rtc_lib().sysml_rtc_load(cbuf, b"sysml_cell_k", ctypes.byref(fn))
            if rc != 0:
                raise RuntimeError(f"hipModuleLoadData failed ({rc})")
            f = (fn, cbuf)
        except RuntimeError as e:
            import warnings
            warnings.warn(f"multi-aggregate kernel not compiled, aggregates run separately: {e}")
            f = None
        _rtc_funcs[key] = f
    if f is None:
        return None
    nout = len(m.progs)
    if col:
        nblk = _lib().sysml_cell_blocks(3, R, Cc)
        part = torch.empty((nblk, nout, Cc), dtype=torch.float64, device=dev)
        gx, gy = (Cc + 4 * MAGG_COL_CW - 1) // (4 * MAGG_COL_CW), nblk
    else:
        nblk = _lib().sysml_cell_blocks(1, R, Cc)
        part = torch.empty(nblk * nout, dtype=torch.float64, device=dev)
        gx, gy = nblk, 1
    A.rows, A.cols, A.total = R, Cc, R * Cc
    A.chunk = (R + nblk - 1) // nblk
    A.out = 0
    A.part = part.data_ptr()
    st = torch.cuda.current_stream(dev).cuda_stream
    rc = _rtc_lib().sysml_rtc_launch(f[0], gx, gy, 256, ctypes.byref(A), ctypes.sizeof(A), st)
    if rc != 0:
        raise RuntimeError(f"multi-aggregate kernel launch failed: {rc}")
    stats["rtc_launches"] += 1
    from . import kernels
    kernels._count("magg")
    del keep
    if col:
        # the workgroup partials of all outputs in one column reduction (agg.hip; torch's
        # per-output sum + cast was two ATen launches per output)
        tot = kernels.fold_rows(part.view(nblk, nout * Cc), "sum", T)
        if tot is None:
            tot = part.sum(0).to(T)
        tot = tot.view(nout, Cc)
        res = []
        for k, prog in enumerate(m.progs):
            r = tot[k:k + 1]
            res.append(r / R if prog.agg[0] == "mean" else r)
        return tuple(res)
    P = part.view(nblk, nout)
    res = []
    for k, prog in enumerate(m.progs):
        o = prog.agg[0]
        col = P[:, k]
        r = col.sum() if AGG_CODES[o] <= 1 else (col.min() if o == "min" else col.max())
        if o == "mean":
            r = r / (R * Cc)
        res.append(C._lazy_out(r))
    return tuple(res)
