"""DML scalar semantics: value types, arithmetic, comparison, casting and
Java-compatible string formatting.

Reference behaviour: runtime/instructions/cp/{Int,Double,Boolean,String}Object.java
(Double.toString, Long.toString, upper-cased booleans), runtime/functionobjects/
{Plus,Minus,Multiply,Divide,Power,Modulus,IntegerDivide,...}.java and
ScalarObjectFactory (INT op INT stays INT except for '/' and '^').
"""
from __future__ import annotations

import math
import weakref
from decimal import Decimal

from ..parser.errors import DMLRuntimeError

INF = float("inf")


class DevScalar:
    """A DML double/boolean scalar that stays resident in HBM as a 0-d fp64 tensor.

    Aggregates over HBM matrices (sum, tak+*, as.scalar, ...) return one instead of a Python
    float when the backend runs with lazy scalars, so an iterative script's scalar algebra
    (alphas, norms, convergence tests) is queued on the device behind the kernels that
    produce it; the host only synchronises where it must branch (a loop or if predicate), or
    where a value leaves the engine (print, casts, indexing, results).  Reference analogue:
    the CP ScalarObject (runtime/instructions/cp/DoubleObject.java), which is always on the
    JVM heap — on the GPU backend that costs a device round trip per scalar.
    """
    __slots__ = ("t", "vt", "_v", "_hb", "_ev", "_seq", "__weakref__")
    is_dev_scalar = True

    def __init__(self, t, vt="d"):
        self.t = t          # 0-d float64 tensor on the device
        self.vt = vt        # 'd' (DOUBLE) | 'b' (BOOLEAN) | 'i' (INT, held as a double)
        self._v = None
        self._hb = None     # pinned host copy in flight (start_read)
        self._ev = None
        self._seq = next(_dev_seq)
        _pending.append(weakref.ref(self))
        if len(_pending) > _PENDING_MAX:
            del _pending[:len(_pending) - _PENDING_MAX]

    def _convert(self, x):
        return (x != 0.0) if self.vt == "b" else (int(x) if self.vt == "i" else x)

    def _read_older(self):
        """One device read for this value and every unread device scalar queued before it (the
        same stream: they are complete when this one is), so the host's later branches and
        scalar algebra on them need no further synchronisation (the solvers' outer-loop
        bookkeeping: objective, ratios, trust-region tests).  Not in run-ahead loops, which
        read their predicate late on purpose."""
        import torch
        dev = self.t.device
        older = []
        for r in _pending:
            d = r()
            if d is not None and d._v is None and d._hb is None and d._seq < self._seq and d.t.device == dev \
                    and d.t.numel() == 1:
                older.append(d)
        if not older:
            return False
        older = older[-_BATCH_MAX:]           # the most recent: the values the next branches use
        older.append(self)
        vals = torch.stack([d.t.reshape(()).to(torch.float64) for d in older]).cpu().tolist()
        for d, x in zip(older, vals):
            d._v = d._convert(x)
        _pending[:] = [r for r in _pending if r() is not None and r()._v is None]
        return True

    def start_read(self):
        """Queue the device-to-host copy of the value behind the work that produces it and
        return at once; a later value() waits for that copy only (an event), not for work
        queued after it -- how a run-ahead loop reads its predicate one iteration late
        (runtime/program.py _exec_while_runahead)."""
        if self._v is None and self._hb is None:
            import torch
            hb = torch.empty(1, dtype=torch.float64, pin_memory=True)
            hb.copy_(self.t.reshape(1), non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            self._hb, self._ev = hb, ev
        return self

    def value(self):
        """Materialise (one device sync, cached)."""
        if self._v is None:
            if self._ev is not None:
                self._ev.synchronize()
                x = float(self._hb[0])
                self._hb = self._ev = None
            else:
                if BATCH_READS and self.t.is_cuda and not _in_runahead() and self._read_older():
                    return self._v
                x = float(self.t.item())
            self._v = self._convert(x)
        return self._v

    def __float__(self):
        return float(self.value())

    def __int__(self):
        return int(self.value())

    def __bool__(self):
        return bool(self.value())

    def __index__(self):
        return int(self.value())

    def __str__(self):
        return to_str(self.value())

    def __format__(self, spec):
        return format(self.value(), spec)

    def __repr__(self):
        return f"DevScalar({self.t!r}, {self.vt})"


_dev_seq = __import__("itertools").count()
_pending = []            # weak references to device scalars, creation order (DevScalar._read_older)
_PENDING_MAX = 256
_BATCH_MAX = 16
# SYSML_BATCH_SCALAR_READS=0: read every device scalar on its own
BATCH_READS = __import__("os").environ.get("SYSML_BATCH_SCALAR_READS", "1") != "0"


def _in_runahead():
    from ..ops.backend import backend
    return backend.defer


def materialize(v):
    """Python value of a possibly device-resident scalar (or deferred string)."""
    t = type(v)
    if t is DevScalar:
        return v.value()
    if t is LazyStr:
        return str(v)
    return v


class LazyStr:
    """A string built inside a run-ahead loop iteration (runtime/program.py) from device
    scalars whose values are not read yet -- LinearRegCG's per-iteration
    `print("Iteration " + it + ": ... " + sqrt(rr / rr0))` and its log appends.  The parts'
    device-to-host copies are queued at once (DevScalar.start_read), so resolving the string
    once the iteration is known to be live waits for those copies only.  The run-ahead loop
    prints a live iteration's strings in order and resolves every deferred string left in the
    variable map when it ends."""
    __slots__ = ("parts",)

    def __init__(self, parts):
        self.parts = parts

    def __str__(self):
        return "".join(p if type(p) is str else to_str(p) for p in self.parts)


def lazy_concat(a, b, sep=""):
    """a + sep + b as a LazyStr (parts flattened; device scalars' reads started)."""
    parts = []
    for x in (a, b):
        if type(x) is LazyStr:
            parts.extend(x.parts)
        elif type(x) is DevScalar:
            parts.append(x.start_read())
        else:
            parts.append(to_str(x))
        if sep and x is a:
            parts.append(sep)
    return LazyStr(parts)


def java_double_str(d: float) -> str:
    """Emulates java.lang.Double.toString."""
    if d != d:
        return "NaN"
    if d == INF:
        return "Infinity"
    if d == -INF:
        return "-Infinity"
    if d == 0.0:
        return "-0.0" if math.copysign(1.0, d) < 0 else "0.0"
    a = abs(d)
    r = repr(float(d))
    if 1e-3 <= a < 1e7:
        if "e" in r or "E" in r:
            r = format(Decimal(r), "f")
        if "." not in r:
            r += ".0"
        return r
    sign, digits, exp = Decimal(r).as_tuple()
    digits = list(digits)
    while len(digits) > 1 and digits[-1] == 0:
        digits.pop()
        exp += 1
    e10 = len(digits) - 1 + exp
    mant = str(digits[0]) + "." + ("".join(map(str, digits[1:])) or "0")
    return ("-" if sign else "") + mant + "E" + str(e10)


def to_str(v) -> str:
    if type(v) is DevScalar:
        v = v.value()
    elif type(v) is LazyStr:
        return str(v)
    if isinstance(v, bool):
        return "TRUE" if v else "FALSE"
    if isinstance(v, int):
        return str(v)
    if isinstance(v, float):
        return java_double_str(v)
    if isinstance(v, str):
        return v
    return str(v)


def vtype_of(v):
    if type(v) is DevScalar:
        return "BOOLEAN" if v.vt == "b" else ("INT" if v.vt == "i" else "DOUBLE")
    if isinstance(v, bool):
        return "BOOLEAN"
    if isinstance(v, int):
        return "INT"
    if isinstance(v, float):
        return "DOUBLE"
    if isinstance(v, str):
        return "STRING"
    return "UNKNOWN"


def as_double(v):
    if isinstance(v, str):
        try:
            return float(v)
        except ValueError:
            raise DMLRuntimeError(f"cannot cast string '{v}' to double")
    return float(v)


def as_int(v):
    if isinstance(v, str):
        try:
            return int(float(v))
        except ValueError:
            raise DMLRuntimeError(f"cannot cast string '{v}' to int")
    if isinstance(v, float):
        if v != v or v in (INF, -INF):
            raise DMLRuntimeError("cannot cast NaN/Inf to int")
        return int(v)   # truncation like Java (long) cast
    return int(v)


def as_bool(v):
    if isinstance(v, str):
        u = v.strip().upper()
        if u in ("TRUE", "T"):
            return True
        if u in ("FALSE", "F"):
            return False
        raise DMLRuntimeError(f"cannot cast string '{v}' to boolean")
    return bool(v != 0)


def _num(v):
    if isinstance(v, bool):
        return 1 if v else 0
    return v


def _r_mod(a, b):
    # R semantics: a - floor(a/b)*b
    if b == 0:
        return float("nan")
    return a - math.floor(a / b) * b


def _r_intdiv(a, b):
    if b == 0:
        if a == 0:
            return float("nan")
        return INF if a > 0 else -INF
    return math.floor(a / b)


def _pow(a, b):
    try:
        r = math.pow(a, b)
    except (OverflowError, ValueError):
        try:
            r = float(a) ** float(b)
            if isinstance(r, complex):
                return float("nan")
        except OverflowError:
            return INF
        except ZeroDivisionError:
            return INF
    return r


def _div(a, b):
    a = float(a)
    b = float(b)
    if b == 0.0:
        if a == 0.0 or a != a:
            return float("nan")
        return math.copysign(INF, a) * math.copysign(1.0, b)
    return a / b


def _cmp_prep(a, b):
    if isinstance(a, str) or isinstance(b, str):
        return to_str(a), to_str(b)
    return _num(a), _num(b)


def binary(op: str, a, b):
    """Scalar-scalar binary operation with DML typing rules."""
    if op == "+":
        if isinstance(a, str) or isinstance(b, str):
            return to_str(a) + to_str(b)
        a, b = _num(a), _num(b)
        return a + b
    if op in ("==", "!=", "<", "<=", ">", ">="):
        a, b = _cmp_prep(a, b)
        if op == "==":
            return a == b
        if op == "!=":
            return a != b
        if op == "<":
            return a < b
        if op == "<=":
            return a <= b
        if op == ">":
            return a > b
        return a >= b
    if op in ("&", "|", "xor"):
        x, y = as_bool(a), as_bool(b)
        if op == "&":
            return x and y
        if op == "|":
            return x or y
        return x != y
    if isinstance(a, str) or isinstance(b, str):
        raise DMLRuntimeError(f"operator '{op}' not supported for strings")
    a, b = _num(a), _num(b)
    both_int = isinstance(a, int) and isinstance(b, int)
    if op == "-":
        return a - b
    if op == "*":
        return a * b
    if op == "/":
        return _div(a, b)
    if op == "^":
        return _pow(float(a), float(b))
    if op == "%%":
        if both_int and b != 0:
            return a - (a // b) * b
        return _r_mod(float(a), float(b))
    if op == "%/%":
        if both_int and b != 0:
            return a // b
        return float(_r_intdiv(float(a), float(b)))
    if op == "min":
        return min(a, b) if both_int else float(min(a, b) if (a == a and b == b) else float("nan"))
    if op == "max":
        return max(a, b) if both_int else float(max(a, b) if (a == a and b == b) else float("nan"))
    if op == "log":
        return _log(float(a), float(b))
    if op == "bitwAnd":
        return int(a) & int(b)
    if op == "bitwOr":
        return int(a) | int(b)
    if op == "bitwXor":
        return int(a) ^ int(b)
    if op == "bitwShiftL":
        return int(a) << int(b)
    if op == "bitwShiftR":
        return int(a) >> int(b)
    raise DMLRuntimeError(f"unknown scalar binary operator {op}")


def _log(a, base=None):
    if a < 0 or a != a:
        return float("nan")
    if a == 0:
        return -INF
    if base is None:
        return math.log(a)
    return math.log(a) / math.log(base)


def _round_half_up(x):
    # Java Math.round semantics (round half up) -> SystemML 'round' uses Math.round
    if x != x or x in (INF, -INF):
        return x
    return float(math.floor(x + 0.5))


def unary(op: str, a):
    if op == "neg":
        if isinstance(a, str):
            raise DMLRuntimeError("cannot negate a string")
        return -_num(a)
    if op == "not":
        return not as_bool(a)
    if op == "ident":
        return a
    if op in ("cast_double",):
        return as_double(a)
    if op == "cast_int":
        return as_int(a)
    if op == "cast_bool":
        return as_bool(a)
    if op == "cast_scalar":
        return a
    x = float(_num(a))
    if op == "abs":
        v = abs(_num(a))
        return v
    if op == "exp":
        try:
            return math.exp(x)
        except OverflowError:
            return INF
    if op == "log":
        return _log(x)
    if op == "sqrt":
        return math.sqrt(x) if x >= 0 else float("nan")
    if op == "round":
        return _round_half_up(x)
    if op == "floor":
        return float(math.floor(x)) if math.isfinite(x) else x
    if op == "ceil":
        return float(math.ceil(x)) if math.isfinite(x) else x
    if op == "sign":
        return float((x > 0) - (x < 0)) if x == x else x
    fn = {"sin": math.sin, "cos": math.cos, "tan": math.tan, "asin": math.asin, "acos": math.acos,
          "atan": math.atan, "sinh": math.sinh, "cosh": math.cosh, "tanh": math.tanh,
          "sigmoid": lambda v: 1.0 / (1.0 + math.exp(-v)) if v > -700 else 0.0}.get(op)
    if fn is not None:
        try:
            return fn(x)
        except (ValueError, OverflowError):
            return float("nan") if op in ("asin", "acos") else (INF if x > 0 else -INF)
    raise DMLRuntimeError(f"unknown scalar unary operator {op}")


def parse_literal_arg(s: str):
    """Type a command-line argument value (reference: DMLScript argument typing)."""
    if isinstance(s, (bool, int, float)):
        return s
    t = s.strip()
    if t in ("TRUE", "true", "True"):
        return True
    if t in ("FALSE", "false", "False"):
        return False
    try:
        return int(t)
    except ValueError:
        pass
    try:
        return float(t)
    except ValueError:
        pass
    if len(t) >= 2 and t[0] == t[-1] and t[0] in "\"'":
        return t[1:-1]
    return s
