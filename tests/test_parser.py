"""Parser tests (reference test strategy: functions/misc parser tests, every bundled script parses)."""
import glob
import os

import pytest

from systemml_amd.parser import parse_dml, ParseError
from systemml_amd.parser import ast as A

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bin(e):
    return (e.op, _bin(e.left), _bin(e.right)) if isinstance(e, A.BinOp) else \
        (("u" + e.op), _bin(e.operand)) if isinstance(e, A.UnOp) else \
        (e.value if isinstance(e, A.Literal) else e.name)


def expr(src):
    p = parse_dml("x = " + src)
    return _bin(p.statements[0].value)


def test_precedence():
    assert expr("1 + 2 * 3") == ("+", 1, ("*", 2, 3))
    assert expr("a %*% b + c") == ("+", ("%*%", "a", "b"), "c")
    assert expr("2 ^ 3 ^ 2") == ("^", 2, ("^", 3, 2))
    assert expr("-a ^ 2") == ("u-", ("^", "a", 2))
    assert expr("-a %*% b") == ("%*%", ("u-", "a"), "b")
    assert expr("a < b & c | d") == ("|", ("&", ("<", "a", "b"), "c"), "d")
    assert expr("!a & b") == ("&", ("u!", "a"), "b")
    assert expr("!a == b") == ("u!", ("==", "a", "b"))
    assert expr("a %/% b * c") == ("*", ("%/%", "a", "b"), "c")
    assert expr("a - b - c") == ("-", ("-", "a", "b"), "c")


def test_statements():
    src = """
    source("nn/layers/affine.dml") as affine
    f = function(matrix[double] X, int k = 3) return (matrix[double] Y, double s) {
      Y = X * k; s = sum(Y)
    }
    [A, s] = f(X=matrix(1, rows=2, cols=2))
    X[1:2, ] = A
    x += 1
    if (s > 2) print("big") else { print("small") }
    for (i in 1:10) { x = x + i }
    parfor (i in seq(1, 10, 2), check=0) { y = i }
    while (FALSE) { z = 1 }
    v = ifdef($v, 5)
    """
    p = parse_dml(src)
    kinds = [type(s).__name__ for s in p.statements]
    assert kinds == ["Import", "MultiAssign", "Assign", "Assign", "If", "For", "For", "While", "Assign"]
    assert "f" in p.functions
    f = p.functions["f"]
    assert [x.name for x in f.inputs] == ["X", "k"] and f.inputs[1].default is not None
    assert p.statements[6].parfor and "check" in p.statements[6].params


def test_indexing_forms():
    p = parse_dml("a = X[1, ]; b = X[, 2]; c = X[1:3, 2:4]; d = L[2]; e = X[i]")
    st = p.statements
    assert st[0].value.cols is not None and st[0].value.cols.lower is None
    assert st[2].value.rows.is_range and st[2].value.cols.is_range
    assert st[3].value.cols is None


def test_comments_and_strings():
    p = parse_dml("/* block \n comment */ x = 'its' # c\n y = \"a\\tb\"")
    assert p.statements[1].value.value == "a\tb"


def test_errors():
    with pytest.raises(ParseError):
        parse_dml("x = (1 + ")
    with pytest.raises(ParseError):
        parse_dml("x = 'unterminated")


def test_bundled_scripts_parse():
    files = glob.glob(os.path.join(HERE, "systemml_amd", "scripts", "**", "*.dml"), recursive=True)
    assert files
    for f in files:
        with open(f) as fh:
            parse_dml(fh.read(), filename=f)


@pytest.mark.skipif(not os.path.isdir("/root/reference/scripts"), reason="reference not mounted")
def test_reference_scripts_parse():
    files = glob.glob("/root/reference/scripts/algorithms/*.dml") + \
        glob.glob("/root/reference/scripts/nn/**/*.dml", recursive=True)
    for f in files:
        with open(f) as fh:
            parse_dml(fh.read(), filename=f)
