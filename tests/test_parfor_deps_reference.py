"""Parfor dependency analysis against the reference's own expectations: every case of
ParForDependencyAnalysisTest.java (script, expected "dependency detected") is run through
compiler/parfor_deps.py.  The reference marks parfor32c's detected dependency as a false
positive of its own analysis ("32c: dep (no, dep is false positive)"); the linear analysis
here proves it independent.  parfor48b is a validation error (matrix loop bound), raised by
the translator rather than the dependency analysis."""
import os
import re

import pytest

from systemml_amd.api.executor import compile_script
from systemml_amd.compiler.parfor_deps import check_program
from systemml_amd.parser.dml_parser import parse_dml
from systemml_amd.parser.errors import LanguageError

REF = "/root/reference/src/test"
JAVA = os.path.join(REF, "java/org/apache/sysml/test/integration/functions/parfor/ParForDependencyAnalysisTest.java")
SCRIPTS = os.path.join(REF, "scripts/functions/parfor")
KNOWN = {"parfor32c.dml": "reference false positive", "parfor48b.dml": "translator validation error"}


def _cases():
    if not os.path.exists(JAVA):
        return []
    src = open(JAVA).read()
    return re.findall(r'runTest\("(\w+\.dml)", (true|false)\)', src)


CASES = _cases()


@pytest.mark.skipif(not CASES, reason="reference test sources not mounted")
@pytest.mark.parametrize("script,expected", CASES)
def test_dependency_analysis_matches_reference(script, expected):
    path = os.path.join(SCRIPTS, script)
    src = open(path).read()
    try:
        check_program(parse_dml(src, path))
        got = "false"
    except LanguageError:
        got = "true"
    if script in KNOWN:
        assert got == "false"
        if script == "parfor48b.dml":
            with pytest.raises(LanguageError, match="must be a scalar"):
                compile_script(src)
        return
    assert got == expected, script


def test_parity_count():
    if not CASES:
        pytest.skip("reference test sources not mounted")
    assert len(CASES) >= 70


def test_scalar_accumulation_is_an_output_dependency():
    # the reference accumulates matrices only; a scalar `s += ...` in a parfor body
    # is an output dependency (ParForStatementBlock.rCheckCandidates)
    with pytest.raises(LanguageError):
        compile_script("s = 0\nparfor (i in 1:4) { s += i }\nprint(s)")
    compile_script("A = matrix(0, 2, 2)\nparfor (i in 1:4) { A += i }\nprint(sum(A))")
