"""Tokenizer shared by the DML and PyDML front ends.

Token classes follow the lexer rules of the reference grammars
(reference: src/main/java/org/apache/sysml/parser/dml/Dml.g4:196-219 and
parser/pydml/Pydml.g4): INT (optional L suffix), DOUBLE (with exponent),
single/double quoted STRING with escapes, $named / $positional command-line
ids, `ns::name` namespaced ids, and the R-style operators `%*%`, `%/%`,
`%%`, `<-`.  PyDML mode additionally emits NEWLINE / INDENT / DEDENT tokens.
"""
from __future__ import annotations

import re
from dataclasses import dataclass

from .errors import ParseError


@dataclass
class Token:
    kind: str     # 'ID','INT','DOUBLE','STRING','CMD','OP','EOF','NEWLINE','INDENT','DEDENT'
    value: object
    line: int
    col: int

    def __repr__(self):
        return f"Token({self.kind},{self.value!r}@{self.line}:{self.col})"


_DML_OPS = [
    "%*%", "%/%", "%%", "<-", "<=", ">=", "==", "!=", "&&", "||", "+=", "::",
    "^", "*", "/", "+", "-", "<", ">", "!", "&", "|", "=", "(", ")", "[", "]",
    "{", "}", ",", ";", ":",
]
_PYDML_OPS = [
    "**", "//", "<=", ">=", "==", "!=", "+=", "->", "::",
    "^", "*", "/", "%", "+", "-", "<", ">", "!", "&", "|", "=", "(", ")", "[", "]",
    "{", "}", ",", ";", ":", "@",
]

_ESC = {"b": "\b", "t": "\t", "n": "\n", "f": "\f", "r": "\r", '"': '"', "'": "'", "\\": "\\"}


def _is_id_start(c):
    return c.isalpha() or c == "_"


def _is_id_char(c):
    return c.isalnum() or c == "_" or c == "."


_NUM = r"(?:\d+\.(?!\.)\d*|\.\d+|\d+)(?:[eE][+-]?\d+)?"
_DML_RE = re.compile(
    r"(?P<ws>[ \t\r]+)|(?P<nl>\n)|(?P<com>#[^\n]*)|(?P<bcom>/\*)|"
    r"(?P<num>" + _NUM + r")(?P<lsuf>[lL])?|"
    r"(?P<id>[^\W\d][\w.]*(?:::[^\W\d][\w.]*)?)|"
    r"(?P<cmd>\$\w*)|(?P<str>[\"'])|"
    r"(?P<op>" + "|".join(re.escape(o) for o in _DML_OPS) + r")")


def _tokenize_dml(src: str, filename: str):
    """DML tokens via one compiled master regex (same rules as the character loop below,
    which is kept for PyDML's indentation handling); ~10x faster on the algorithm scripts."""
    toks = []
    append = toks.append
    i, n = 0, len(src)
    line, col0 = 1, 0
    match = _DML_RE.match

    def err(msg):
        raise ParseError(f"{filename or '<script>'} line {line}: {msg}")

    while i < n:
        m = match(src, i)
        if m is None:
            err(f"unexpected character {src[i]!r}")
        kind = m.lastgroup
        if kind == "lsuf":
            kind = "num"
        j = m.end()
        if kind == "ws" or kind == "com":
            i = j
            continue
        if kind == "nl":
            line += 1
            i = j
            col0 = i
            continue
        col = i - col0
        if kind == "id":
            word = m.group("id")
            if "::" not in word:
                while word.endswith("."):
                    word = word[:-1]
                    j -= 1
            append(Token("ID", word, line, col))
        elif kind == "num":
            text = m.group("num")
            if "." in text or "e" in text or "E" in text:
                append(Token("DOUBLE", float(text), line, col))
            else:
                append(Token("INT", int(text), line, col))
        elif kind == "op":
            append(Token("OP", m.group("op"), line, col))
        elif kind == "cmd":
            if j == i + 1:
                err("invalid command-line parameter")
            append(Token("CMD", src[i + 1:j], line, col))
        elif kind == "bcom":
            k = src.find("*/", i + 2)
            if k < 0:
                err("unterminated block comment")
            nl = src.count("\n", i, k + 2)
            if nl:
                line += nl
                col0 = src.rfind("\n", i, k + 2) + 1
            j = k + 2
        else:   # string literal
            c = src[i]
            j = i + 1
            buf = []
            while j < n and src[j] != c:
                if src[j] == "\\" and j + 1 < n:
                    e = src[j + 1]
                    buf.append(_ESC.get(e, "\\" + e))
                    j += 2
                    continue
                if src[j] == "\n":
                    line += 1
                    col0 = j + 1
                buf.append(src[j])
                j += 1
            if j >= n:
                err("unterminated string literal")
            append(Token("STRING", "".join(buf), line, col))
            j += 1
        i = j
    append(Token("EOF", None, line, 0))
    return toks


def tokenize(src: str, pydml: bool = False, filename: str = ""):
    if not pydml:
        return _tokenize_dml(src, filename)
    ops = _PYDML_OPS if pydml else _DML_OPS
    toks = []
    i, n = 0, len(src)
    line, col0 = 1, 0
    # PyDML indentation tracking
    indent_stack = [0]
    paren_depth = 0
    at_line_start = True

    def err(msg):
        raise ParseError(f"{filename or '<script>'} line {line}: {msg}")

    while i < n:
        c = src[i]
        if pydml and at_line_start and paren_depth > 0:
            at_line_start = False      # implicit line joining inside brackets
        if pydml and at_line_start and paren_depth == 0:
            # measure indentation of logical line
            j = i
            width = 0
            while j < n and src[j] in " \t":
                width += 4 if src[j] == "\t" else 1
                j += 1
            if j < n and src[j] in "\r\n#":
                # blank / comment-only line: skip indentation handling
                i = j
                at_line_start = False
                continue
            if j >= n:
                i = j
                break
            if width > indent_stack[-1]:
                indent_stack.append(width)
                toks.append(Token("INDENT", width, line, 0))
            else:
                while width < indent_stack[-1]:
                    indent_stack.pop()
                    toks.append(Token("DEDENT", width, line, 0))
                if width != indent_stack[-1]:
                    err("inconsistent indentation")
            i = j
            at_line_start = False
            continue
        if c == "\n":
            if pydml and paren_depth == 0 and toks and toks[-1].kind not in ("NEWLINE", "INDENT", "DEDENT"):
                toks.append(Token("NEWLINE", None, line, i - col0))
            line += 1
            i += 1
            col0 = i
            at_line_start = True
            continue
        if c in " \t\r":
            i += 1
            continue
        if c == "\\" and pydml and i + 1 < n and src[i + 1] == "\n":  # line continuation
            i += 2
            line += 1
            col0 = i
            continue
        if c == "#":
            j = src.find("\n", i)
            i = n if j < 0 else j
            continue
        if c == "/" and i + 1 < n and src[i + 1] == "*":
            j = src.find("*/", i + 2)
            if j < 0:
                err("unterminated block comment")
            line += src.count("\n", i, j + 2)
            if src.count("\n", i, j + 2):
                col0 = src.rfind("\n", i, j + 2) + 1
            i = j + 2
            continue
        if pydml and c in "\"'" and src.startswith(c * 3, i):
            # triple quoted string (docstrings in PyDML) -> treated as comment-like string
            q = c * 3
            j = src.find(q, i + 3)
            if j < 0:
                err("unterminated triple-quoted string")
            s = src[i + 3:j]
            toks.append(Token("STRING", s, line, i - col0))
            line += src.count("\n", i, j + 3)
            if src.count("\n", i, j + 3):
                col0 = src.rfind("\n", i, j + 3) + 1
            i = j + 3
            continue
        col = i - col0
        # numbers
        if c.isdigit() or (c == "." and i + 1 < n and src[i + 1].isdigit()):
            j = i
            while j < n and src[j].isdigit():
                j += 1
            is_double = False
            if j < n and src[j] == "." and not (j + 1 < n and src[j + 1] == "."):
                # avoid treating '1.' followed by identifier char weirdly
                is_double = True
                j += 1
                while j < n and src[j].isdigit():
                    j += 1
            if j < n and src[j] in "eE":
                k = j + 1
                if k < n and src[k] in "+-":
                    k += 1
                if k < n and src[k].isdigit():
                    is_double = True
                    j = k
                    while j < n and src[j].isdigit():
                        j += 1
            text = src[i:j]
            if j < n and src[j] in "lL":
                j += 1
            if is_double:
                toks.append(Token("DOUBLE", float(text), line, col))
            else:
                toks.append(Token("INT", int(text), line, col))
            i = j
            continue
        if _is_id_start(c):
            j = i
            while j < n and _is_id_char(src[j]):
                j += 1
            # namespace separator ns::name
            if src.startswith("::", j) and j + 2 < n and _is_id_start(src[j + 2]):
                k = j + 2
                while k < n and _is_id_char(src[k]):
                    k += 1
                toks.append(Token("ID", src[i:k], line, col))
                i = k
                continue
            word = src[i:j]
            # strip trailing dots (e.g. "x." is not an id)
            while word.endswith("."):
                word = word[:-1]
                j -= 1
            toks.append(Token("ID", word, line, col))
            i = j
            continue
        if c == "$":
            j = i + 1
            while j < n and (src[j].isalnum() or src[j] == "_"):
                j += 1
            if j == i + 1:
                err("invalid command-line parameter")
            toks.append(Token("CMD", src[i + 1:j], line, col))
            i = j
            continue
        if c in "\"'":
            j = i + 1
            buf = []
            while j < n and src[j] != c:
                if src[j] == "\\" and j + 1 < n:
                    e = src[j + 1]
                    buf.append(_ESC.get(e, "\\" + e))
                    j += 2
                    continue
                if src[j] == "\n":
                    line += 1
                    col0 = j + 1
                buf.append(src[j])
                j += 1
            if j >= n:
                err("unterminated string literal")
            toks.append(Token("STRING", "".join(buf), line, col))
            i = j + 1
            continue
        for op in ops:
            if src.startswith(op, i):
                toks.append(Token("OP", op, line, col))
                if op in "([{":
                    paren_depth += 1
                elif op in ")]}":
                    paren_depth = max(0, paren_depth - 1)
                i += len(op)
                break
        else:
            err(f"unexpected character {c!r}")
    if pydml:
        if toks and toks[-1].kind not in ("NEWLINE", "INDENT", "DEDENT"):
            toks.append(Token("NEWLINE", None, line, 0))
        while len(indent_stack) > 1:
            indent_stack.pop()
            toks.append(Token("DEDENT", 0, line, 0))
    toks.append(Token("EOF", None, line, 0))
    return toks
