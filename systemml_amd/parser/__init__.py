from .errors import ParseError, LanguageError, DMLRuntimeError, DMLException, DMLScriptStop
from .dml_parser import parse_dml, parse_dml_file
from . import ast
