"""Exception hierarchy (reference: parser/ParseException.java, parser/LanguageException.java,
runtime/DMLRuntimeException.java, api/DMLException.java)."""


class DMLException(Exception):
    pass


class ParseError(DMLException):
    pass


class LanguageError(DMLException):
    pass


class DMLRuntimeError(DMLException):
    pass


class DMLScriptStop(DMLRuntimeError):
    """Raised by the DML `stop()` builtin."""
    pass
