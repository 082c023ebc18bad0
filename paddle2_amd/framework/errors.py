"""Typed framework errors and enforce helpers (reference: paddle/common/errors.h error codes,
paddle/common/enforce.h PADDLE_ENFORCE_* and the ``FLAGS_call_stack_level`` message policy).

Each error type keeps the reference's code name in its message prefix — ``(InvalidArgument) ...`` — and
subclasses the Python exception a caller would naturally catch (ValueError for bad arguments, IndexError for
out-of-range, NotImplementedError for unimplemented, ...), so ``except ValueError`` code keeps working.

Message policy by ``FLAGS_call_stack_level``: 0 = the error summary only; 1 (default) = summary + hint +
the innermost framework-external Python frame that raised it; 2 = summary + the full Python stack.
"""
from __future__ import annotations

import traceback


class EnforceNotMet(Exception):
    """Base of the typed errors (the reference's EnforceNotMet)."""

    code = "Fatal"


def _mk(name, code, base):
    cls = type(name, (EnforceNotMet, base), {"code": code})
    cls.__doc__ = f"({code}) error; also a {base.__name__}."
    return cls


InvalidArgumentError = _mk("InvalidArgumentError", "InvalidArgument", ValueError)
NotFoundError = _mk("NotFoundError", "NotFound", LookupError)
OutOfRangeError = _mk("OutOfRangeError", "OutOfRange", IndexError)
AlreadyExistsError = _mk("AlreadyExistsError", "AlreadyExists", RuntimeError)
ResourceExhaustedError = _mk("ResourceExhaustedError", "ResourceExhausted", MemoryError)
PreconditionNotMetError = _mk("PreconditionNotMetError", "PreconditionNotMet", RuntimeError)
PermissionDeniedError = _mk("PermissionDeniedError", "PermissionDenied", PermissionError)
ExecutionTimeoutError = _mk("ExecutionTimeoutError", "ExecutionTimeout", TimeoutError)
UnimplementedError = _mk("UnimplementedError", "Unimplemented", NotImplementedError)
UnavailableError = _mk("UnavailableError", "Unavailable", RuntimeError)
FatalError = _mk("FatalError", "Fatal", RuntimeError)
ExternalError = _mk("ExternalError", "External", RuntimeError)

_BY_CODE = {c.code: c for c in (InvalidArgumentError, NotFoundError, OutOfRangeError, AlreadyExistsError,
                                ResourceExhaustedError, PreconditionNotMetError, PermissionDeniedError,
                                ExecutionTimeoutError, UnimplementedError, UnavailableError, FatalError,
                                ExternalError)}


def _level():
    from . import flags

    return int(flags.flag("FLAGS_call_stack_level", 1))


def format_error(code, msg, hint=None, stack=None):
    lvl = _level()
    text = f"({code}) {msg}"
    if lvl >= 1 and hint:
        text += f"\n  [Hint: {hint}]"
    if stack is None:  # drop this module's own frames
        stack = [f for f in traceback.extract_stack()[:-1] if f.filename != __file__]
    if lvl == 1:
        user = [f for f in stack if "paddle2_amd" not in f.filename]
        if user:
            f = user[-1]
            text += f"\n  [at {f.filename}:{f.lineno} in {f.name}]"
    elif lvl >= 2:
        text += "\n  Python call stack:\n" + "".join("    " + ln for ln in traceback.format_list(stack))
    return text


def raise_error(code, msg, hint=None):
    raise _BY_CODE[code](format_error(code, msg, hint))


def enforce(cond, error=InvalidArgumentError, msg="", hint=None):
    """PADDLE_ENFORCE: raise ``error`` (a typed class or a code name) with the formatted message if not cond."""
    if not cond:
        cls = _BY_CODE[error] if isinstance(error, str) else error
        raise cls(format_error(cls.code, msg, hint))


def _cmp(op, sym):
    def check(a, b, msg="", error=InvalidArgumentError):
        if not op(a, b):
            cls = _BY_CODE[error] if isinstance(error, str) else error
            raise cls(format_error(cls.code, msg or "enforce failed", f"Expected {a!r} {sym} {b!r}, but received "
                                                                        f"{a!r} vs {b!r}."))
    check.__name__ = "enforce_" + {"==": "eq", "!=": "ne", ">": "gt", ">=": "ge", "<": "lt", "<=": "le"}[sym]
    return check


enforce_eq = _cmp(lambda a, b: a == b, "==")
enforce_ne = _cmp(lambda a, b: a != b, "!=")
enforce_gt = _cmp(lambda a, b: a > b, ">")
enforce_ge = _cmp(lambda a, b: a >= b, ">=")
enforce_lt = _cmp(lambda a, b: a < b, "<")
enforce_le = _cmp(lambda a, b: a <= b, "<=")


def enforce_not_null(x, name="value", error=NotFoundError):
    if x is None:
        cls = _BY_CODE[error] if isinstance(error, str) else error
        raise cls(format_error(cls.code, f"{name} should not be null"))
    return x
