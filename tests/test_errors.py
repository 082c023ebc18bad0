"""Typed errors + enforce helpers (reference: paddle/common/enforce.h, errors.h; FLAGS_call_stack_level)."""
import pytest

import paddle2_amd as paddle
from paddle2_amd.framework import errors as E


def test_typed_errors_are_python_exceptions_too():
    with pytest.raises(ValueError, match=r"\(InvalidArgument\)"):
        E.enforce(False, E.InvalidArgumentError, "bad")
    with pytest.raises(IndexError, match=r"\(OutOfRange\)"):
        E.enforce(False, "OutOfRange", "idx")
    with pytest.raises(NotImplementedError):
        E.raise_error("Unimplemented", "nope")
    with pytest.raises(E.EnforceNotMet):
        E.enforce_eq(1, 2, "mismatch")


def test_enforce_cmp_hint_and_stack_levels():
    paddle.set_flags({"FLAGS_call_stack_level": 1})
    with pytest.raises(ValueError) as ei:
        E.enforce_ge(3, 5, "too small")
    msg = str(ei.value)
    assert "Expected 3 >= 5" in msg and "[at " in msg and "test_errors.py" in msg
    paddle.set_flags({"FLAGS_call_stack_level": 0})
    with pytest.raises(ValueError) as ei:
        E.enforce_lt(9, 1, "x")
    assert "Hint" not in str(ei.value)
    paddle.set_flags({"FLAGS_call_stack_level": 2})
    with pytest.raises(ValueError) as ei:
        E.enforce_ne(1, 1)
    assert "Python call stack" in str(ei.value)
    paddle.set_flags({"FLAGS_call_stack_level": 1})


def test_reshape_reports_reference_style_errors():
    x = paddle.ones([2, 3])
    with pytest.raises(E.InvalidArgumentError, match="size is 6"):
        paddle.reshape(x, [4, 2])
    with pytest.raises(ValueError, match="Only one dimension"):
        paddle.reshape(x, [-1, -1])
    assert paddle.reshape(x, [0, -1]).shape == [2, 3]
