"""Per-op NaN/Inf checking (framework/nan_inf.py dispatch mode): the offending ATen op is named, for forward
and backward kernels (reference: paddle/fluid/eager/nan_inf_utils.cc CheckTensorHasNanOrInf per op)."""
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.framework import nan_inf


@pytest.fixture
def checker():
    paddle.set_flags({"FLAGS_check_nan_inf": True, "FLAGS_check_nan_inf_level": 0})
    yield
    paddle.set_flags({"FLAGS_check_nan_inf": False})
    assert nan_inf._mode[0] is None


def test_forward_op_named(checker):
    x = paddle.to_tensor([1.0, -1.0])
    with pytest.raises(RuntimeError, match=r"op aten\.log"):
        paddle.log(x)


def test_backward_op_named(checker):
    x = paddle.to_tensor([0.0, 4.0], stop_gradient=False)
    y = paddle.sqrt(x).sum()          # finite forward
    with pytest.raises(RuntimeError, match=r"backward op aten\.\w+"):
        y.backward()                  # d sqrt(x)/dx at 0 = inf, produced inside the backward kernels


def test_level1_logs_and_continues():
    paddle.set_flags({"FLAGS_check_nan_inf": True, "FLAGS_check_nan_inf_level": 1})
    try:
        n0 = len(nan_inf.records())
        out = paddle.to_tensor([0.0]) / paddle.to_tensor([0.0])
        assert torch.isnan(out._t).all()
        assert len(nan_inf.records()) > n0
    finally:
        paddle.set_flags({"FLAGS_check_nan_inf": False, "FLAGS_check_nan_inf_level": 0})


def test_off_by_default_costs_nothing():
    assert nan_inf._mode[0] is None
    paddle.log(paddle.to_tensor([-1.0]))  # no raise
