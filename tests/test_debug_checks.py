"""Debugging subsystems: NaN/Inf checker (FLAGS_check_nan_inf) and collective static/dynamic checks."""
import pytest
import torch

import paddle2_amd as paddle
from _dist import run_workers


class _Bad(paddle.nn.Layer):
    def forward(self, x):
        return x / 0.0


def test_nan_inf_checker_raises_and_logs():
    paddle.set_device("cpu")
    from paddle2_amd.framework import nan_inf

    net = paddle.nn.Sequential(paddle.nn.Linear(4, 4), _Bad())
    x = paddle.ones([2, 4])
    net(x)  # off by default: no error
    paddle.set_flags({"FLAGS_check_nan_inf": True, "FLAGS_check_nan_inf_level": 0})
    try:
        with pytest.raises(RuntimeError, match="check_nan_inf.*_Bad|check_nan_inf"):
            net(x)
        paddle.set_flags({"FLAGS_check_nan_inf_level": 1})
        n0 = len(nan_inf.records())
        net(x)
        assert len(nan_inf.records()) > n0
        # backward scan: finite forward, NaN gradient injected downstream
        paddle.set_flags({"FLAGS_check_nan_inf_level": 0})
        lin = paddle.nn.Linear(4, 4)
        y = lin(x)
        with pytest.raises(RuntimeError, match="backward|op aten.mul"):  # per-op scan catches the forward mul
            (y._t * torch.tensor(float("nan"))).sum().backward()
    finally:
        paddle.set_flags({"FLAGS_check_nan_inf": False, "FLAGS_check_nan_inf_level": 0})
    assert not nan_inf.enabled


def test_comm_dynamic_and_static_checks():
    res = run_workers("commcheck_worker.py", 2)
    for r in res:
        assert r["ok"] == [2.0, 4.0, 6.0]
        assert r["caught"] is True
        assert r["static"] is True


def test_conv_exhaustive_search_flag_drives_miopen_find():
    """FLAGS_cudnn_exhaustive_search (reference: conv algorithm search) switches MIOpen Find on through
    torch.backends.cudnn.benchmark; FLAGS_cudnn_deterministic keeps it off while set."""
    import torch

    import paddle2_amd as paddle

    old = paddle.get_flags(["FLAGS_cudnn_exhaustive_search", "FLAGS_cudnn_deterministic"])
    try:
        paddle.set_flags({"FLAGS_cudnn_exhaustive_search": True})
        assert torch.backends.cudnn.benchmark
        paddle.set_flags({"FLAGS_cudnn_deterministic": True})
        assert not torch.backends.cudnn.benchmark
        paddle.set_flags({"FLAGS_cudnn_deterministic": False})
        assert torch.backends.cudnn.benchmark
        paddle.set_flags({"FLAGS_cudnn_exhaustive_search": False})
        assert not torch.backends.cudnn.benchmark
    finally:
        paddle.set_flags(old)
