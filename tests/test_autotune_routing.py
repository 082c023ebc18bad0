"""Measured native-MFMA vs hipBLASLt routing of the Linear GEMMs (incubate/autotune.py route): decisions are
timed once per (pass, shape), cached to JSON, reused, and either route gives the same numerics."""
import json

import pytest
import torch

from paddle2_amd.incubate import autotune
from paddle2_amd.ops import torch_ops as T

pytestmark = pytest.mark.gpu


def test_routing_autotune_decides_and_caches(tmp_path):
    f = tmp_path / "routing.json"
    autotune.enable_routing_autotune(str(f), iters=2)
    try:
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(2048, 1024, generator=g, device="cuda").to(torch.bfloat16).requires_grad_()
        w = (torch.randn(1024, 3072, generator=g, device="cuda") * 0.02).to(torch.bfloat16).requires_grad_()
        y = T.linear(x, w)
        y.backward(torch.ones_like(y))
        table = json.loads(f.read_text())
        assert any(k.startswith("fwd:2048x3072x1024") for k in table)
        assert any(k.startswith("dgrad:") for k in table) and any(k.startswith("wgrad") for k in table)
        assert set(table.values()) <= {"native", "blas"}
        ref = x.detach().float() @ w.detach().float()
        assert (y.float() - ref).abs().max() / ref.abs().max() < 1e-2
        n = len(table)
        T.linear(x, w).sum().backward()  # cached: no new entries
        assert len(autotune.routing_table()) == n
    finally:
        autotune.disable_routing_autotune()
