"""paddle.incubate.nn.memory_efficient_attention with the attn_bias descriptors (reference
test/legacy_test/test_memory_efficient_attention.py): each bias kind against a dense fp32 softmax reference."""
import math

import numpy as np
import torch

import paddle2_amd as paddle
from paddle2_amd.incubate.nn import attn_bias as AB
from paddle2_amd.incubate.nn import memory_efficient_attention


def _ref(q, k, v, bias):
    qf, kf, vf = (torch.tensor(t).transpose(1, 2) for t in (q, k, v))
    s = qf @ kf.transpose(-1, -2) / math.sqrt(q.shape[-1]) + bias
    return (torch.softmax(s, -1) @ vf).transpose(1, 2).numpy()


def test_all_bias_kinds():
    rs = np.random.RandomState(0)
    q, k, v = (rs.randn(2, 6, 2, 8).astype("float32") for _ in range(3))
    T = paddle.to_tensor
    out = memory_efficient_attention(T(q), T(k), T(v))
    np.testing.assert_allclose(out.numpy(), _ref(q, k, v, 0.0), rtol=1e-4, atol=1e-5)
    causal = AB.LowerTriangularMask()
    out = memory_efficient_attention(T(q), T(k), T(v), causal)
    np.testing.assert_allclose(out.numpy(), _ref(q, k, v, causal.materialize((6, 6))), rtol=1e-4, atol=1e-5)
    tb = rs.randn(2, 2, 6, 6).astype("float32")
    out = memory_efficient_attention(T(q), T(k), T(v), T(tb))
    np.testing.assert_allclose(out.numpy(), _ref(q, k, v, torch.tensor(tb)), rtol=1e-4, atol=1e-5)
    cb = causal.add_bias(T(tb))
    out = memory_efficient_attention(T(q), T(k), T(v), cb)
    np.testing.assert_allclose(out.numpy(), _ref(q, k, v, cb.materialize((2, 2, 6, 6))), rtol=1e-4, atol=1e-5)
    # packed sequences of lengths 2 and 4 in one [1, 6, H, D] batch, causal within each
    qp, kp, vp = q[:1], k[:1], v[:1]
    bd = AB.BlockDiagonalMask.from_seqlens([2, 4]).make_causal()
    out = memory_efficient_attention(T(qp), T(kp), T(vp), bd)
    np.testing.assert_allclose(out.numpy(), _ref(qp, kp, vp, bd.materialize((6, 6))), rtol=1e-4, atol=1e-5)
    # the op-table entry takes the ops.yaml signature
    o, _, _ = paddle._C_ops.memory_efficient_attention(T(q), T(k), T(v), None, None, None, None, None, -1, -1, True)
    np.testing.assert_allclose(o.numpy(), _ref(q, k, v, causal.materialize((6, 6))), rtol=1e-4, atol=1e-5)
