"""Rank worker: p_send_array / p_recv_array (static pipeline tensor-array p2p) over gloo."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.ops import extra_ops as E  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
r = dist.get_rank()
res = {}
if r == 0:
    E.p_send_array([paddle.to_tensor(torch.arange(6.0).reshape(2, 3)), paddle.to_tensor(torch.ones(2, 3))], peer=1)
    E.p_send_array([paddle.to_tensor(torch.arange(4.0)), paddle.to_tensor(torch.full((2, 2, 2), 3.0))], peer=1,
                   dynamic_shape=True)
else:
    a = E.p_recv_array(peer=0, dtype="float32", out_shape=[2, 3])
    b = E.p_recv_array(peer=0, dtype="float32", dynamic_shape=True)
    res = {"a": [t.numpy().tolist() for t in a], "b_shapes": [list(t.shape) for t in b],
           "b_sum": [float(t.numpy().sum()) for t in b]}
write_result(res)
