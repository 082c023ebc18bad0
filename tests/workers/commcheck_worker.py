"""Rank worker: FLAGS_enable_nccl_dynamic_check catches a cross-rank shape mismatch before the collective."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed.comm_check import CommCheckError  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
r = dist.get_rank()
paddle.set_flags({"FLAGS_enable_nccl_dynamic_check": True})
out = {}
t = paddle.to_tensor([1.0, 2.0, 3.0])
dist.all_reduce(t)                      # consistent: passes
out["ok"] = t.numpy().tolist()
bad = paddle.to_tensor([1.0] * (3 + r))  # rank 1 has a different shape
try:
    dist.all_reduce(bad)
    out["caught"] = False
except CommCheckError as e:
    out["caught"] = "shape" in str(e)
try:
    dist.all_gather_into_tensor(paddle.zeros([5]), paddle.ones([2]))
    out["static"] = False
except CommCheckError:
    out["static"] = True
write_result(out)
dist.destroy_process_group()
