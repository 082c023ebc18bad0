"""Rank worker (4 ranks): cross-mesh reshard between mesh A = [0, 1] and mesh B = [2, 3] and back."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed.auto_parallel.reshard import COMM_LOG  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
rank = dist.get_rank()
A = dist.ProcessMesh([0, 1], dim_names=["x"])
B = dist.ProcessMesh([2, 3], dim_names=["x"])
A._device_mesh()
B._device_mesh()
g = np.arange(24, dtype="float32").reshape(4, 6)
AP = paddle.distributed.auto_parallel
out = {}


def local(t):
    return AP.local_tensor(t).numpy().tolist()


a = dist.shard_tensor(paddle.to_tensor(g), A, [dist.Shard(0)])   # every rank holds the DistTensor object
COMM_LOG.clear()
b = dist.reshard(a, B, [dist.Shard(0)])          # same status: coordinate k of A -> coordinate k of B (p2p)
out["same_status"] = {"local": local(b), "comm": [k for k, _ in COMM_LOG]}
COMM_LOG.clear()
c = dist.reshard(a, B, [dist.Shard(1)])          # general: replicate on A, send, slice on B
out["general"] = {"local": local(c), "comm": [k for k, _ in COMM_LOG]}
back = dist.reshard(c, A, [dist.Replicate()])    # and back, replicated on A
out["back"] = local(back)
write_result(out)
