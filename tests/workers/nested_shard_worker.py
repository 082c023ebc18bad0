"""Rank worker (4 ranks, 2x2 mesh): one tensor axis sharded over BOTH mesh dims ([Shard(0), Shard(0)]) reshards
back to replicated in the original row order (gathered inner mesh dim first)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
mesh = dist.ProcessMesh([[0, 1], [2, 3]], dim_names=["x", "y"])
g = np.arange(48, dtype="float32").reshape(8, 6)
AP = paddle.distributed.auto_parallel
a = dist.shard_tensor(paddle.to_tensor(g), mesh, [dist.Shard(0), dist.Shard(0)])
out = {"local": AP.local_tensor(a).numpy().tolist()}
r = dist.reshard(a, mesh, [dist.Replicate(), dist.Replicate()])
out["full"] = AP.local_tensor(r).numpy().tolist()
s = dist.reshard(r, mesh, [dist.Shard(0), dist.Shard(0)])
out["again"] = AP.local_tensor(s).numpy().tolist()
write_result(out)
