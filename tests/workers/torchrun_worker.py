"""Rank worker started by torch.distributed.run: init_parallel_env on the elastic agent's store + one all_reduce."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed import collective  # noqa: E402

dist.init_parallel_env()
r = dist.get_rank()
t = paddle.to_tensor([float(r + 1)] * 2)
dist.all_reduce(t)
with open(os.path.join(os.environ["PD_TEST_OUT_DIR"], f"rank{r}.json"), "w") as f:
    json.dump({"all_reduce": t.numpy().tolist(), "store": collective.pg_status().get("store")}, f)
dist.barrier()
