"""FusedCommBuffer (all-reduce / reduce-scatter buckets) and fleet.collective_perf on gloo ranks."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
from _dist import write_result  # noqa: E402
from paddle2_amd.distributed import fleet  # noqa: E402
from paddle2_amd.distributed.fleet.utils.tensor_fusion_helper import (HOOK_ACTION, FusedCommBuffer,  # noqa: E402
                                                                       assign_group_by_size)

strategy = fleet.DistributedStrategy()
strategy.hybrid_configs = {"dp_degree": 2, "mp_degree": 1, "pp_degree": 1}
fleet.init(is_collective=True, strategy=strategy)
rank = paddle.distributed.get_rank()
res = {}

paddle.seed(0)
lin = paddle.nn.Linear(8, 6)
params = list(lin.parameters())
groups = assign_group_by_size(params, group_size=1 << 20)
res["groups"] = [len(v) for v in groups.values()]
grads = {}
for act, name in ((HOOK_ACTION.ALL_REDUCE, "ar"), (HOOK_ACTION.REDUCE_SCATTER, "rs")):
    buf = FusedCommBuffer(0, params, None, acc_steps=2, act=act)
    for step in range(2):  # gradient accumulation: two backward passes before communication
        x = paddle.to_tensor(torch.full((3, 8), float(rank + 1 + step)))
        lin(x).sum().backward()
        for p in params:
            buf.add_grad(p)
            p._t.grad = None
    buf.scale_grads()
    grads[name] = [buf._slot(i).reshape(-1)[:4].tolist() for i in range(len(params))]
    if act == HOOK_ACTION.REDUCE_SCATTER:
        n = buf._numel // 2
        grads["rs_shard_rank"] = rank
        grads["rs_shard_head"] = buf.grad_storage[rank * n: rank * n + 2].tolist()
res["grads"] = grads
perf = fleet.collective_perf("allreduce", round=3, size_and_time={1 << 16: None, 1 << 18: 100.0})
res["perf"] = [(r["bytes"], r["nranks"], r["time_ms"] > 0, r["busbw_GBs"] > 0) for r in perf]
write_result(res)
# leave together: a rank exiting while its peer's gloo threads still talk to it can abort the peer
import torch.distributed as _tdist  # noqa: E402

_tdist.barrier()
_tdist.destroy_process_group()
