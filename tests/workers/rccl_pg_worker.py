"""One-rank RCCL worker: the ProcessGroup surface on the nccl (RCCL) backend with GPU tensors."""
import json
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402

# a one-rank world still builds a real RCCL communicator when created explicitly (init_parallel_env skips
# torch.distributed for world size 1)
torch.cuda.set_device(0)
torch.distributed.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
dist.init_parallel_env()
pg = dist.new_group([0]).process_group
out = {"backend": type(pg).__name__}
x = paddle.to_tensor([1.0, 2.0, 3.0, 4.0])
pg.all_reduce_on_calc_stream(x)
y = paddle.to_tensor([2.0, 4.0])
pg.all_reduce(y, dist.ReduceOp.AVG, sync_op=False).wait()
rs = paddle.zeros([4])
pg.reduce_scatter_tensor_on_calc_stream(rs, paddle.to_tensor([1.0, 2.0, 3.0, 4.0]))
ag = paddle.zeros([3])
pg.all_gather_into_tensor(ag, paddle.to_tensor([5.0, 6.0, 7.0]))
a2a = []
pg.all_to_all_on_calc_stream(a2a, [paddle.to_tensor([9.0])])
pg.broadcast_on_calc_stream(x, 0)
pg.barrier()
torch.cuda.synchronize()
out.update(x=x.numpy().tolist(), y=y.numpy().tolist(), rs=rs.numpy().tolist(), ag=ag.numpy().tolist(),
           a2a=[float(t.numpy()[0]) for t in a2a], device=str(x._t.device))
with open(os.environ["PD_TEST_OUT"], "w") as f:
    json.dump(out, f)
dist.destroy_process_group()
