"""Rank worker: the reference ProcessGroup method surface (group.process_group.*) over gloo."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
r, w = dist.get_rank(), dist.get_world_size()
pg = dist.new_group(list(range(w))).process_group
res = {"name": pg.name(), "rank": pg.rank(), "size": pg.size()}

x = paddle.to_tensor([float(r + 1)] * 4)
pg.all_reduce(x).wait()
res["all_reduce"] = x.numpy().tolist()
y = paddle.to_tensor([float(r + 1)] * 2)
t = pg.all_reduce(y, dist.ReduceOp.AVG, sync_op=False)
t.wait()
res["avg"] = y.numpy().tolist()
res["task"] = [t.is_completed(), t.is_sync()]
z = paddle.to_tensor([float(r)] * 3)
pg.broadcast_on_calc_stream(z, src=w - 1)
res["bcast"] = z.numpy().tolist()
outs = []
pg.all_gather(outs, paddle.to_tensor([float(r)]))
res["gather_list"] = [float(o.numpy()[0]) for o in outs]
cat = paddle.zeros([w * 2])
pg.all_gather_into_tensor_on_calc_stream(cat, paddle.to_tensor([float(r), float(r) + 0.5]))
res["gather_tensor"] = cat.numpy().tolist()
part = paddle.zeros([w])
src = paddle.to_tensor([float(10 * r + i) for i in range(w)])
pg.all_gather_partial_on_calc_stream(part, src, w, r)
res["gather_partial"] = part.numpy().tolist()
rs_out = paddle.zeros([2])
pg.reduce_scatter_tensor_on_calc_stream(rs_out, paddle.to_tensor([float(i) for i in range(2 * w)]))
res["reduce_scatter"] = rs_out.numpy().tolist()
a2a_in = [paddle.to_tensor([float(100 * r + j)]) for j in range(w)]
a2a_out = []
pg.all_to_all_on_calc_stream(a2a_out, a2a_in)
res["all_to_all"] = [float(o.numpy()[0]) for o in a2a_out]
sc = paddle.zeros([1])
pg.scatter_on_calc_stream(sc, [paddle.to_tensor([float(7 * j)]) for j in range(w)], src=0)
res["scatter"] = float(sc.numpy()[0])
g = []
pg.gather(g, paddle.to_tensor([float(r * r)]), dst=0)
res["gather"] = [float(o.numpy()[0]) for o in g]
red = paddle.to_tensor([float(r + 1)])
pg.reduce_on_calc_stream(red, dst=0)
res["reduce_root"] = float(red.numpy()[0]) if r == 0 else None
# point to point, incl. the partial send / recv of the pipeline
buf = paddle.zeros([4])
if r == 0:
    pg.send_on_calc_stream(paddle.to_tensor([1.0, 2.0, 3.0, 4.0]), dst=1)
    pg.send_partial_on_calc_stream(paddle.to_tensor([5.0, 6.0, 7.0, 8.0]), 1, 2, 1)
elif r == 1:
    pg.recv_on_calc_stream(buf, src=0)
    res["recv"] = buf.numpy().tolist()
    pbuf = paddle.zeros([4])
    pg.recv_partial_on_calc_stream(pbuf, 0, 2, 1)
    res["recv_partial"] = pbuf.numpy().tolist()
pg.barrier()
write_result(res)
