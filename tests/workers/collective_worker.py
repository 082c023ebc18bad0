"""Rank worker: every paddle.distributed collective on gloo + DataParallel vs single-process
(reference: test/collective/collective_*_api_dygraph.py, test_parallel_dygraph_dataparallel.py)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
r, n = dist.get_rank(), dist.get_world_size()
out = {}

t = paddle.to_tensor([float(r + 1)] * 3)
dist.all_reduce(t)
out["all_reduce"] = t.numpy().tolist()
t = paddle.to_tensor([float(r + 1)])
dist.all_reduce(t, op=dist.ReduceOp.MAX)
out["all_reduce_max"] = t.numpy().tolist()
lst = []
dist.all_gather(lst, paddle.to_tensor([r, r * 10]))
out["all_gather"] = [x.numpy().tolist() for x in lst]
b = paddle.to_tensor([r * 1.0 + 5])
dist.broadcast(b, src=1)
out["broadcast"] = b.numpy().tolist()
rd = paddle.to_tensor([1.0 * (r + 1)])
dist.reduce(rd, dst=0)
out["reduce"] = rd.numpy().tolist()
rs = paddle.zeros([2])
dist.reduce_scatter(rs, [paddle.to_tensor([1.0 * r, 2.0]), paddle.to_tensor([3.0, 4.0 * r])])
out["reduce_scatter"] = rs.numpy().tolist()
outs = []
dist.alltoall(outs, [paddle.to_tensor([r * 10 + 0]), paddle.to_tensor([r * 10 + 1])])
out["alltoall"] = [x.numpy().tolist() for x in outs]
sc = paddle.zeros([2])
dist.scatter(sc, [paddle.to_tensor([1.0, 1.0]), paddle.to_tensor([2.0, 2.0])] if r == 0 else None, src=0)
out["scatter"] = sc.numpy().tolist()
objs = []
dist.all_gather_object(objs, {"rank": r})
out["all_gather_object"] = objs
ol = [{"x": r}]
dist.broadcast_object_list(ol, src=1)
out["broadcast_object_list"] = ol
if r == 0:
    dist.send(paddle.to_tensor([42.0]), dst=1)
    out["p2p"] = None
else:
    rv = paddle.zeros([1])
    dist.recv(rv, src=0)
    out["p2p"] = rv.numpy().tolist()
peer = 1 - r
sbuf, rbuf = paddle.to_tensor([float(r)]), paddle.zeros([1])
tasks = dist.batch_isend_irecv([dist.P2POp(dist.isend, sbuf, peer), dist.P2POp(dist.irecv, rbuf, peer)])
for tk in tasks:
    tk.wait()
out["batch_p2p"] = rbuf.numpy().tolist()
g = dist.new_group([0, 1])
t = paddle.to_tensor([1.0])
dist.all_reduce(t, group=g)
out["group_sum"] = t.numpy().tolist()
task = dist.all_reduce(paddle.to_tensor([1.0]), sync_op=False)
task.wait()
dist.barrier()

# DataParallel vs single process on the global batch
paddle.seed(3)
net = paddle.nn.Sequential(paddle.nn.Linear(6, 16), paddle.nn.Tanh(), paddle.nn.Linear(16, 1))
ref = paddle.nn.Sequential(paddle.nn.Linear(6, 16), paddle.nn.Tanh(), paddle.nn.Linear(16, 1))
ref.set_state_dict(net.state_dict())
dp = paddle.DataParallel(net)
o = paddle.optimizer.SGD(0.1, parameters=dp.parameters())
ro = paddle.optimizer.SGD(0.1, parameters=ref.parameters())
gen = np.random.RandomState(0)
for s in range(3):
    X = gen.randn(8, 6).astype("float32")
    Y = gen.randn(8, 1).astype("float32")
    xs, ys = X[r * 4:(r + 1) * 4], Y[r * 4:(r + 1) * 4]
    loss = ((dp(paddle.to_tensor(xs)) - paddle.to_tensor(ys)) ** 2).mean()
    loss.backward()
    o.step()
    o.clear_grad()
    rl = ((ref(paddle.to_tensor(X)) - paddle.to_tensor(Y)) ** 2).mean()
    rl.backward()
    ro.step()
    ro.clear_grad()
out["dp_diff"] = float(max(np.abs(a.numpy() - b.numpy()).max() for a, b in zip(net.parameters(), ref.parameters())))
# no_sync accumulates locally
with dp.no_sync():
    ((dp(paddle.ones([2, 6]))) ** 2).mean().backward()
out["no_sync_ok"] = True
# partial p2p / allgather: rank 0 sends its second half, rank 1 receives it into its second half;
# then each rank holds its own quarter valid and partial_allgather completes the tensor
buf = paddle.to_tensor(np.arange(8, dtype="float32") + 100 * r)
if r == 0:
    dist.partial_send(buf, dst=1, num=2, id=1)
else:
    dist.partial_recv(buf, src=0, num=2, id=1)
out["partial_p2p"] = buf.numpy().tolist()
pa = paddle.to_tensor(np.where(np.arange(4) // 2 == r, np.arange(4, dtype="float32"), -1.0).astype("float32"))
dist.partial_allgather(pa, num=2, id=r)
out["partial_allgather"] = pa.numpy().tolist()
write_result(out)
