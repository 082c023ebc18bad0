"""Rank worker: semi-auto parallel DistTensor API + distributed checkpoint save/load with reshard."""
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
rank, world = dist.get_rank(), dist.get_world_size()
out = {}
mesh = dist.ProcessMesh([0, 1], dim_names=["x"])

# shard / reshard / unshard
g = np.arange(16, dtype="float32").reshape(4, 4)
d = dist.shard_tensor(paddle.to_tensor(g), mesh, [dist.Shard(0)])
out["local_rows"] = paddle.distributed.auto_parallel.local_tensor(d).numpy().tolist()
r = dist.reshard(d, mesh, [dist.Replicate()])
out["replicated_ok"] = bool(np.allclose(paddle.distributed.auto_parallel.local_tensor(r).numpy(), g))
out["unshard_ok"] = bool(np.allclose(dist.unshard_dtensor(d).numpy(), g))

# a column-sharded linear trains like the single-process one
paddle.seed(5)
lin = paddle.nn.Linear(4, 6)
ref = paddle.nn.Linear(4, 6)
ref.set_state_dict(lin.state_dict())


def shard_fn(name, layer, m):
    if isinstance(layer, paddle.nn.Linear):
        layer.weight = dist.shard_tensor(layer.weight, m, [dist.Shard(1)])


dist.shard_layer(lin, mesh, shard_fn)
opt = paddle.optimizer.AdamW(0.1, parameters=lin.parameters())
ropt = paddle.optimizer.AdamW(0.1, parameters=ref.parameters())
x = paddle.to_tensor(np.random.RandomState(0).randn(3, 4).astype("float32"))
xd = dist.shard_tensor(x, mesh, [dist.Replicate()])
for _ in range(3):
    loss = (lin(xd) ** 2).mean()
    loss.backward()
    opt.step()
    opt.clear_grad()
    rl = (ref(x) ** 2).mean()
    rl.backward()
    ropt.step()
    ropt.clear_grad()
full_w = dist.unshard_dtensor(lin.weight).numpy()
out["linear_diff"] = float(np.abs(full_w - ref.weight.numpy()).max())

# distributed checkpoint: save Shard(0) layout, load into Shard(1) and replicated targets
path = os.environ["PD_CKPT_DIR"]
sd = {"w": dist.shard_tensor(paddle.to_tensor(g), mesh, [dist.Shard(0)]), "b": paddle.to_tensor([1.0, 2.0])}
dist.save_state_dict(sd, path)
tgt = {"w": dist.shard_tensor(paddle.zeros([4, 4]), mesh, [dist.Shard(1)]), "b": paddle.zeros([2])}
dist.load_state_dict(tgt, path)
out["ckpt_shard1_ok"] = bool(np.allclose(dist.unshard_dtensor(tgt["w"]).numpy(), g))
out["ckpt_b_ok"] = tgt["b"].numpy().tolist() == [1.0, 2.0]
tgt2 = {"w": paddle.zeros([4, 4])}
dist.load_state_dict(tgt2, path)
out["ckpt_dense_ok"] = bool(np.allclose(tgt2["w"].numpy(), g))
out["files"] = sorted(os.listdir(path))
write_result(out)
