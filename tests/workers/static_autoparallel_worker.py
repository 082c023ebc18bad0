"""Rank worker: static auto-parallel engine — completion + partitioner on a recorded Program, TP (column / row
parallel) and DP plans against the serial run (loss, gradients, one SGD step, the collective plan)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed.auto_parallel.reshard import COMM_LOG  # noqa: E402
from paddle2_amd.distributed.auto_parallel.static import CostModel, parallelize_program  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
rank = dist.get_rank()
mesh = dist.ProcessMesh([0, 1], dim_names=["x"])
out = {}


class MLP(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc1 = paddle.nn.Linear(8, 16)
        self.fc2 = paddle.nn.Linear(16, 8)
        self.ln = paddle.nn.LayerNorm(8)

    def forward(self, x):
        h = paddle.nn.functional.gelu(self.fc1(x))
        y = self.ln(self.fc2(h) + x)
        return (y * y).mean()


paddle.seed(0)
net = MLP()
xv = np.random.RandomState(1).randn(4, 8).astype("float32")

# serial reference
x = paddle.to_tensor(xv)
ref_loss = net(x)
ref_loss.backward()
ref_g = {n: p.grad.numpy().copy() for n, p in net.named_parameters()}
net.clear_gradients()

main = paddle.static.Program()
paddle.enable_static()
with paddle.static.program_guard(main, paddle.static.Program()):
    xs = paddle.static.data("x", [4, 8], "float32")
    loss = net(xs)
paddle.disable_static()


def check(tag, ann, shard_of):
    dp = parallelize_program(main, mesh, ann)
    COMM_LOG.clear()
    lval = dp.run({"x": xv}, [loss])[0]
    fwd_log = list(COMM_LOG)
    lval._t.backward()
    ok = bool(abs(float(lval.numpy()) - float(ref_loss.numpy())) < 1e-5)
    gerr = 0.0
    for n, p in net.named_parameters():
        loc = dp.local_param(p)
        g = loc.grad.numpy()
        axis = shard_of.get(n)
        full = ref_g[n]
        want = np.split(full, 2, axis=axis)[rank] if axis is not None else full
        gerr = max(gerr, float(np.abs(g - want).max()))
    # one SGD step on the local shards == the serial step's slice
    with torch.no_grad():
        for t in dp.parameters():
            t -= 0.1 * t.grad
    w1 = dp.local_param(net.fc1.weight).detach().numpy()
    want_w1 = net.fc1.weight.numpy() - 0.1 * ref_g["fc1.weight"]
    ax = shard_of.get("fc1.weight")
    want_w1 = np.split(want_w1, 2, axis=ax)[rank] if ax is not None else want_w1
    out[tag] = {"loss_ok": ok, "grad_err": gerr, "step_ok": bool(np.allclose(w1, want_w1, atol=1e-6)),
                "fwd_comm": [k for k, _ in fwd_log], "all_comm": [k for k, _ in COMM_LOG],
                "plan": [p.key for p in dp.ctx.plans if p is not None],
                "est": CostModel().estimate(dp.ctx)["comm_s"]}


# tensor parallel: fc1 column-parallel, fc2 row-parallel (Megatron pairing)
check("tp", {net.fc1.weight: [dist.Shard(1)], net.fc1.bias: [dist.Shard(0)], net.fc2.weight: [dist.Shard(0)]},
      {"fc1.weight": 1, "fc1.bias": 0, "fc2.weight": 0})
# data parallel: the batch is sharded, every parameter replicated
check("dp", {"x": [dist.Shard(0)]}, {})


# Engine: the same MLP trained 3 steps under the TP plan (parameters hold local shards, user's SGD steps them)
from paddle2_amd.distributed.auto_parallel.static import Engine  # noqa: E402

paddle.seed(0)
net2 = MLP()
ref2 = MLP()
ref2.set_state_dict(net2.state_dict())
eng = Engine(net2, loss=lambda out, label: out, optimizer=paddle.optimizer.SGD(0.1, parameters=net2.parameters()), mesh=mesh,
             annotations={net2.fc1.weight: [dist.Shard(1)], net2.fc1.bias: [dist.Shard(0)],
                          net2.fc2.weight: [dist.Shard(0)]})
opt_ref = paddle.optimizer.SGD(0.1, parameters=ref2.parameters())
losses, ref_losses = [], []
dummy = np.zeros([4], "float32")
for i in range(3):
    xi = np.random.RandomState(10 + i).randn(4, 8).astype("float32")
    losses.append(float(eng.run([xi], [dummy], "train").numpy()))
    lr_ = ref2(paddle.to_tensor(xi))
    lr_.backward()
    opt_ref.step()
    opt_ref.clear_grad()
    ref_losses.append(float(lr_.numpy()))
out["engine"] = {"losses": losses, "ref": ref_losses,
                 "w1_local_shape": list(net2.fc1.weight._t.shape),
                 "pred_shape": list(eng.run([np.ones([4, 8], "float32")], None, "predict").shape)}
write_result(out)
