"""Rank worker: the Resharder's explicit dist_main_program — a minimize'd serial Program (MLP + SGD) completed under a
TP plan (fc1 column-parallel, fc2 row-parallel) or a DP plan, partitioned, materialised with communication ops and
trained 3 steps by the framework's static Executor against the serial dygraph run."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed.auto_parallel.static import build_dist_main_program, parallelize_program  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
mesh = dist.ProcessMesh([0, 1], dim_names=["x"])
mode = sys.argv[1]
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
net, ref = MLP(), MLP()
ref.set_state_dict(net.state_dict())
main = paddle.static.Program()
paddle.enable_static()
with paddle.static.program_guard(main, paddle.static.Program()):
    xs = paddle.static.data("x", [4, 8], "float32")
    loss = net(xs)
    paddle.optimizer.SGD(0.1, parameters=net.parameters()).minimize(loss)
paddle.disable_static()

if mode == "tp":
    ann = {net.fc1.weight: [dist.Shard(1)], net.fc1.bias: [dist.Shard(0)], net.fc2.weight: [dist.Shard(0)]}
else:
    ann = {"x": [dist.Shard(0)]}
dmp = build_dist_main_program(parallelize_program(main, mesh, ann), [loss])
out["comm_ops"] = dmp.comm_ops()
out["program"] = repr(dmp.program)
out["w1_local"] = list(net.fc1.weight._t.shape)
exe = paddle.static.Executor()
ropt = paddle.optimizer.SGD(0.1, parameters=ref.parameters())
losses, ref_losses = [], []
for i in range(3):
    xi = np.random.RandomState(20 + i).randn(4, 8).astype("float32")
    (lv,) = exe.run(dmp.program, feed=dmp.local_feed({"x": xi}), fetch_list=[dmp.fetch(loss)])
    losses.append(float(lv))
    rl = ref(paddle.to_tensor(xi))
    rl.backward()
    ropt.step()
    ropt.clear_grad()
    ref_losses.append(float(rl.numpy()))
out["losses"], out["ref"] = losses, ref_losses
# trained parameters: this rank's shard of the serial ones
r = dist.get_rank()
w1_ref = ref.fc1.weight.numpy()
w1_ref = np.split(w1_ref, 2, axis=1)[r] if mode == "tp" else w1_ref
w2_ref = ref.fc2.weight.numpy()
w2_ref = np.split(w2_ref, 2, axis=0)[r] if mode == "tp" else w2_ref
out["param_err"] = max(float(np.abs(net.fc1.weight._t.detach().numpy() - w1_ref).max()),
                       float(np.abs(net.fc2.weight._t.detach().numpy() - w2_ref).max()),
                       float(np.abs(net.fc2.bias._t.detach().numpy() - ref.fc2.bias.numpy()).max()),
                       float(np.abs(net.ln.weight._t.detach().numpy() - ref.ln.weight.numpy()).max()))
write_result(out)
