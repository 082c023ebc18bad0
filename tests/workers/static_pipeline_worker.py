"""Rank worker: static pipeline training with incubate.optimizer.PipelineOptimizer — a Program whose layers are
placed on stages by device_guard("gpu:<k>") trains on 2 ranks (one stage each) through the FThenB / 1F1B / Eager1F1B
job lists with micro-batches, and the parameters match a serial dygraph run of the same model; plus
DistributedFusedLamb's sharded update against single-process LAMB."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.incubate.optimizer import DistributedFusedLamb, PipelineOptimizer  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
rank = torch.distributed.get_rank()
mode = sys.argv[1]
out = {"mode": mode}


class Net(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc1 = paddle.nn.Linear(8, 16)
        self.fc2 = paddle.nn.Linear(16, 16)
        self.fc3 = paddle.nn.Linear(16, 16)
        self.fc4 = paddle.nn.Linear(16, 1)

    def stage0(self, x):
        return paddle.nn.functional.gelu(self.fc2(paddle.tanh(self.fc1(x))))

    def stage1(self, h, y):
        return ((self.fc4(paddle.tanh(self.fc3(h))) - y) ** 2).mean()


if mode == "dfl":
    paddle.seed(3)
    net, ref = Net(), Net()
    ref.set_state_dict(net.state_dict())
    opt = DistributedFusedLamb(0.01, parameters=net.parameters())
    ropt = paddle.optimizer.Lamb(0.01, parameters=ref.parameters())
    for i in range(3):
        rs = np.random.RandomState(i)
        x = paddle.to_tensor(rs.randn(8, 8).astype("float32"))
        y = paddle.to_tensor(rs.randn(8, 1).astype("float32"))
        net.stage1(net.stage0(x), y).backward()    # same data on both ranks: the averaged gradient is the same
        opt.step()
        opt.clear_grad()
        ref.stage1(ref.stage0(x), y).backward()
        ropt.step()
        ropt.clear_grad()
    out["param_err"] = max(float(np.abs(a.numpy() - b.numpy()).max())
                           for a, b in zip(net.parameters(), ref.parameters()))
    write_result(out)
    sys.exit(0)

M = 4
paddle.seed(0)
net, ref = Net(), Net()
ref.set_state_dict(net.state_dict())
main = paddle.static.Program()
paddle.enable_static()
opt = PipelineOptimizer(paddle.optimizer.Adam(0.02, parameters=net.parameters()), num_microbatches=M,
                        schedule_mode=mode)
with paddle.static.program_guard(main, paddle.static.Program()):
    xs = paddle.static.data("x", [8, 8], "float32")
    ys = paddle.static.data("y", [8, 1], "float32")
    with paddle.static.device_guard("gpu:0"):
        h = net.stage0(xs)
    with paddle.static.device_guard("gpu:1"):
        loss = net.stage1(h, ys)
    opt.minimize(loss)
paddle.disable_static()
exe = paddle.static.Executor()
ropt = paddle.optimizer.Adam(0.02, parameters=ref.parameters())
losses, ref_losses = [], []
for i in range(3):
    rs = np.random.RandomState(10 + i)
    x, y = rs.randn(8 * M // 4 * 4, 8).astype("float32")[:8], rs.randn(8, 1).astype("float32")
    (lv,) = exe.run(main, feed={"x": x, "y": y}, fetch_list=[loss])
    losses.append(None if lv is None else float(lv))
    # serial reference: the mean over equal micro-batches of their mean losses = the full-batch mean
    rl = ref.stage1(ref.stage0(paddle.to_tensor(x)), paddle.to_tensor(y))
    rl.backward()
    ropt.step()
    ropt.clear_grad()
    ref_losses.append(float(rl.numpy()))
out["losses"], out["ref"] = losses, ref_losses
mine = [net.fc1, net.fc2] if rank == 0 else [net.fc3, net.fc4]
theirs = [ref.fc1, ref.fc2] if rank == 0 else [ref.fc3, ref.fc4]
out["param_err"] = max(float(np.abs(a.numpy() - b.numpy()).max())
                       for la, lb in zip(mine, theirs) for a, b in zip(la.parameters(), lb.parameters()))
other = [net.fc3, net.fc4] if rank == 0 else [net.fc1, net.fc2]
other_ref = [ref.fc3, ref.fc4] if rank == 0 else [ref.fc1, ref.fc2]
# parameters of the other stage are never stepped here
out["other_moved"] = max(float(np.abs(a.numpy() - b.numpy()).max())
                         for la, lb in zip(other, other_ref) for a, b in zip(la.parameters(), lb.parameters()))
runner = main._pipeline_opt["runner"]
out["stage"], out["n_local_ops"] = runner.stage, len(runner._local.ops)
out["n_send"], out["n_recv"] = len(runner._send), len(runner._recv)
write_result(out)
