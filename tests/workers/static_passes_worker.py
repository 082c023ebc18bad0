"""Rank worker: static auto-parallel passes on a dist_main_program (DP plan over 2 ranks) — fused gradient
all-reduce, gradient merge, recompute, sharding stage 1 and AMP — each trained against the serial run."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed.auto_parallel.static import (allreduce_matmul_grad_overlap_pass,  # noqa: E402
                                                           amp_pass, build_dist_main_program,
                                                           fuse_allreduce_pass, gradient_merge_pass,
                                                           parallelize_program, recompute_pass,
                                                           sequence_parallel_optimization_pass, sharding_pass)
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
mesh = dist.ProcessMesh([0, 1], dim_names=["dp"])
passes = sys.argv[1].split(",")
out = {}


class MLP(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.fc1 = paddle.nn.Linear(8, 16)
        self.fc2 = paddle.nn.Linear(16, 4)

    def forward(self, x):
        return self.fc2(paddle.nn.functional.gelu(self.fc1(x))).pow(2).mean()


class TPMLP(paddle.nn.Layer):
    """column fc1 / row fc2 (Megatron MLP) + residual + an fc3 head whose loss rows are sharded: the plan carries a
    row-parallel all-reduce -> row-local ops -> sequence split chain and a column-parallel input c_identity"""

    def __init__(self):
        super().__init__()
        self.fc1 = paddle.nn.Linear(8, 16)
        self.fc2 = paddle.nn.Linear(16, 8)
        self.fc3 = paddle.nn.Linear(8, 4)

    def forward(self, x, y):
        h = self.fc2(paddle.nn.functional.gelu(self.fc1(x)))
        h = paddle.nn.functional.relu(h + x)
        return (self.fc3(h) - y).pow(2).mean()


class DeepMLP(paddle.nn.Layer):
    """8 equal layers: stage 3's per-use gathers must keep only a few of them gathered at a time"""

    def __init__(self):
        super().__init__()
        self.fcs = paddle.nn.LayerList([paddle.nn.Linear(8, 8) for _ in range(8)])

    def forward(self, x):
        for fc in self.fcs:
            x = paddle.nn.functional.gelu(fc(x))
        return x.pow(2).mean()


tp = any(p_ in ("spopt", "overlap") for p_ in passes)
paddle.seed(0)
if "deep" in passes:
    net, ref = DeepMLP(), DeepMLP()
else:
    net, ref = (TPMLP(), TPMLP()) if tp else (MLP(), MLP())
ref.set_state_dict(net.state_dict())
main = paddle.static.Program()
paddle.enable_static()
opt = paddle.optimizer.Adam(0.05, parameters=net.parameters())
with paddle.static.program_guard(main, paddle.static.Program()):
    xs = paddle.static.data("x", [8, 8], "float32")
    if tp:
        ys = paddle.static.data("y", [8, 4], "float32")
        loss = net(xs, ys)
    else:
        loss = net(xs)
    opt.minimize(loss)
paddle.disable_static()
if tp:
    ann = {"y": [dist.Shard(0)], net.fc1.weight: [dist.Shard(1)], net.fc1.bias: [dist.Shard(0)],
           net.fc2.weight: [dist.Shard(0)]}
else:
    ann = {"x": [dist.Shard(0)]}
dmp = build_dist_main_program(parallelize_program(main, mesh, ann), [loss])
out["comm_before"] = dmp.comm_ops()
k = 2 if "merge" in passes else 1
for name in passes:   # in the order given: fuse-then-merge and merge-then-fuse must both sum once per merged step
    if name == "fuse":
        fused = fuse_allreduce_pass(dmp, bucket_mb=1)
        out["buckets"] = len(fused.buckets())
    elif name == "merge":
        gradient_merge_pass(dmp, k)
if "recompute" in passes:
    first = [i for i, o in enumerate(dmp.program.ops) if o.kind == "torch"]
    recompute_pass(dmp, [(first[1], first[4])])
    out["recompute_ops"] = [o.name for o in dmp.program.ops if getattr(o.fn, "recompute", False)]
if "sharding" in passes:
    owners = sharding_pass(dmp, 0)
for st in (2, 3):
    if f"sharding{st}" in passes:
        owners = sharding_pass(dmp, 0, stage=st)
if "amp" in passes and passes.index("amp") < passes.index("spopt") if "spopt" in passes else False:
    # AMP first: the fc3 weight reaches its matmul as a bf16 cast GRAPH value of shape [8, 4] — its leading dim
    # equals the row count, the coincidence the sequence-parallel rewrite must not take for an activation
    out["amp_ops"] = amp_pass(dmp)
if "spopt" in passes:
    out["spopt"] = sequence_parallel_optimization_pass(dmp)
if "overlap" in passes:
    out["overlap"] = allreduce_matmul_grad_overlap_pass(dmp)
out["comm_after"] = dmp.comm_ops()
if "amp" in passes and "amp_ops" not in out:
    out["amp_ops"] = amp_pass(dmp)
exe = paddle.static.Executor()
ropt = paddle.optimizer.Adam(0.05, parameters=ref.parameters())
losses, ref_losses = [], []
for i in range(4):
    xi = np.random.RandomState(30 + i).randn(8, 8).astype("float32")
    yi = np.random.RandomState(60 + i).randn(8, 4).astype("float32")
    feed = {"x": xi, "y": yi} if tp else {"x": xi}
    (lv,) = exe.run(dmp.program, feed=dmp.local_feed(feed), fetch_list=[dmp.fetch(loss)])
    losses.append(float(lv))
    rl = ref(paddle.to_tensor(xi), paddle.to_tensor(yi)) if tp else ref(paddle.to_tensor(xi))
    (rl / k).backward()
    if (i + 1) % k == 0:
        ropt.step()
        ropt.clear_grad()
    ref_losses.append(float(rl.numpy()))
out["losses"], out["ref"] = losses, ref_losses
if any(f"sharding{st}" in passes for st in (2, 3)):
    bk2 = getattr(dmp, "stage2_buckets", None)
    if bk2 is not None:
        out["stage2_buckets"] = len(bk2.buckets)
        out["stage2_from_backward"] = bk2.from_backward
        out["stage2_issued"] = bk2.issued
    st3 = getattr(dmp, "stage3_state", None)
    if st3 is not None:
        nb = lambda p: p._t.numel() * p._t.element_size()  # noqa: E731
        out["stage3_peak"] = st3.peak
        out["stage3_gathers"] = st3.n_gathers
        out["stage3_units"] = len(st3.units)
        out["own_bytes"] = sum(nb(p) for p in net.parameters() if p._t.numel())
        out["unit_bytes"] = max(sum(4 * int(np.prod(st3.shapes[p.name])) for p in u) for u in st3.units)
        out["total_bytes"] = sum(4 * int(np.prod(v)) for v in st3.shapes.values())
    out["released"] = sum(1 for p in net.parameters() if p._t.numel() == 0)
    out["n_params_total"] = len(list(net.parameters()))
    dmp.gather_params()
if tp:
    # TP-sharded parameters: compare the local shard with the matching slice of the serial parameter
    def _local(ref_p, p):
        r = ref_p.numpy()
        if tuple(r.shape) == tuple(p._t.shape):
            return r
        ax = [d for d in range(r.ndim) if r.shape[d] != p._t.shape[d]][0]
        k = p._t.shape[ax]
        return np.take(r, range(dist.get_rank() * k, (dist.get_rank() + 1) * k), axis=ax)

    out["param_err"] = max(float(np.abs(_local(b, a) - a.numpy()).max()) for a, b in zip(net.parameters(),
                                                                                         ref.parameters()))
else:
    out["param_err"] = max(float(np.abs(a.numpy() - b.numpy()).max()) for a, b in zip(net.parameters(), ref.parameters()))
if any(p_.startswith("sharding") for p_ in passes):
    out["my_acc"] = len(opt._accumulators.get("moment1", {}))
    out["n_params"] = len(opt._parameter_list)
if "fuse" in passes:
    out["fused_calls"] = fused.calls
write_result(out)
