"""Rank worker: a Llama model (embedding + 1 decoder layer + final norm) with semi-auto tensor-parallel
placements (vocab-sharded embedding, column/row-sharded projections) on 2 gloo ranks vs one process.
Every hot op goes through the SPMD dispatch at op entry (dist_ops.TRACE records them)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed.auto_parallel import _reshard_engine as RS, dist_ops  # noqa: E402
from paddle2_amd.models import LlamaConfig  # noqa: E402
from paddle2_amd.models.llama import LlamaModel  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
rank = dist.get_rank()
mesh = dist.ProcessMesh([0, 1], dim_names=["mp"])
cfg = LlamaConfig.tiny(dtype="float32", num_hidden_layers=1, fuse_attention_qkv=False, fuse_attention_ffn=False)
paddle.seed(3)
model = LlamaModel(cfg)
ref = LlamaModel(cfg)
ref.set_state_dict(model.state_dict())

COL = ("q_proj", "k_proj", "v_proj", "gate_proj", "up_proj")
ROW = ("o_proj", "down_proj")


def shard_fn(name, layer, m):
    leaf = name.split(".")[-1]
    if leaf in COL:
        layer.weight = dist.shard_tensor(layer.weight, m, [dist.Shard(1)])
    elif leaf in ROW:
        layer.weight = dist.shard_tensor(layer.weight, m, [dist.Shard(0)])
    elif leaf == "embed_tokens":
        layer.weight = dist.shard_tensor(layer.weight, m, [dist.Shard(0)])


dist.shard_layer(model, mesh, shard_fn)
ids = paddle.to_tensor(np.random.RandomState(1).randint(0, cfg.vocab_size, (2, 16)).astype("int64"))
dist_ops.TRACE.clear()
RS.COMM_LOG.clear()
out, _ = model(dist.shard_tensor(ids, mesh, [dist.Replicate()])), None
h = out[0] if isinstance(out, tuple) else out
loss = (h * h).mean()
loss.backward()
r = ref(ids)
rh = r[0] if isinstance(r, tuple) else r
rloss = (rh * rh).mean()
rloss.backward()

res = {"loss": float(dist.unshard_dtensor(loss).numpy()) if hasattr(loss._t, "full_tensor") else float(loss),
       "ref_loss": float(rloss), "out_diff": float(np.abs(dist.unshard_dtensor(h).numpy() - rh.numpy()).max())}
gd = {}
rp = dict(ref.named_parameters())
for n, p in model.named_parameters():
    g = p._t.grad
    if g is None:
        gd[n] = None
        continue
    gfull = g.full_tensor() if hasattr(g, "full_tensor") else g
    gd[n] = float((gfull.detach() - rp[n]._t.grad).abs().max())
res["grad_diff"] = gd
res["ops"] = sorted({t[0] for t in dist_ops.TRACE})
res["trace"] = [list(map(str, t)) for t in dist_ops.TRACE]
res["comms"] = sorted({c[0] for c in RS.COMM_LOG})
write_result(res)
