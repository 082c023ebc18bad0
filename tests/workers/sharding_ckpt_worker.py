"""Rank worker: stage-3 sharding with offload / exclude_layer on W ranks, and checkpoint portability.

mode "train <opt> <ckpt_dir>": W ranks train 3 steps of a tiny fp32 Llama (global batch 4), compare the
losses with a single-process run on the same global batches, and save the sharded model + optimizer
state (reference layout, full tensors) to ckpt_dir.
mode "resume <opt> <ckpt_dir>": W ranks (a different degree) load that checkpoint, train steps 4-5 and
compare with a single-process run of 5 uninterrupted steps.
<opt> is "plain", "offload" or "exclude" (exclude_layer=["LlamaRMSNorm"]).
"""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
from paddle2_amd.distributed import collective as C  # noqa: E402
from paddle2_amd.distributed.sharding import group_sharded_parallel  # noqa: E402
from paddle2_amd.models import LlamaConfig, LlamaForCausalLM  # noqa: E402
from _dist import write_result  # noqa: E402

mode, opt_kind, ckpt = sys.argv[1], sys.argv[2], sys.argv[3]
C.init_parallel_env()
rank, world = C.get_rank(), C.get_world_size()
cfg = LlamaConfig.tiny(dtype="float32", num_hidden_layers=2)
GB = 4
g = torch.Generator().manual_seed(123)
data = [torch.randint(0, cfg.vocab_size, (GB, 17), generator=g) for _ in range(5)]


def make():
    paddle.seed(11)
    m = LlamaForCausalLM(cfg)
    o = paddle.optimizer.AdamW(5e-3, parameters=m.parameters(), weight_decay=0.01,
                               grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    return m, o


def wrap(m, o):
    kw = {}
    if opt_kind == "offload":
        kw["offload"] = True
    if opt_kind == "exclude":
        kw["exclude_layer"] = ["LlamaRMSNorm"]
    return group_sharded_parallel(m, o, "p_g_os", **kw)[:2]


def run_steps(m, o, steps, sharded):
    per = GB // world
    out = []
    for s in steps:
        batch = data[s][rank * per:(rank + 1) * per] if sharded else data[s]
        ids = paddle.Tensor._wrap(batch)
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        o.step()
        o.clear_grad()
        if sharded:
            t = loss._t.detach().clone()
            C._all_reduce_torch(t)
            out.append(float(t) / world)
        else:
            out.append(float(loss))
    return out


res = {}
if mode == "train":
    m, o = wrap(*make())
    res["losses"] = run_steps(m, o, range(3), True)
    msd, osd = m.state_dict(), o.state_dict()  # collective: every rank takes part
    if rank == 0:
        os.makedirs(ckpt, exist_ok=True)
        paddle.save(msd, os.path.join(ckpt, "model.pdparams"))
        paddle.save(osd, os.path.join(ckpt, "model.pdopt"))
    C.barrier()
    m2, o2 = make()
    res["ref"] = run_steps(m2, o2, range(3), False)
    if opt_kind == "exclude":
        norm_w = [p for n, p in m._layer.named_parameters() if "norm" in n]
        res["norm_full"] = all(p._t.numel() == cfg.hidden_size for p in norm_w)
else:
    m, o = wrap(*make())
    m.set_state_dict(paddle.load(os.path.join(ckpt, "model.pdparams")))
    o.set_state_dict(paddle.load(os.path.join(ckpt, "model.pdopt")))
    res["losses"] = run_steps(m, o, range(3, 5), True)
    m2, o2 = make()
    res["ref"] = run_steps(m2, o2, range(5), False)[3:]
write_result(res)
C.destroy_process_group()
