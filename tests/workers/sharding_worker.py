"""Rank worker: tiny Llama trained with group_sharded_parallel(level) vs. a single-process run on the
concatenated global batch; every rank writes its losses + a parameter checksum."""
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

level = sys.argv[1]
steps = 3
C.init_parallel_env()
rank, world = C.get_rank(), C.get_world_size()
cfg = LlamaConfig.tiny(dtype="float32", num_hidden_layers=int(os.environ.get("PD_TEST_LAYERS", "2")))


def make():
    paddle.seed(7)
    m = LlamaForCausalLM(cfg)
    o = paddle.optimizer.AdamW(1e-2, parameters=m.parameters(), weight_decay=0.01,
                               grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
    return m, o


g = torch.Generator().manual_seed(99)
data = [torch.randint(0, cfg.vocab_size, (world * 2, 33), generator=g) for _ in range(steps)]

# sharded run: each rank takes its 2 sequences
m, o = make()
m, o, _ = group_sharded_parallel(m, o, level)
losses = []
for s in range(steps):
    ids = paddle.Tensor._wrap(data[s][rank * 2:(rank + 1) * 2])
    loss = m(ids[:, :-1], labels=ids[:, 1:])
    loss.backward()
    o.step()
    o.clear_grad()
    t = loss._t.detach().clone()
    C._all_reduce_torch(t)
    losses.append(float(t) / world)
held_after_eval = held_next = None
if os.environ.get("PD_TEST_EVAL_NO_BWD") == "1" and level == "p_g_os":
    # a grad-enabled forward that never gets a backward: its kept units must not stay gathered for good
    ids = paddle.Tensor._wrap(data[0][rank * 2:(rank + 1) * 2])
    m(ids[:, :-1], labels=ids[:, 1:])
    held_after_eval = sum(1 for u in m._units if u.layer is not None and u.full is not None)
    with paddle.no_grad():
        m(ids[:, :-1], labels=ids[:, 1:])
    held_next = sum(1 for u in m._units if u.layer is not None and u.full is not None)
peak_live = getattr(m, "peak_live_flat", None)
pool_bufs = sum(len(v) for v in getattr(m, "_flat_pool", {}).values())
sizes = len({u.padded for u in getattr(m, "_units", [])})
gathers = sum(getattr(u, "n_gathers", 0) for u in getattr(m, "_units", []))
keep = getattr(m, "keep_gathered", None)
sd = m.state_dict()
csum = float(sum(v._t.double().sum() for v in sd.values()))

# single-process reference on the full batch
m2, o2 = make()
ref = []
for s in range(steps):
    ids = paddle.Tensor._wrap(data[s])
    loss = m2(ids[:, :-1], labels=ids[:, 1:])
    loss.backward()
    o2.step()
    o2.clear_grad()
    ref.append(float(loss))
csum_ref = float(sum(v._t.double().sum() for v in m2.state_dict().values()))
write_result({"losses": losses, "ref": ref, "csum": csum, "csum_ref": csum_ref, "peak_live_flat": peak_live,
              "pool_bufs": pool_bufs, "unit_sizes": sizes, "gathers": gathers, "keep": keep,
              "n_units": len(getattr(m, "_units", [])),
              "held_after_eval": held_after_eval, "held_next": held_next})
C.destroy_process_group()
