"""One rank, stage-3 tiny Llama: the N > 1 collective path forced on a 1-rank group
(PADDLE2_AMD_STAGE3_FORCE_COMM=1) or the N = 1 short-circuit; writes losses, every parameter's bytes digest and
which path ran.  Device from PD_TEST_DEVICE (cpu: gloo; cuda: the framework's RCCL group)."""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
from paddle2_amd.distributed import collective as C  # noqa: E402
from paddle2_amd.distributed.sharding import group_sharded_parallel  # noqa: E402
from paddle2_amd.models import LlamaConfig, LlamaForCausalLM  # noqa: E402

dev = os.environ.get("PD_TEST_DEVICE", "cpu")
C.init_parallel_env()
dtype = "bfloat16" if dev == "cuda" else "float32"
cfg = LlamaConfig.tiny(dtype=dtype, num_hidden_layers=3)
paddle.seed(7)
m = LlamaForCausalLM(cfg)
o = paddle.optimizer.AdamW(1e-2, parameters=m.parameters(), weight_decay=0.01,
                           grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0), multi_precision=True)
m, o, _ = group_sharded_parallel(m, o, "p_g_os")
g = torch.Generator().manual_seed(99)
losses = []
acc = int(os.environ.get("PD_TEST_ACC", "1"))
for s in range(4):
    for j in range(acc):
        ids = paddle.Tensor._wrap(torch.randint(0, cfg.vocab_size, (2, 65), generator=g).to(dev))
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        (loss / acc if acc > 1 else loss).backward()
    o.step()
    o.clear_grad()
    losses.append(float(loss))
if dev == "cuda":
    torch.cuda.synchronize()
h = hashlib.sha256()
for u in m._units:
    h.update(u.shard.detach().float().cpu().numpy().tobytes())
    if u.master is not None:
        h.update(u.master.detach().cpu().numpy().tobytes())
res = {"losses": losses, "digest": h.hexdigest(), "comm": [u.comm for u in m._units],
       "peak_live_flat": m.peak_live_flat, "pg": C.pg_status().get("backend"),
       "initialized": torch.distributed.is_initialized()}
with open(os.environ["PD_TEST_OUT"], "w") as f:
    json.dump(res, f)
