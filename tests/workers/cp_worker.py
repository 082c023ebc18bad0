"""Rank worker for context parallelism (sep axis) on gloo.

mode attn <ulysses|ring> <causal>: sharded attention output and q/k/v grads vs. full-sequence attention.
mode llama <ulysses|ring>: tiny Llama, sep_degree=world, sharded sequence; loss and sep-averaged grads after
    fleet's sep grad sync vs. a single-process full-sequence model.
"""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
from paddle2_amd.distributed import fleet  # noqa: E402
from paddle2_amd.distributed import collective as C  # noqa: E402
from paddle2_amd.distributed.fleet.meta_parallel import context_parallel as CP  # noqa: E402
from paddle2_amd.ops import torch_ops as T  # noqa: E402
from _dist import write_result  # noqa: E402

mode = sys.argv[1]
C.init_parallel_env()
rank, world = C.get_rank(), C.get_world_size()
strategy = fleet.DistributedStrategy()
strategy.hybrid_configs = {"dp_degree": 1, "mp_degree": 1, "pp_degree": 1, "sep_degree": world}
fleet.init(is_collective=True, strategy=strategy)
hcg = fleet.get_hybrid_communicate_group()
sep = hcg.get_sep_parallel_group()


def run_attn(kind, causal):
    g = torch.Generator().manual_seed(0)
    B, S, Hq, Hk, D = 2, 8 * world, 4, 2, 16
    q, k, v = (torch.randn(B, S, h, D, generator=g) for h in (Hq, Hk, Hk))
    go = torch.randn(B, S, Hq, D, generator=g)
    qr, kr, vr = (t.clone().requires_grad_(True) for t in (q, k, v))
    ref, _ = T.flash_attention(qr, kr, vr, causal)
    ref.backward(go)
    r = hcg.get_sep_parallel_rank()
    sh = (lambda t: CP.shard_sequence(t, world, r, kind))
    ql, kl, vl = (sh(t).clone().requires_grad_(True) for t in (q, k, v))
    fn = CP.ring_flash_attention if kind == "ring" else CP.ulysses_attention
    out = fn(ql, kl, vl, sep, causal=causal)
    out.backward(sh(go))
    err = lambda a, b: float((a - b).abs().max())  # noqa: E731
    write_result({"out": err(out, sh(ref)), "dq": err(ql.grad, sh(qr.grad)), "dk": err(kl.grad, sh(kr.grad)),
                  "dv": err(vl.grad, sh(vr.grad))})


def run_llama(kind):
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    g = torch.Generator().manual_seed(1)
    S = 16 * world
    ids = torch.randint(0, 512, (2, S + 1), generator=g)
    inputs, labels = ids[:, :-1], ids[:, 1:]

    def make(sep_deg):
        paddle.seed(5)
        return LlamaForCausalLM(LlamaConfig.tiny(dtype="float32", num_attention_heads=4, num_key_value_heads=2,
                                                 sep_parallel_degree=sep_deg, context_parallel=kind))

    ref = make(1)
    loss_ref = ref(paddle.Tensor._wrap(inputs), labels=paddle.Tensor._wrap(labels))
    loss_ref.backward()
    m = make(world)
    model = fleet.distributed_model(m)
    r = hcg.get_sep_parallel_rank()
    li = CP.shard_sequence(inputs, world, r, kind)
    ll = CP.shard_sequence(labels, world, r, kind)
    loss = model(paddle.Tensor._wrap(li), labels=paddle.Tensor._wrap(ll))
    loss.backward()
    # sep ranks hold replicas: average their grads (what HybridParallelOptimizer's dp_sep sync does)
    from paddle2_amd.distributed.fleet.utils.hybrid_parallel_util import fused_allreduce_gradients

    fused_allreduce_gradients(list(m.parameters()), hcg)
    lt = torch.tensor([float(loss)])
    torch.distributed.all_reduce(lt, group=sep.pg)
    gerr = 0.0
    for (n1, p1), (n2, p2) in zip(ref.named_parameters(), m.named_parameters()):
        g1, g2 = p1._t.grad, p2._t.grad
        gerr = max(gerr, float((g1 - g2).abs().max() / (g1.abs().max() + 1e-6)))
    write_result({"loss": float(lt) / world, "loss_ref": float(loss_ref), "grad_rel": gerr})


if mode == "attn":
    run_attn(sys.argv[2], sys.argv[3] == "1")
elif mode == "llama":
    run_llama(sys.argv[2])
