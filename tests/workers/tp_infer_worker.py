"""Rank worker: tensor-parallel fused inference ops (ring_id all-reduce) vs. the same op on one rank with the full
weights (reference test: test/legacy_test/test_fused_multi_transformer_op.py with nranks > 1)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
from paddle2_amd.distributed import collective as C  # noqa: E402
from paddle2_amd.incubate.nn import functional as IF  # noqa: E402
from paddle2_amd.serving import fused_multi_transformer  # noqa: E402
from _dist import write_result  # noqa: E402

C.init_parallel_env()
rank, world = C.get_rank(), C.get_world_size()
W = paddle.Tensor._wrap
g = torch.Generator().manual_seed(0)
L, b, s, d, nh, hd, f = 2, 2, 5, 32, 4, 8, 48
nl, fl = nh // world, f // world
rn = lambda *sh: torch.randn(*sh, generator=g) * 0.2  # noqa: E731
full = {
    "ln": [1 + rn(d) for _ in range(L)], "lnb": [rn(d) for _ in range(L)],
    "qkv": [rn(3, nh, hd, d) for _ in range(L)], "qkvb": [rn(3 * nh * hd) for _ in range(L)],
    "lin": [rn(nh * hd, d) for _ in range(L)], "linb": [rn(d) for _ in range(L)],
    "fln": [1 + rn(d) for _ in range(L)], "flnb": [rn(d) for _ in range(L)],
    "f1": [rn(d, f) for _ in range(L)], "f1b": [rn(f) for _ in range(L)],
    "f2": [rn(f, d) for _ in range(L)], "f2b": [rn(d) for _ in range(L)],
}
x = rn(b, s, d)


def shard(k, t):
    hs = slice(rank * nl, (rank + 1) * nl)
    fs = slice(rank * fl, (rank + 1) * fl)
    if k == "qkv":
        return t[:, hs].contiguous()
    if k == "qkvb":
        return t.reshape(3, nh, hd)[:, hs].reshape(-1).contiguous()
    if k == "lin":
        return t.reshape(nh, hd, d)[hs].reshape(-1, d).contiguous()
    if k in ("f1", "f1b"):
        return t[..., fs].contiguous()
    if k == "f2":
        return t[fs].contiguous()
    return t


def run_fmt(ws, heads, ring):
    ps = {k: [W(t) for t in v] for k, v in ws.items()}
    caches = [W(torch.zeros(2, b, heads, 16, hd)) for _ in range(L)]
    ctx, _ = fused_multi_transformer(W(x[:, :s - 1].contiguous()), ps["ln"], ps["lnb"], ps["qkv"], ps["qkvb"],
                                     ps["lin"], ps["linb"], ps["fln"], ps["flnb"], ps["f1"], ps["f1b"], ps["f2"],
                                     ps["f2b"], cache_kvs=caches, ring_id=ring)
    last, _ = fused_multi_transformer(W(x[:, s - 1:].contiguous()), ps["ln"], ps["lnb"], ps["qkv"], ps["qkvb"],
                                      ps["lin"], ps["linb"], ps["fln"], ps["flnb"], ps["f1"], ps["f1b"], ps["f2"],
                                      ps["f2b"], cache_kvs=caches, time_step=s - 1, ring_id=ring)
    return torch.cat([ctx._t, last._t], 1)


ref = run_fmt(full, nh, -1)
tp = run_fmt({k: [shard(k, t) for t in v] for k, v in full.items()}, nl, 0)
out = {"fmt_diff": float((ref - tp).abs().max())}

# fused_feedforward (pre-LN, eval)
def ffn(w1, b1, w2, ring):
    return IF.fused_feedforward(W(x), W(w1), W(w2), W(b1), W(full["f2b"][0]), W(full["ln"][0]), W(full["lnb"][0]),
                                pre_layer_norm=True, training=False, activation="gelu", ring_id=ring)._t


r = ffn(full["f1"][0], full["f1b"][0], full["f2"][0], -1)
t = ffn(shard("f1", full["f1"][0]), shard("f1b", full["f1b"][0]), shard("f2", full["f2"][0]), 0)
out["ffn_diff"] = float((r - t).abs().max())

# fused_multi_head_attention (pre-LN, fp32 path)
def mha(qkv, qkvb, lin, ring):
    return IF.fused_multi_head_attention(W(x), W(qkv), W(lin), pre_layer_norm=True, pre_ln_scale=W(full["ln"][0]),
                                         pre_ln_bias=W(full["lnb"][0]), qkv_bias=W(qkvb.reshape(3, -1, hd)),
                                         linear_bias=W(full["linb"][0]), training=False, ring_id=ring)._t


r = mha(full["qkv"][0], full["qkvb"][0], full["lin"][0], -1)
t = mha(shard("qkv", full["qkv"][0]), shard("qkvb", full["qkvb"][0]), shard("lin", full["lin"][0]), 0)
out["mha_diff"] = float((r - t).abs().max())
try:
    fused_multi_transformer(W(x), *[[W(t) for t in full[k]] for k in ("ln", "lnb", "qkv", "qkvb", "lin", "linb",
                                                                       "fln", "flnb", "f1", "f1b", "f2", "f2b")],
                            ring_id=77)
    out["bad_ring"] = "accepted"
except ValueError:
    out["bad_ring"] = "raised"
write_result(out)
