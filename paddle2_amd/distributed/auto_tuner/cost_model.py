"""Analytical memory / time model for decoder-only transformers on MI355X
(reference: auto_tuner/memory_cost_model.py, cost_model.py).

Memory per GPU (bytes), P = parameters, mp/pp/sh = degrees, s = seq, b = micro batch, h = hidden,
L = layers / pp:
  params bf16 2P/(mp pp) (/sh at stage 3), grads bf16 2P/(mp pp) (/sh at stage >= 2),
  AdamW fp32 master + m + v 12P/(mp pp sh) (stage >= 1), activations per layer
  s b h (34 / mp) bytes with flash attention (no s^2 term; Korthikanti et al. with SP), or 2 s b h
  with full recompute, times the number of in-flight micro batches (pp for 1F1B).
Time: 6 P tokens / (mp pp dp sh) FLOPs at an assumed 40% of the 2.5 PF dense bf16 peak, plus the
pipeline bubble (pp-1)/acc and a bandwidth term for sharding/dp gradient traffic over xGMI.
"""
from __future__ import annotations

HBM_GB = 288.0
PEAK_FLOPS = 2.5e15
XGMI_GBS = 7 * 153.0


def _params(m):
    h, L, v = m["hidden_size"], m["num_layers"], m.get("vocab_size", 32000)
    ffn = m.get("intermediate_size", int(8 * h / 3 // 256 * 256 + 256))
    kv = m.get("num_key_value_heads", m.get("num_attention_heads", 1))
    heads = m.get("num_attention_heads", 1)
    attn = h * h * 2 + 2 * h * (h // heads * kv)
    mlp = 3 * h * ffn if m.get("gated_mlp", True) else 2 * h * ffn
    return L * (attn + mlp + 2 * h) + 2 * v * h


def estimate_memory_gb(model_cfg, cfg):
    P = _params(model_cfg)
    mp, pp, sh = cfg.get("mp_degree", 1), cfg.get("pp_degree", 1), cfg.get("sharding_degree", 1)
    stage = cfg.get("sharding_stage", 1 if sh > 1 else 0)
    b, s, h = cfg.get("micro_batch_size", 1), model_cfg.get("seq_length", 4096), model_cfg["hidden_size"]
    L = model_cfg["num_layers"] / pp
    pw = 2 * P / (mp * pp) / (sh if stage >= 3 else 1)
    gr = 2 * P / (mp * pp) / (sh if stage >= 2 else 1)
    opt = 12 * P / (mp * pp) / (sh if stage >= 1 else 1)
    per_layer = layer_activation_bytes(s, b, h, mp, cfg)
    act = per_layer * L * inflight_micro_batches(pp, cfg.get("vpp_degree", 1) or 1)
    logits = 2 * s * b * model_cfg.get("vocab_size", 32000) * 4 / mp  # fp32 logits + grad
    return (pw + gr + opt + act + logits) / 2**30


# per-layer activation bytes (bf16) with flash attention, by recompute granularity: the attention block
# (qkv / rope / flash out / o-proj inputs) accounts for ~11 sbh of the 34 sbh/mp, core attention (flash
# output + softmax lse) for ~2 sbh; a recomputed block keeps only its input (2 sbh, not split by mp)
_ATTN_BLOCK, _CORE_ATTN = 11.0, 2.0


def layer_activation_bytes(s, b, h, mp, cfg):
    if not cfg.get("use_recompute", False):
        return s * b * h * 34 / mp
    gran = cfg.get("recompute_granularity") or "full"
    if gran == "full":
        return 2 * s * b * h
    if gran == "full_attn":
        return s * b * h * (34 - _ATTN_BLOCK) / mp + 2 * s * b * h
    return s * b * h * (34 - _CORE_ATTN) / mp


def inflight_micro_batches(pp, vpp=1):
    """Micro-batches whose activations the first 1F1B stage holds (interleaving adds (pp-1)/(pp*vpp))."""
    if pp <= 1:
        return 1
    return pp * (1 + (pp - 1) / (pp * vpp)) if vpp > 1 else pp


def get_mem(total_cards, parallel_cfg, l, h, a, V, s, gbs):
    """Peak GiB per GPU of a decoder-only model (reference cost_model.get_mem signature)."""
    m = {"num_layers": l, "hidden_size": h, "num_attention_heads": a, "vocab_size": V, "seq_length": s,
         "global_batch_size": gbs}
    return estimate_memory_gb(m, parallel_cfg)


def get_not_oom_cfgs(cfgs, tuner_cfg):
    """Structurally valid configs annotated with ``memory_cost`` (GiB), dropping those above
    ``per_card_memory`` (default: 288 GB HBM3E)."""
    m = tuner_cfg["model_cfg"]
    total = tuner_cfg.get("search_algo", {}).get("estimated_num_gpus", tuner_cfg.get("num_gpus"))
    cap = tuner_cfg.get("per_card_memory", HBM_GB)
    L, h, a, V, gbs = m["num_layers"], m["hidden_size"], m["num_attention_heads"], m["vocab_size"], \
        m["global_batch_size"]
    out = []
    for c in cfgs:
        mp, sh, mbs, pp, vpp, dp = (c["mp_degree"], c["sharding_degree"], c["micro_batch_size"], c["pp_degree"],
                                    c.get("vpp_degree", 1), c["dp_degree"])
        if mp * sh * pp * dp != total or gbs % (sh * dp * mbs) or L % (pp * vpp) or (vpp != 1 and pp <= 2):
            continue
        if a % mp or V % mp or h % mp:
            continue
        c = dict(c, memory_cost=get_mem(total, c, L, h, a, V, m.get("seq_length", 4096), gbs))
        if c["memory_cost"] <= cap:
            out.append(c)
    return out


def estimate_step_time(model_cfg, cfg, global_batch):
    P = _params(model_cfg)
    mp, pp = cfg.get("mp_degree", 1), cfg.get("pp_degree", 1)
    dp, sh = cfg.get("dp_degree", 1), cfg.get("sharding_degree", 1)
    s = model_cfg.get("seq_length", 4096)
    b = cfg.get("micro_batch_size", 1)
    acc = max(1, global_batch // (dp * sh * b))
    flops = 6 * P * s * global_batch * (4 / 3 if cfg.get("use_recompute", False) else 1)
    t = flops / (mp * pp * dp * sh) / (0.4 * PEAK_FLOPS)
    t *= 1 + (pp - 1) / acc
    t *= 1 + 0.1 / b  # small micro batches run the GEMMs / attention below MFMA saturation
    if mp > 1:
        t *= 1 + 0.05 * (mp - 1)  # per-layer activation all-reduce / gather cost
    comm_bytes = 2 * P / (mp * pp) * (2 if sh > 1 else 1)
    t += comm_bytes / (XGMI_GBS * 1e9) * (1 if dp * sh > 1 else 0) * 0.3  # mostly overlapped
    return t
