"""Mixture-of-Experts layer with expert parallelism (reference:
incubate/distributed/models/moe/moe_layer.py — ``MoELayer`` :263, ``prepare_forward`` :43,
``MoEScatter`` :99 / ``MoEGather`` :149 PyLayers over global_scatter / global_gather).

Dispatch: the (token, k) assignments are sorted by global expert id (one stable argsort), counts
per expert are exchanged with one all-to-all, tokens travel with ONE variable-split
``all_to_all_single`` each way (paddle2_amd.distributed.utils.moe_utils), local experts run on
contiguous row ranges, and the combine is a batched [1 x k] . [k x d] product per token.
"""
from __future__ import annotations

import torch

from .....framework.tensor import Tensor
from ..... import nn
from .....distributed.utils import moe_utils
from .gate import BaseGate, GShardGate, NaiveGate, SwitchGate

_wrap = Tensor._wrap


def prepare_forward(gate_idx, num_expert, world_size, moe_group=None):
    """-> (pos, local_expert_count, global_expert_count, fwd_expert_count, fwd_batch_size)."""
    idx = gate_idx._t if isinstance(gate_idx, Tensor) else gate_idx
    flat = idx.reshape(-1)
    tot = num_expert * world_size
    valid = flat >= 0
    key = torch.where(valid, flat, torch.full_like(flat, tot))
    pos = torch.argsort(key, stable=True)[: int(valid.sum())]
    local = torch.bincount(flat[valid], minlength=tot)
    glob = moe_utils.exchange_counts(local, moe_group) if world_size > 1 else local.clone()
    fwd = glob.reshape(world_size, num_expert).sum(0)
    return pos, local, glob, fwd, int(fwd.sum())


class MoELayer(nn.Layer):
    def __init__(self, d_model, experts, gate=None, moe_group=None, mp_group=None, recompute_interval=0,
                 recompute_ctx=None):
        super().__init__()
        self.recompute_ctx = recompute_ctx
        gate = {} if gate is None else gate
        self.group = moe_group
        self.world_size = moe_group.nranks if moe_group is not None else 1
        self.num_expert = len(experts)
        self.recompute_interval = recompute_interval
        self.experts = experts
        self.mp_group = mp_group
        self.d_model = d_model
        if isinstance(gate, dict):
            self.top_k = gate.get("top_k", 2)
            kind = gate.get("type", "gshard")
            if kind in ("naive", None):
                gate = NaiveGate(d_model, self.num_expert, self.world_size, topk=self.top_k)
            elif kind == "gshard":
                gate = GShardGate(d_model, self.num_expert, self.world_size, topk=self.top_k, group=self.group)
            elif kind == "switch":
                gate = SwitchGate(d_model, self.num_expert, self.world_size, topk=self.top_k, group=self.group)
            else:
                raise AssertionError(f"unsupported gate type {kind}")
        elif isinstance(gate, NaiveGate):
            self.top_k = gate.top_k
        elif isinstance(gate, BaseGate):
            raise TypeError(f"Unimplemented gate type: {type(gate)}")
        else:
            raise TypeError("gate must be a dict or a BaseGate")
        self.gate = gate

    def _experts_fwd(self, x, counts):
        outs, start = [], 0
        for e, c in enumerate(counts):
            if c <= 0:
                continue
            outs.append(self.experts[e](_wrap(x[start:start + c]))._t)
            start += c
        if not outs:
            return x[:0]
        return torch.cat(outs, 0)

    def forward(self, inp):
        assert len(inp.shape) == 3
        shp = inp.shape
        x = inp._t.reshape(-1, shp[2])
        value, gidx = self.gate(_wrap(x))
        k = gidx._t.shape[1] if gidx._t.dim() == 2 else 1
        pos, lcount, gcount, fcount, _ = prepare_forward(gidx, self.num_expert, self.world_size, self.group)
        lc, gc = [int(v) for v in lcount.tolist()], [int(v) for v in gcount.tolist()]
        xs = x.index_select(0, torch.div(pos, k, rounding_mode="floor"))
        if self.world_size > 1:
            xs = moe_utils._GlobalScatter.apply(xs, lc, gc, self.group)
        counts = [int(v) for v in fcount.tolist()]
        if self.recompute_interval > 0 and xs.shape[0] > 0:
            from .....distributed.fleet.recompute import recompute

            y = recompute(lambda t: _wrap(self._experts_fwd(t._t, counts)), _wrap(xs))._t
        else:
            y = self._experts_fwd(xs, counts)
        if self.world_size > 1:
            y = moe_utils._GlobalGather.apply(y, lc, gc, self.group)
        # scatter back into (token, k) slots; dropped assignments contribute 0
        n = x.shape[0]
        full = torch.zeros(n * k, y.shape[-1], dtype=y.dtype, device=y.device)
        full = full.index_copy(0, pos, y)
        full = full.reshape(n, k, -1)
        w = value._t.reshape(n, 1, k).to(full.dtype)
        out = torch.bmm(w, full).reshape(shp)
        return _wrap(out)
