"""MoE gates (reference: incubate/distributed/models/moe/gate/{base,naive,gshard,switch}_gate.py)."""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from ......framework.tensor import Tensor
from ...... import nn

_wrap = Tensor._wrap


class BaseGate(nn.Layer):
    def __init__(self, num_expert, world_size):
        super().__init__()
        self.world_size = world_size
        self.num_expert = num_expert
        self.tot_expert = world_size * num_expert
        self.loss = None

    def forward(self, x):
        raise NotImplementedError

    def set_loss(self, loss):
        self.loss = loss

    def get_loss(self, clear=True):
        loss = self.loss
        if clear:
            self.loss = None
        return loss


class NaiveGate(BaseGate):
    """top-k of a linear router's raw logits (values are the combine weights, as in the reference)."""

    def __init__(self, d_model, num_expert, world_size, topk=2):
        super().__init__(num_expert, world_size)
        self.gate = nn.Linear(d_model, self.tot_expert)
        self.top_k = topk

    def forward(self, inp, return_all_scores=False):
        gate = self.gate(inp)._t
        val, idx = torch.topk(gate, k=self.top_k, dim=-1, largest=True, sorted=False)
        if return_all_scores:
            return _wrap(val), _wrap(idx), _wrap(gate)
        return _wrap(val), _wrap(idx)


def limit_by_capacity(topk_idx, num_expert, world_size, capacity, group=None):
    """Drop (-> -1) assignments beyond each expert's global ``capacity``.  Ranks claim capacity in
    rank order, tokens within a rank in token order (reference utils.limit_by_capacity)."""
    idx = topk_idx._t if isinstance(topk_idx, Tensor) else topk_idx
    tot = num_expert * world_size
    flat = idx.reshape(-1)
    valid = flat >= 0
    local = torch.bincount(flat[valid], minlength=tot)
    if world_size > 1:
        allc = [torch.empty_like(local) for _ in range(world_size)]
        g = group
        dist.all_gather(allc, local, group=None if g is None else g.pg)
        allc = torch.stack(allc)
        rank = dist.get_rank(None if g is None else g.pg)
        before = allc[:rank].sum(0) if rank > 0 else torch.zeros_like(local)
    else:
        before = torch.zeros_like(local)
    allowed = (capacity - before).clamp(min=0)
    # position of each assignment among earlier assignments to the same expert (token order)
    e = flat.clamp(min=0)
    onehot = torch.nn.functional.one_hot(e, tot) * valid[:, None]
    rank_in_e = (onehot.cumsum(0) - 1).gather(1, e[:, None]).squeeze(1)
    keep = valid & (rank_in_e < allowed[e])
    new = torch.where(keep, flat, torch.full_like(flat, -1)).reshape(idx.shape)
    new_local = torch.bincount(new.reshape(-1)[keep], minlength=tot)
    return _wrap(new_local), None, _wrap(new)


class GShardGate(NaiveGate):
    def __init__(self, d_model, num_expert, world_size, topk=2, capacity=(1.2, 2.4), random_routing=True,
                 group=None):
        assert topk == 2, "topk should be 2 in gshard"
        super().__init__(d_model, num_expert, world_size, topk)
        self.capacity = capacity
        self.random_routing = random_routing
        self.group = group

    def forward(self, x):
        val, idx, score = super().forward(x, return_all_scores=True)
        v, i, sc = val._t, idx._t, score._t
        s = sc.shape[0]
        top1 = i[:, 0] if i.dim() == 2 else i.reshape(-1)
        c_e = torch.bincount(top1.reshape(-1), minlength=self.tot_expert).float() / s
        m_e = torch.softmax(sc.float(), dim=1).mean(0)
        self.set_loss(_wrap((c_e * m_e).mean() * (self.num_expert ** 2)))
        cap = math.ceil((self.capacity[0] if self.training else self.capacity[1]) * x.shape[0])
        _, _, i2 = limit_by_capacity(i, self.num_expert, self.world_size, cap, self.group)
        i = i2._t
        if self.random_routing:
            prob = torch.rand(sc.shape[0], device=sc.device)
            drop2 = 2 * v[:, 1].float() < prob
            i = i.clone()
            i[:, 1] = torch.where(drop2, torch.full_like(i[:, 1], -1), i[:, 1])
        return _wrap(v), _wrap(i)


class SwitchGate(NaiveGate):
    def __init__(self, d_model, num_expert, world_size, topk=1, switch_eps=0.1, capacity=(1.2, 2.4), group=None):
        assert topk == 1, "topk should be 1 in switch"
        super().__init__(d_model, num_expert, world_size, topk=1)
        self.switch_eps = switch_eps
        self.capacity = capacity
        self.group = group

    def forward(self, inp):
        score = self.gate(inp)._t
        if self.training:
            noise = torch.rand_like(score) * 2 * self.switch_eps + 1.0 - self.switch_eps
            score = score + noise
        score = torch.softmax(score.float(), dim=-1)
        top1_score, top1_idx = torch.topk(score, k=1, dim=-1)
        cap = math.ceil((self.capacity[0] if self.training else self.capacity[1]) * inp.shape[0])
        _, _, i2 = limit_by_capacity(top1_idx, self.num_expert, self.world_size, cap, self.group)
        top1_idx = i2._t
        valid = top1_idx[top1_idx > -1]
        frac = torch.bincount(valid, minlength=self.tot_expert).float() / max(1, valid.numel())
        prob = score.sum(0) / max(1, valid.numel())
        self.set_loss(_wrap((frac * prob).sum() * self.tot_expert))
        return _wrap(top1_score.to(inp._t.dtype)), _wrap(top1_idx)
