"""MoE routing helpers (reference: python/paddle/distributed/models/moe/utils.py): the index bookkeeping between a
gate's top-k choice and the expert all-to-all (global_scatter / global_gather).

* ``_number_count(numbers, upper_range)``: tokens per expert id (ids < 0 are dropped tokens);
* ``_assign_pos(x, cum_count)``: token indices grouped by expert, expert e's tokens at
  ``[cum_count[e-1], cum_count[e])`` — the send order of the scatter;
* ``_random_routing(topk_idx, topk_value, prob, topk=2)``: GShard's random second-expert routing (the 2nd choice is
  kept only where 2 * its gate value >= a uniform sample);
* ``_limit_by_capacity(expert_count, capacity, n_worker)``: clip the [n_worker, n_expert] counts so no expert receives
  more than its capacity, filling workers in order;
* ``_prune_gate_by_capacity(gate_idx, expert_count, n_expert, n_worker)``: gate -1 for the tokens past their
  expert's (clipped) count, in token order.

They run on the framework's ops (``ops/extra_ops.py``: number_count, assign_pos, random_routing, limit_by_capacity,
prune_gate_by_capacity — device tensors in, device tensors out, no per-token host loop).
"""
from __future__ import annotations

from ....ops import extra_ops as _E
from ....framework.tensor import Tensor

__all__ = []


def _raw(x):
    return x._t if isinstance(x, Tensor) else x


def _number_count(numbers, upper_range):
    return _E.number_count(numbers, upper_range)


def _assign_pos(x, cum_count):
    cc = _raw(cum_count)
    return _E.assign_pos(x, cum_count, cc.reshape(-1)[-1:])


def _random_routing(topk_idx, topk_value, prob, topk=2):
    if topk != 2:
        raise RuntimeError("_random_routing supports topk=2 only (GShard)")
    return _E.random_routing(topk_idx, topk_value, prob)


def _limit_by_capacity(expert_count, capacity, n_worker):
    return _E.limit_by_capacity(expert_count, capacity, n_worker)


def _prune_gate_by_capacity(gate_idx, expert_count, n_expert, n_worker):
    return _E.prune_gate_by_capacity(gate_idx, expert_count, n_expert, n_worker)
