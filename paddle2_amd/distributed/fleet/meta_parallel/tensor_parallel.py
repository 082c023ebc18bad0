"""TensorParallel model wrapper (reference: fleet/meta_parallel/tensor_parallel.py); ShardingParallel and
SegmentParallel are in sharding_parallel.py / segment_parallel.py.

At construction they make replicated state identical across the relevant groups: non-distributed
params over the mp group, everything over the dp / sharding / sep groups.  Gradient reduction
happens in :class:`HybridParallelOptimizer` (one bucketed all-reduce per step), as in the reference.
"""
from __future__ import annotations

from ..utils.hybrid_parallel_util import broadcast_dp_parameters, broadcast_mp_parameters, \
    broadcast_sep_parameters, broadcast_sharding_parameters
from .meta_parallel_base import MetaParallelBase


def _broadcast_inputs(obj, src, group):
    """mp_configs.need_broadcast_data: every tensor input takes mp rank 0's value (in place)."""
    import torch
    import torch.distributed as dist

    from ....framework.tensor import Tensor

    if isinstance(obj, Tensor):
        obj = obj._t
    if isinstance(obj, torch.Tensor):
        c = obj.detach().contiguous()
        dist.broadcast(c, src=src, group=group.pg)
        if c.data_ptr() != obj.data_ptr():
            with torch.no_grad():
                obj.copy_(c)
    elif isinstance(obj, (list, tuple)):
        for o in obj:
            _broadcast_inputs(o, src, group)
    elif isinstance(obj, dict):
        for o in obj.values():
            _broadcast_inputs(o, src, group)


class TensorParallel(MetaParallelBase):
    def _prepare_for_model(self):
        hcg = self._hcg
        broadcast_mp_parameters(self._layers, hcg)
        mpc = self._strategy.hybrid_configs["mp_configs"] if self._strategy is not None else {}
        self._need_broadcast_data = bool(mpc.get("need_broadcast_data", True)) and \
            hcg.get_model_parallel_world_size() > 1
        if hcg.get_sharding_parallel_world_size() > 1:
            broadcast_sharding_parameters(self._layers, hcg)
        if hcg.get_sep_parallel_world_size() > 1:
            broadcast_sep_parameters(self._layers, hcg)
        if hcg.get_data_parallel_world_size() > 1:
            broadcast_dp_parameters(self._layers, hcg)

    def forward(self, *inputs, **kwargs):
        if self._need_broadcast_data:
            hcg = self._hcg
            _broadcast_inputs((inputs, kwargs), hcg.get_model_parallel_group_src_rank(),
                              hcg.get_model_parallel_group())
        return self._layers(*inputs, **kwargs)


# the sharding / segment wrappers live in their reference modules; re-exported for existing imports
from .segment_parallel import SegmentParallel  # noqa: E402,F401
from .sharding_parallel import ShardingParallel  # noqa: E402,F401
