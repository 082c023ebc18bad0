"""TensorParallel / ShardingParallel / SegmentParallel model wrappers (reference:
fleet/meta_parallel/tensor_parallel.py, sharding_parallel.py, segment_parallel.py:26-40).

At construction they make replicated state identical across the relevant groups: non-distributed
params over the mp group, everything over the dp / sharding / sep groups.  Gradient reduction
happens in :class:`HybridParallelOptimizer` (one bucketed all-reduce per step), as in the reference.
"""
from __future__ import annotations

from ..utils.hybrid_parallel_util import broadcast_dp_parameters, broadcast_mp_parameters, \
    broadcast_sep_parameters, broadcast_sharding_parameters
from .meta_parallel_base import MetaParallelBase


class TensorParallel(MetaParallelBase):
    def _prepare_for_model(self):
        hcg = self._hcg
        broadcast_mp_parameters(self._layers, hcg)
        if hcg.get_sharding_parallel_world_size() > 1:
            broadcast_sharding_parameters(self._layers, hcg)
        if hcg.get_sep_parallel_world_size() > 1:
            broadcast_sep_parameters(self._layers, hcg)
        if hcg.get_data_parallel_world_size() > 1:
            broadcast_dp_parameters(self._layers, hcg)


class ShardingParallel(MetaParallelBase):
    def _prepare_for_model(self):
        broadcast_sharding_parameters(self._layers, self._hcg)
        if self._hcg.get_data_parallel_world_size() > 1:
            broadcast_dp_parameters(self._layers, self._hcg)


class SegmentParallel(MetaParallelBase):
    def _prepare_for_model(self):
        hcg = self._hcg
        broadcast_sep_parameters(self._layers, hcg)
        if hcg.get_model_parallel_world_size() > 1:
            broadcast_mp_parameters(self._layers, hcg)
        if hcg.get_sharding_parallel_world_size() > 1:
            broadcast_sharding_parameters(self._layers, hcg)
        if hcg.get_data_parallel_world_size() > 1:
            broadcast_dp_parameters(self._layers, hcg)
