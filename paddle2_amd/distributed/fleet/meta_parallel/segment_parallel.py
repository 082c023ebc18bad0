"""SegmentParallel model wrapper (reference: python/paddle/distributed/fleet/meta_parallel/segment_parallel.py:26-40).

Segment (sequence) parallelism — the "sep" axis of the hybrid topology — splits every sequence of a batch across
the sep group; the attention layers exchange heads / segments with all-to-all (``fleet/utils/sequence_parallel_utils``
and the Ulysses / ring attention in ``meta_parallel/context_parallel.py``).  The wrapper itself makes the
replicated starting state identical along every axis that replicates it: sep first, then the model-parallel,
sharding and data-parallel groups when they are > 1.
"""
from __future__ import annotations

from ..utils.hybrid_parallel_util import broadcast_dp_parameters, broadcast_mp_parameters, \
    broadcast_sep_parameters, broadcast_sharding_parameters
from .meta_parallel_base import MetaParallelBase


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
