"""ShardingParallel model wrapper (reference: python/paddle/distributed/fleet/meta_parallel/sharding_parallel.py).

Under a hybrid topology with a sharding axis the wrapper only makes the replicated starting state identical: every
parameter is broadcast from the sharding group's first rank (and over the data-parallel group when that axis is
also > 1).  Partitioning the optimizer state, gradients and parameters is the sharding optimizer's job
(``meta_optimizers/dygraph_optimizer`` DygraphShardingOptimizer, ``distributed/sharding/group_sharded.py``), and the
gradient reduction happens in HybridParallelOptimizer — the same split of duties as the reference.
"""
from __future__ import annotations

from ..utils.hybrid_parallel_util import broadcast_dp_parameters, broadcast_sharding_parameters
from .meta_parallel_base import MetaParallelBase


class ShardingParallel(MetaParallelBase):
    def _prepare_for_model(self):
        hcg = self._hcg
        broadcast_sharding_parameters(self._layers, hcg)
        if hcg.get_data_parallel_world_size() > 1:
            broadcast_dp_parameters(self._layers, hcg)
