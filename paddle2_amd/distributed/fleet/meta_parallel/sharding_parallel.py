"""Module-path alias (reference: python/paddle/distributed/fleet/meta_parallel/sharding_parallel.py): the
implementations are in ``tensor_parallel.py``; the sharding itself is ``distributed/sharding/group_sharded.py``."""
from .tensor_parallel import SegmentParallel, ShardingParallel  # noqa
