from .tensor_parallel import SegmentParallel, ShardingParallel  # noqa
