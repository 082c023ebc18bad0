from .tensor_parallel import SegmentParallel  # noqa
