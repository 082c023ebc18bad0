"""Module-path alias (reference: python/paddle/distributed/fleet/meta_parallel/segment_parallel.py): the
implementation is ``SegmentParallel`` in ``tensor_parallel.py``."""
from .tensor_parallel import SegmentParallel  # noqa
