"""Module-path alias (reference: python/paddle/distributed/fleet/meta_optimizers/dygraph_optimizer/
hybrid_parallel_optimizer.py): the implementation is in ``dygraph_optimizer/hybrid_parallel_optimizer.py``."""
from .dygraph_optimizer.hybrid_parallel_optimizer import *  # noqa
from .dygraph_optimizer.hybrid_parallel_optimizer import HybridParallelOptimizer  # noqa
