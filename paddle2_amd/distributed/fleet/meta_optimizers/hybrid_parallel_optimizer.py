from .dygraph_optimizer.hybrid_parallel_optimizer import *  # noqa
from .dygraph_optimizer.hybrid_parallel_optimizer import HybridParallelOptimizer  # noqa
