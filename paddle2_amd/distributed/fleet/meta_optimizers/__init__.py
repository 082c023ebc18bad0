from .dygraph_optimizer import DygraphShardingOptimizer, HybridParallelClipGrad, HybridParallelOptimizer  # noqa
