from .hybrid_parallel_optimizer import DygraphShardingOptimizer, HybridParallelClipGrad, HybridParallelOptimizer  # noqa
