"""paddle.distributed.fleet.meta_parallel."""
from .meta_parallel_base import MetaParallelBase  # noqa
from .parallel_layers import (ColumnParallelLinear, LayerDesc, ParallelCrossEntropy, PipelineLayer,  # noqa
                              RNGStatesTracker, RowParallelLinear, SharedLayerDesc, VocabParallelEmbedding,
                              get_rng_state_tracker, model_parallel_random_seed)
from .pipeline_parallel import (PipelineParallel, PipelineParallelFThenB, PipelineParallelWithInterleave,  # noqa
                                PipelineParallelWithInterleaveFthenB, PipelineParallelZeroBubble)
from .tensor_parallel import SegmentParallel, ShardingParallel, TensorParallel  # noqa
