from .pp_layers import LayerDesc, PipelineLayer, SegmentLayers, SharedLayerDesc  # noqa
from ...layers.mpu.mp_layers import ColumnParallelLinear, ParallelCrossEntropy, RowParallelLinear, VocabParallelEmbedding  # noqa
from ...layers.mpu.random import RNGStatesTracker, get_rng_state_tracker, model_parallel_random_seed  # noqa
