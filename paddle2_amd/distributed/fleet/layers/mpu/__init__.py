from .mp_layers import ColumnParallelLinear, ParallelCrossEntropy, RowParallelLinear, VocabParallelEmbedding  # noqa
from .random import RNGStatesTracker, get_rng_state_tracker, model_parallel_random_seed  # noqa
from . import mp_ops  # noqa
