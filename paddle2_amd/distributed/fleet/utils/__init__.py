"""paddle.distributed.fleet.utils (reference: python/paddle/distributed/fleet/utils/)."""
from ..recompute import recompute, recompute_hybrid, recompute_sequential  # noqa
from . import hybrid_parallel_util, mix_precision_utils, sequence_parallel_utils  # noqa
from .fs import HDFSClient, LocalFS  # noqa
from .hybrid_parallel_util import fused_allreduce_gradients  # noqa
from .timer_helper import get_timers, set_timers  # noqa
from . import hybrid_parallel_inference, log_util, pp_parallel_adaptor  # noqa
from .hybrid_parallel_inference import HybridParallelInferenceHelper  # noqa
