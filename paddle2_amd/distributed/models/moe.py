"""paddle.distributed.models.moe.utils equivalents (reference: distributed/models/moe/utils.py)."""
from ...incubate.distributed.models.moe import *  # noqa: F401,F403
from ..utils.moe_utils import global_gather, global_scatter  # noqa: F401
