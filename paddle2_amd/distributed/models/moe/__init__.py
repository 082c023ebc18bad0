"""paddle.distributed.models.moe (reference: python/paddle/distributed/models/moe/): the routing helpers in
``utils``; the MoE layer and gates are ``paddle.incubate.distributed.models.moe``, the expert all-to-all
``distributed/utils/moe_utils.py`` (global_scatter / global_gather)."""
from . import utils  # noqa: F401
from ....incubate.distributed.models.moe import *  # noqa: F401,F403
from ...utils.moe_utils import global_gather, global_scatter  # noqa: F401
