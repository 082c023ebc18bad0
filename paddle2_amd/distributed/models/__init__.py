"""paddle.distributed.models (reference: python/paddle/distributed/models/moe): MoE utilities."""
from . import moe  # noqa: F401
