from . import moe_utils  # noqa
from .moe_utils import global_gather, global_scatter  # noqa
