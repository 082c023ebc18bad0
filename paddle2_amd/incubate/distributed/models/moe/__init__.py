from .gate import BaseGate, GShardGate, NaiveGate, SwitchGate, limit_by_capacity  # noqa
from .moe_layer import MoELayer, prepare_forward  # noqa
