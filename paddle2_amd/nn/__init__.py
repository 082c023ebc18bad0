"""paddle.nn (reference: python/paddle/nn/__init__.py)."""
from . import functional, initializer, utils  # noqa: F401
from .decode import BeamSearchDecoder, dynamic_decode  # noqa: F401
from .clip import ClipGradByGlobalNorm, ClipGradByNorm, ClipGradByValue  # noqa: F401
from .layer import *  # noqa: F401,F403
from .layer.layers import Layer  # noqa: F401
from ..framework.param import ParamAttr, Parameter  # noqa: F401
