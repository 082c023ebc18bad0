"""paddle.optimizer (reference: python/paddle/optimizer/__init__.py)."""
from . import lr  # noqa: F401
from .optimizer import (SGD, ASGD, Adadelta, Adagrad, Adam, Adamax, AdamW, L1Decay, L2Decay, Lamb,  # noqa: F401
                        Momentum, NAdam, Optimizer, RAdam, RMSProp, Rprop)
from .lbfgs import LBFGS  # noqa: F401
