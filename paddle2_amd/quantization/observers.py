"""paddle.quantization.observers (reference: python/paddle/quantization/observers/)."""
from . import (AbsmaxObserver, AbsmaxObserverLayer, GroupWiseWeightObserver,  # noqa: F401
               GroupWiseWeightObserverLayer)

__all__ = ["AbsmaxObserver", "GroupWiseWeightObserver"]
