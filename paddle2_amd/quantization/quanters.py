"""paddle.quantization.quanters (reference: python/paddle/quantization/quanters/abs_max.py)."""
from . import FakeQuanterWithAbsMaxObserver, FakeQuanterWithAbsMaxObserverLayer  # noqa: F401

__all__ = ["FakeQuanterWithAbsMaxObserver"]
