"""paddle.regularizer (reference: python/paddle/regularizer.py)."""
from .optimizer.optimizer import L1Decay, L2Decay  # noqa: F401
WeightDecayRegularizer = L2Decay
