"""paddle.regularizer (reference: python/paddle/regularizer.py): weight-decay rules attached to an optimizer
(``regularization=``) or to one parameter (``ParamAttr(regularizer=...)``, which wins over the optimizer's).

The reference appends a ``scale`` / ``sign`` op per parameter to the program; here a rule is a small value object
the optimizers consult when they assemble each parameter's gradient (``Optimizer._reg_grad``):

    L2Decay:  g + coeff * w              L1Decay:  g + coeff * sign(w)

A bare float passed as ``regularization`` means L2Decay(float).  AdamW's decoupled ``weight_decay`` is not a
regularizer (it scales the parameter in the update, not the gradient) and does not go through this module.
"""
from __future__ import annotations

import torch

__all__ = ["L1Decay", "L2Decay", "WeightDecayRegularizer"]


class WeightDecayRegularizer:
    """Base class: ``decay(param, grad)`` returns the gradient with the rule's term added."""

    def __init__(self, coeff=0.0):
        self._coeff = float(coeff)

    @property
    def coeff(self):
        return self._coeff

    def decay(self, param: torch.Tensor, grad: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def __call__(self, param, grad, block=None):
        # reference signature (param, grad, block); block is the static-graph block and unused here
        return self.decay(param, grad)

    def __repr__(self):
        return f"{type(self).__name__}(coeff={self._coeff})"


class L2Decay(WeightDecayRegularizer):
    """L2 weight decay: loss + coeff / 2 * ||w||^2, i.e. grad + coeff * w."""

    def decay(self, param, grad):
        return grad + self._coeff * param.to(grad.dtype) if self._coeff else grad

    def __str__(self):
        return f"L2Decay, coeff={self._coeff}"


class L1Decay(WeightDecayRegularizer):
    """L1 weight decay: loss + coeff * ||w||_1, i.e. grad + coeff * sign(w)."""

    def decay(self, param, grad):
        return grad + self._coeff * torch.sign(param).to(grad.dtype) if self._coeff else grad

    def __str__(self):
        return f"L1Decay, coeff={self._coeff}"


def as_regularizer(reg):
    """None, a float (-> L2Decay) or a WeightDecayRegularizer -> a WeightDecayRegularizer or None."""
    if reg is None or isinstance(reg, WeightDecayRegularizer):
        return reg
    return L2Decay(float(reg))
