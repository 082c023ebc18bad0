"""Exponential-family base (reference: python/paddle/distribution/exponential_family.py).

p(x; theta) = h(x) exp(<t(x), theta> - A(theta)).  Subclasses give the natural parameters and the log
normalizer A; entropy (and the fallback KL in kl.py) come from the Bregman divergence of A, whose gradient
(the expected sufficient statistic) is taken with autograd.
"""
from __future__ import annotations

import torch

from .distribution import Distribution, _wrap


class ExponentialFamily(Distribution):
    @property
    def _natural_parameters(self):
        raise NotImplementedError

    def _log_normalizer(self, *natural):
        raise NotImplementedError

    @property
    def _mean_carrier_measure(self):
        raise NotImplementedError

    def _nat(self):
        nat = self._natural_parameters
        return nat() if callable(nat) else nat

    def entropy(self):
        """H = A(theta) - <theta, grad A(theta)> - E[log h(x)]."""
        nat = [t.detach().requires_grad_(True) for t in self._nat()]
        with torch.enable_grad():
            lognorm = self._log_normalizer(*nat)
            grads = torch.autograd.grad(lognorm.sum(), nat, create_graph=True)
        ent = lognorm
        for p, g in zip(nat, grads):
            ent = ent - p * g
        try:
            ent = ent - self._mean_carrier_measure
        except NotImplementedError:
            pass
        return _wrap(ent)
