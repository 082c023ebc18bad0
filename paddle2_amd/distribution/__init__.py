"""paddle.distribution (reference: python/paddle/distribution/) on torch.distributions."""
from __future__ import annotations

import torch
import torch.distributions as D

from ..framework.tensor import Tensor

_w = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x, dtype=torch.float32)


class Distribution:
    _cls = None

    def __init__(self, *args, **kwargs):
        self._d = self._cls(*[_t(a) for a in args], **{k: _t(v) for k, v in kwargs.items()})

    def sample(self, shape=()):
        return _w(self._d.sample(tuple(shape)))

    def rsample(self, shape=()):
        return _w(self._d.rsample(tuple(shape)))

    def log_prob(self, value):
        return _w(self._d.log_prob(_t(value)))

    def prob(self, value):
        return _w(self._d.log_prob(_t(value)).exp())

    def entropy(self):
        return _w(self._d.entropy())

    @property
    def mean(self):
        return _w(self._d.mean)

    @property
    def variance(self):
        return _w(self._d.variance)

    def kl_divergence(self, other):
        return _w(D.kl_divergence(self._d, other._d))


def _mk(name, cls):
    return type(name, (Distribution,), {"_cls": cls})


Normal = _mk("Normal", D.Normal)
Uniform = _mk("Uniform", D.Uniform)
Categorical = _mk("Categorical", lambda logits: D.Categorical(logits=logits))
Bernoulli = _mk("Bernoulli", lambda probs: D.Bernoulli(probs=probs))
Beta = _mk("Beta", D.Beta)
Dirichlet = _mk("Dirichlet", D.Dirichlet)
Exponential = _mk("Exponential", D.Exponential)
Gamma = _mk("Gamma", D.Gamma)
Laplace = _mk("Laplace", D.Laplace)
LogNormal = _mk("LogNormal", D.LogNormal)
Multinomial = _mk("Multinomial", lambda total_count, probs: D.Multinomial(int(total_count), probs=probs))
Gumbel = _mk("Gumbel", D.Gumbel)
Geometric = _mk("Geometric", lambda probs: D.Geometric(probs=probs))
Cauchy = _mk("Cauchy", D.Cauchy)
Poisson = _mk("Poisson", D.Poisson)
Binomial = _mk("Binomial", lambda total_count, probs: D.Binomial(total_count, probs=probs))
StudentT = _mk("StudentT", D.StudentT)
Chi2 = _mk("Chi2", D.Chi2)
MultivariateNormal = _mk("MultivariateNormal", D.MultivariateNormal)


def kl_divergence(p, q):
    return p.kl_divergence(q)
