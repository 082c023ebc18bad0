"""KL-divergence registry (reference: python/paddle/distribution/kl.py).

``register_kl(P, Q)`` registers a closed form; ``kl_divergence(p, q)`` dispatches on the most specific
registered (P, Q) pair along both MROs, and falls back to the Bregman divergence of the log normalizer for two
exponential-family members of the same type."""
from __future__ import annotations

import functools

import torch

from .continuous import (Beta, Cauchy, ContinuousBernoulli, Dirichlet, Exponential, Gamma, Laplace, LogNormal,
                         MultivariateNormal, Normal, Uniform)
from .discrete import Bernoulli, Binomial, Categorical, Geometric, Poisson
from .distribution import Distribution, _wrap, raw, sum_rightmost
from .exponential_family import ExponentialFamily

__all__ = ["register_kl", "kl_divergence"]

_REGISTRY = {}


def register_kl(cls_p, cls_q):
    if not (issubclass(cls_p, Distribution) and issubclass(cls_q, Distribution)):
        raise TypeError(f"cls_p and cls_q must be subclass of Distribution, but got {cls_p} and {cls_q}")

    def deco(f):
        _REGISTRY[cls_p, cls_q] = f
        _dispatch.cache_clear()
        return f

    return deco


@functools.lru_cache(maxsize=None)
def _dispatch(cls_p, cls_q):
    matches = [(p, q) for (p, q) in _REGISTRY if issubclass(cls_p, p) and issubclass(cls_q, q)]
    if not matches:
        raise NotImplementedError(f"KL divergence between {cls_p.__name__} and {cls_q.__name__} is not registered")

    def rank(pair):  # distance along each MRO: smaller = more specific
        return (cls_p.__mro__.index(pair[0]), cls_q.__mro__.index(pair[1]))

    return _REGISTRY[min(matches, key=rank)]


def kl_divergence(p, q):
    """KL(p || q)."""
    return _dispatch(type(p), type(q))(p, q)


@register_kl(Bernoulli, Bernoulli)
def _kl_bernoulli(p, q):
    return p.kl_divergence(q)


@register_kl(Beta, Beta)
def _kl_beta(p, q):
    a1, b1, a2, b2 = raw(p.alpha), raw(p.beta), raw(q.alpha), raw(q.beta)
    s1 = a1 + b1
    lb = lambda a, b: torch.lgamma(a) + torch.lgamma(b) - torch.lgamma(a + b)  # noqa: E731
    return _wrap(lb(a2, b2) - lb(a1, b1) + (a1 - a2) * torch.digamma(a1) + (b1 - b2) * torch.digamma(b1)
                 + (a2 - a1 + b2 - b1) * torch.digamma(s1))


@register_kl(Binomial, Binomial)
def _kl_binomial(p, q):
    return p.kl_divergence(q)


@register_kl(Dirichlet, Dirichlet)
def _kl_dirichlet(p, q):
    c1, c2 = raw(p.concentration), raw(q.concentration)
    s1, s2 = c1.sum(-1), c2.sum(-1)
    return _wrap(torch.lgamma(s1) - torch.lgamma(s2) - (torch.lgamma(c1) - torch.lgamma(c2)).sum(-1)
                 + ((c1 - c2) * (torch.digamma(c1) - torch.digamma(s1).unsqueeze(-1))).sum(-1))


@register_kl(Categorical, Categorical)
def _kl_categorical(p, q):
    return p.kl_divergence(q)


@register_kl(Cauchy, Cauchy)
def _kl_cauchy(p, q):
    return p.kl_divergence(q)


@register_kl(ContinuousBernoulli, ContinuousBernoulli)
def _kl_cb(p, q):
    return p.kl_divergence(q)


@register_kl(Normal, Normal)
def _kl_normal(p, q):
    return p.kl_divergence(q)


@register_kl(MultivariateNormal, MultivariateNormal)
def _kl_mvn(p, q):
    return p.kl_divergence(q)


@register_kl(Uniform, Uniform)
def _kl_uniform(p, q):
    lo1, hi1, lo2, hi2 = raw(p.low), raw(p.high), raw(q.low), raw(q.high)
    kl = ((hi2 - lo2) / (hi1 - lo1)).log()
    return _wrap(torch.where((lo2 > lo1) | (hi2 < hi1), torch.full_like(kl, float("inf")), kl))


@register_kl(Laplace, Laplace)
def _kl_laplace(p, q):
    return p.kl_divergence(q)


@register_kl(Geometric, Geometric)
def _kl_geometric(p, q):
    return p.kl_divergence(q)


@register_kl(ExponentialFamily, ExponentialFamily)
def _kl_expfamily(p, q):
    """KL = A(theta_q) - A(theta_p) - <theta_q - theta_p, grad A(theta_p)> (same family only)."""
    if type(p) is not type(q):
        raise NotImplementedError(f"KL between {type(p).__name__} and {type(q).__name__} is not registered")
    pn = [t.detach().requires_grad_(True) for t in p._nat()]
    qn = list(q._nat())
    with torch.enable_grad():
        ap = p._log_normalizer(*pn)
        grads = torch.autograd.grad(ap.sum(), pn, create_graph=True)
    kl = q._log_normalizer(*qn) - ap
    for tp, tq, g in zip(pn, qn, grads):
        term = (tq - tp) * g
        kl = kl - sum_rightmost(term, len(q.event_shape))
    return _wrap(kl)


@register_kl(Exponential, Exponential)
def _kl_exponential(p, q):
    return p.kl_divergence(q)


@register_kl(Gamma, Gamma)
def _kl_gamma(p, q):
    return p.kl_divergence(q)


@register_kl(LogNormal, LogNormal)
def _kl_lognormal(p, q):
    return p._base.kl_divergence(q._base)


@register_kl(Poisson, Poisson)
def _kl_poisson(p, q):
    return p.kl_divergence(q)
