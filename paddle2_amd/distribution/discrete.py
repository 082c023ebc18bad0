"""Discrete distributions (reference: python/paddle/distribution/{bernoulli,binomial,categorical,geometric,
multinomial,poisson}.py)."""
from __future__ import annotations

import numbers

import torch
import torch.nn.functional as F

from ..framework.tensor import Tensor
from .distribution import Distribution, _wrap, check_shape, params, raw, value_like
from .exponential_family import ExponentialFamily


def _clip_probs(p):
    eps = torch.finfo(p.dtype).eps
    return p.clamp(eps, 1 - eps)


# =============================================================================================== Bernoulli
class Bernoulli(ExponentialFamily):
    def __init__(self, probs, name=None):
        self.name = name or "Bernoulli"
        (self.probs,) = params(probs) if not isinstance(probs, Tensor) else (probs,)
        p = raw(self.probs)
        self.logits = _wrap(_clip_probs(p).log() - torch.log1p(-_clip_probs(p)))
        self.dtype = p.dtype
        super().__init__(tuple(p.shape))

    @property
    def mean(self):
        return self.probs

    @property
    def variance(self):
        p = raw(self.probs)
        return _wrap(p * (1 - p))

    def sample(self, shape=()):
        with torch.no_grad():
            p = raw(self.probs)
            full = tuple(check_shape(shape)) + self.batch_shape
            return _wrap(torch.bernoulli(p.expand(full)))

    def rsample(self, shape=(), temperature=1.0):
        """Relaxed (Gumbel-sigmoid) reparameterized sample."""
        p = raw(self.probs)
        full = tuple(check_shape(shape)) + self.batch_shape
        u = torch.rand(full, dtype=p.dtype, device=p.device).clamp(torch.finfo(p.dtype).tiny, 1.0)
        logits = raw(self.logits)
        return _wrap(torch.sigmoid((logits + u.log() - torch.log1p(-u)) / temperature))

    def cdf(self, value):
        v = value_like(self.probs, value)
        p = raw(self.probs)
        zero, one = torch.zeros_like(v + p), torch.ones_like(v + p)
        return _wrap(torch.where(v < 0, zero, torch.where(v < 1, (1 - p) * one, one)))

    def log_prob(self, value):
        v = value_like(self.probs, value)
        logits = raw(self.logits)
        lg, vv = torch.broadcast_tensors(logits, v)
        return _wrap(-F.binary_cross_entropy_with_logits(lg, vv, reduction="none"))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def entropy(self):
        p = raw(self.probs)
        return _wrap(F.binary_cross_entropy_with_logits(raw(self.logits), p, reduction="none"))

    def kl_divergence(self, other):
        p, q = _clip_probs(raw(self.probs)), _clip_probs(raw(other.probs))
        return _wrap(p * (p.log() - q.log()) + (1 - p) * (torch.log1p(-p) - torch.log1p(-q)))

    def _natural_parameters(self):
        return (raw(self.logits),)

    def _log_normalizer(self, x):
        return F.softplus(x)


# =============================================================================================== Binomial
class Binomial(Distribution):
    def __init__(self, total_count, probs):
        self.total_count, self.probs = params(total_count, probs)
        n, p = raw(self.total_count), raw(self.probs)
        if bool((n < 0).any()):
            raise ValueError("Every element of input parameter `total_count` should be grater than or equal to 0.")
        if bool(((p < 0) | (p > 1)).any()):
            raise ValueError("Every element of input parameter `probs` should be in [0, 1].")
        super().__init__(tuple(torch.broadcast_shapes(n.shape, p.shape)))

    @property
    def mean(self):
        return _wrap(raw(self.total_count) * raw(self.probs))

    @property
    def variance(self):
        n, p = raw(self.total_count), raw(self.probs)
        return _wrap(n * p * (1 - p))

    def sample(self, shape=()):
        with torch.no_grad():
            n, p = raw(self.total_count), raw(self.probs)
            full = tuple(check_shape(shape)) + self.batch_shape
            return _wrap(torch.binomial(n.to(p.dtype).expand(full).contiguous(), p.expand(full).contiguous()))

    def log_prob(self, value):
        v = value_like(self.probs, value)
        n, p = raw(self.total_count).to(v.dtype), raw(self.probs)
        comb = torch.lgamma(n + 1) - torch.lgamma(v + 1) - torch.lgamma(n - v + 1)
        return _wrap(comb + torch.xlogy(v, p) + torch.xlogy(n - v, 1 - p))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def _enumerate_support(self):
        n = raw(self.total_count)
        vals = torch.arange(int(n.max().item()) + 1, dtype=raw(self.probs).dtype, device=n.device)
        return vals.reshape((-1,) + (1,) * len(self.batch_shape))

    def entropy(self):
        n = raw(self.total_count)
        vals = self._enumerate_support()
        lp = raw(self.log_prob(_wrap(vals.expand((vals.shape[0],) + self.batch_shape))))
        valid = vals <= n
        return _wrap(-torch.where(valid, lp.exp() * lp, torch.zeros_like(lp)).sum(0))

    def kl_divergence(self, other):
        n1, n2 = raw(self.total_count), raw(other.total_count)
        if not torch.equal(n1.expand(torch.broadcast_shapes(n1.shape, n2.shape)),
                           n2.expand(torch.broadcast_shapes(n1.shape, n2.shape))):
            raise NotImplementedError("KL between Binomials with different total_count is not implemented")
        p, q = raw(self.probs), raw(other.probs)
        return _wrap(n1 * (torch.xlogy(p, p) - torch.xlogy(p, q) + torch.xlogy(1 - p, 1 - p)
                           - torch.xlogy(1 - p, 1 - q)))


# =============================================================================================== Categorical
class Categorical(Distribution):
    """Categorical over the last axis of ``logits``.  As in the reference: ``probs`` / ``log_prob`` use the
    normalized input (logits / sum), ``sample`` / ``entropy`` / ``kl_divergence`` treat it as logits."""

    def __init__(self, logits, name=None):
        self.name = name or "Categorical"
        (self.logits,) = params(logits) if not isinstance(logits, Tensor) else (logits,)
        lg = raw(self.logits)
        self.dtype = lg.dtype
        self._prob = _wrap(lg / lg.sum(-1, keepdim=True))
        super().__init__(tuple(lg.shape[:-1]))

    def sample(self, shape):
        with torch.no_grad():
            shape = check_shape(shape)
            n = 1
            for s in shape:
                n *= s
            lg = raw(self.logits)
            probs = torch.softmax(lg.reshape(-1, lg.shape[-1]), -1)
            idx = torch.multinomial(probs, n, replacement=True)          # [batch, n]
            idx = idx.transpose(0, 1).reshape(tuple(shape) + tuple(lg.shape[:-1]))
            return _wrap(idx.to(torch.int64))

    def kl_divergence(self, other):
        a = raw(self.logits) - raw(self.logits).amax(-1, keepdim=True)
        b = raw(other.logits) - raw(other.logits).amax(-1, keepdim=True)
        za, zb = a.exp().sum(-1, keepdim=True), b.exp().sum(-1, keepdim=True)
        pa = a.exp() / za
        return _wrap((pa * (a - za.log() - b + zb.log())).sum(-1, keepdim=True))

    def entropy(self):
        a = raw(self.logits) - raw(self.logits).amax(-1, keepdim=True)
        z = a.exp().sum(-1, keepdim=True)
        p = a.exp() / z
        return _wrap(-(p * (a - z.log())).sum(-1))

    def probs(self, value):
        v = raw(value).to(torch.int64)
        prob = raw(self._prob)
        if prob.dim() == 1:
            return _wrap(prob[v.reshape(-1)].reshape(v.shape))
        if v.dim() == 1:
            idx = v.reshape((1,) * (prob.dim() - 1) + (-1,)).expand(tuple(prob.shape[:-1]) + (v.shape[0],))
            return _wrap(torch.gather(prob, -1, idx))
        return _wrap(torch.gather(prob, -1, v))

    def log_prob(self, value):
        return _wrap(raw(self.probs(value)).log())

    def prob(self, value):
        return self.probs(value)


# =============================================================================================== Geometric
class Geometric(Distribution):
    """Number of failures before the first success: P(k) = (1-p)^k p, k = 0, 1, ..."""

    def __init__(self, probs):
        if isinstance(probs, numbers.Real):
            probs = float(probs)
        (self.probs,) = params(probs) if not isinstance(probs, Tensor) else (probs,)
        p = raw(self.probs)
        if bool(((p <= 0) | (p > 1)).any()):
            raise ValueError("Expected parameter probs of distribution Geometric to satisfy the constraint "
                             "Interval(lower_bound=0.0, upper_bound=1.0)")
        super().__init__(tuple(p.shape))

    @property
    def mean(self):
        return _wrap(1.0 / raw(self.probs) - 1.0)

    @property
    def variance(self):
        p = raw(self.probs)
        return _wrap((1.0 / p - 1.0) / p)

    @property
    def stddev(self):
        return _wrap(raw(self.variance).sqrt())

    def _k(self, k):
        if not isinstance(k, (numbers.Integral, Tensor)):
            raise TypeError(f"Expected type of k is number.Real|framework.Variable|Value, but got {type(k)}")
        return raw(k).to(raw(self.probs).dtype) if isinstance(k, Tensor) else float(k)

    def pmf(self, k):
        p = raw(self.probs)
        return _wrap(torch.pow(1.0 - p, self._k(k)) * p)

    def log_pmf(self, k):
        p = raw(self.probs)
        return _wrap(torch.log(torch.pow(1.0 - p, self._k(k)) * p))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        p = raw(self.probs)
        full = tuple(check_shape(shape)) + self.batch_shape
        u = torch.rand(full, dtype=p.dtype, device=p.device).clamp(torch.finfo(p.dtype).tiny, 1.0)
        return _wrap(torch.floor(u.log() / torch.log1p(-p)))

    def entropy(self):
        p = raw(self.probs)
        return _wrap(-((1.0 - p) * torch.log(1.0 - p) + p * p.log()) / p)

    def cdf(self, k):
        p = raw(self.probs)
        return _wrap(1.0 - torch.pow(1.0 - p, self._k(k) + 1))

    def kl_divergence(self, other):
        # the reference's closed form (the per-trial Bernoulli divergence), kept for numeric parity
        if not isinstance(other, Geometric):
            raise TypeError(f"Exacted type of other is geometric.Geometric, but got {type(other)}")
        p, q = raw(self.probs), raw(other.probs)
        return _wrap(p * (p / q).log() + (1.0 - p) * ((1.0 - p) / (1.0 - q)).log())


# =============================================================================================== Multinomial
class Multinomial(Distribution):
    def __init__(self, total_count, probs):
        if not isinstance(total_count, int) or total_count < 1:
            raise ValueError("input parameter total_count must be int type and grater than zero.")
        (p,) = params(probs) if not isinstance(probs, Tensor) else (probs,)
        pt = raw(p)
        if pt.dim() < 1:
            raise ValueError("probs parameter shoule not be none and over one dimension")
        self.probs = _wrap(pt / pt.sum(-1, keepdim=True))
        self.total_count = total_count
        self._categorical = Categorical(_wrap(pt.clamp_min(torch.finfo(pt.dtype).tiny).log()))
        super().__init__(tuple(pt.shape[:-1]), tuple(pt.shape[-1:]))

    @property
    def mean(self):
        return _wrap(raw(self.probs) * self.total_count)

    @property
    def variance(self):
        p = raw(self.probs)
        return _wrap(self.total_count * p * (1 - p))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def log_prob(self, value):
        v = value_like(self.probs, value)
        p = raw(self.probs)
        n = torch.as_tensor(float(self.total_count), dtype=p.dtype, device=p.device)
        return _wrap(torch.lgamma(n + 1) - torch.lgamma(v + 1).sum(-1) + torch.xlogy(v, p).sum(-1))

    def sample(self, shape=()):
        with torch.no_grad():
            shape = tuple(check_shape(shape))
            p = raw(self.probs)
            k = p.shape[-1]
            draws = torch.multinomial(p.reshape(-1, k), self.total_count * max(1, _numel(shape)), replacement=True)
            draws = draws.reshape(-1, max(1, _numel(shape)), self.total_count)           # [batch, S, n]
            counts = torch.zeros(draws.shape[:2] + (k,), dtype=p.dtype, device=p.device)
            counts.scatter_add_(-1, draws, torch.ones_like(draws, dtype=p.dtype))
            counts = counts.transpose(0, 1).reshape(shape + tuple(p.shape))
            return _wrap(counts)

    def entropy(self):
        p = raw(self.probs)
        n = self.total_count
        support = torch.arange(n + 1, dtype=p.dtype, device=p.device).reshape((-1,) + (1,) * p.dim())
        nn_ = torch.as_tensor(float(n), dtype=p.dtype, device=p.device)
        binom_lp = (torch.lgamma(nn_ + 1) - torch.lgamma(support + 1) - torch.lgamma(nn_ - support + 1)
                    + torch.xlogy(support, p) + torch.xlogy(nn_ - support, 1 - p))
        e_lgamma = (binom_lp.exp() * torch.lgamma(support + 1)).sum(0).sum(-1)
        return _wrap(-torch.lgamma(nn_ + 1) - n * torch.xlogy(p, p).sum(-1) + e_lgamma)


def _numel(shape):
    n = 1
    for s in shape:
        n *= int(s)
    return n


# =============================================================================================== Poisson
class Poisson(Distribution):
    def __init__(self, rate):
        (self.rate,) = params(rate) if not isinstance(rate, Tensor) else (rate,)
        r = raw(self.rate)
        if bool((r < 0).any()):
            raise ValueError("Every element of input parameter `rate` should be nonnegative.")
        super().__init__(tuple(r.shape))

    @property
    def mean(self):
        return self.rate

    @property
    def variance(self):
        return self.rate

    def sample(self, shape=()):
        with torch.no_grad():
            r = raw(self.rate)
            full = tuple(check_shape(shape)) + self.batch_shape
            return _wrap(torch.poisson(r.expand(full).contiguous()))

    def _enumerate_bounded_support(self):
        r = raw(self.rate)
        upper = int((r.max() + 30 * r.max().clamp_min(1).sqrt() + 10).ceil().item())
        return torch.arange(upper + 1, dtype=r.dtype, device=r.device).reshape((-1,) + (1,) * r.dim())

    def entropy(self):
        vals = self._enumerate_bounded_support()
        lp = raw(self.log_prob(_wrap(vals.expand((vals.shape[0],) + self.batch_shape))))
        return _wrap(-(lp.exp() * lp).nan_to_num(0.0).sum(0))

    def log_prob(self, value):
        v = value_like(self.rate, value)
        r = raw(self.rate)
        return _wrap(torch.xlogy(v, r) - r - torch.lgamma(v + 1))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def kl_divergence(self, other):
        a, b = raw(self.rate), raw(other.rate)
        return _wrap(torch.xlogy(a, a) - torch.xlogy(a, b) - a + b)
