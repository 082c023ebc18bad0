"""Continuous distributions (reference: python/paddle/distribution/{normal,uniform,laplace,cauchy,exponential,
gamma,chi2,beta,dirichlet,student_t,continuous_bernoulli,gumbel,lognormal,multivariate_normal,lkj_cholesky}.py).

Closed forms are evaluated on the parameters' torch storage (autograd flows to Tensor parameters); sampling
draws from the framework's seeded generator (``paddle.seed``)."""
from __future__ import annotations

import math

import numpy as np
import torch

from .distribution import EULER, LOG_2PI, Distribution, _wrap, check_shape, params, raw, value_like
from .exponential_family import ExponentialFamily
from .transform import ExpTransform
from .transformed_distribution import TransformedDistribution


def _shape_of(*ts):
    return tuple(torch.broadcast_shapes(*[tuple(raw(t).shape) for t in ts]))


def _uniform(shape, like, low=0.0, high=1.0):
    return torch.rand(shape, dtype=like.dtype, device=like.device) * (high - low) + low


def _tiny(dtype):
    return torch.finfo(dtype).tiny


def _eps(dtype):
    return torch.finfo(dtype).eps


# =============================================================================================== Normal
class Normal(Distribution):
    """N(loc, scale^2); complex ``loc`` gives the circular complex Gaussian."""

    def __init__(self, loc, scale, name=None):
        self.name = name or "Normal"
        self.all_arg_is_float = isinstance(loc, (int, float, complex)) and isinstance(scale, (int, float))
        if isinstance(loc, complex) or (isinstance(loc, np.ndarray) and np.iscomplexobj(loc)):
            a = np.asarray(loc)
            loc = _wrap(torch.as_tensor(a.astype(np.complex64 if a.dtype != np.complex128 else a.dtype)))
        if isinstance(loc, (int, float)):
            loc = float(loc)
        if isinstance(scale, (int, float)):
            scale = float(scale)
        if hasattr(loc, "_t") and raw(loc).is_complex():
            self._complex_gaussian = True
            self.loc = loc
            self.scale = scale if hasattr(scale, "_t") else _wrap(torch.as_tensor(np.asarray(scale, np.float32)))
        else:
            self._complex_gaussian = False
            self.loc, self.scale = params(loc, scale)
        self.dtype = raw(self.loc).dtype
        super().__init__(_shape_of(self.loc, self.scale) if not self.all_arg_is_float else ())

    @property
    def mean(self):
        return self.loc

    @property
    def variance(self):
        return _wrap(raw(self.scale).pow(2))

    def sample(self, shape=(), seed=0):
        with torch.no_grad():
            out = self._draw(check_shape(shape))
        return _wrap(out)

    def rsample(self, shape=()):
        return _wrap(self._draw(check_shape(shape)))

    def _draw(self, shape):
        loc, scale = raw(self.loc), raw(self.scale)
        full = tuple(shape) + _shape_of(loc, scale)
        eps = torch.randn(full, dtype=loc.dtype, device=loc.device)
        return loc + eps * scale

    def entropy(self):
        s = raw(self.scale) + torch.zeros_like(raw(self.loc).real if self._complex_gaussian else raw(self.loc))
        if self._complex_gaussian:
            return _wrap(1.0 + math.log(math.pi) + 2.0 * s.log())
        return _wrap(0.5 + 0.5 * LOG_2PI + s.log())

    def log_prob(self, value):
        v = value_like(self.loc, value)
        loc, scale = raw(self.loc), raw(self.scale)
        d = v - loc
        if self._complex_gaussian:
            return _wrap((-(d.conj() * d) / (scale * scale)).real - 2.0 * scale.log() - math.log(math.pi))
        return _wrap(-(d * d) / (2.0 * scale * scale) - scale.log() - 0.5 * LOG_2PI)

    def probs(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    prob = probs

    def cdf(self, value):
        v = value_like(self.loc, value)
        return _wrap(0.5 * (1 + torch.erf((v - raw(self.loc)) / (raw(self.scale) * math.sqrt(2)))))

    def icdf(self, value):
        v = value_like(self.loc, value)
        return _wrap(raw(self.loc) + raw(self.scale) * torch.erfinv(2 * v - 1) * math.sqrt(2))

    def kl_divergence(self, other):
        if self._complex_gaussian != other._complex_gaussian:
            raise ValueError("The kl divergence must be computed between two distributions in the same number "
                             "field.")
        ratio = (raw(self.scale) / raw(other.scale)) ** 2
        t1 = (raw(self.loc) - raw(other.loc)) / raw(other.scale)
        if self._complex_gaussian:
            return _wrap(ratio + (t1.conj() * t1).real - 1.0 - ratio.log())
        return _wrap(0.5 * ratio + 0.5 * (t1 * t1 - 1.0 - ratio.log()))


# =============================================================================================== Uniform
class Uniform(Distribution):
    """U[low, high)."""

    def __init__(self, low, high, name=None):
        self.name = name or "Uniform"
        self.all_arg_is_float = isinstance(low, (int, float)) and isinstance(high, (int, float))
        self.low, self.high = params(float(low) if isinstance(low, int) else low,
                                     float(high) if isinstance(high, int) else high)
        self.dtype = raw(self.low).dtype
        super().__init__(_shape_of(self.low, self.high) if not self.all_arg_is_float else ())

    @property
    def mean(self):
        return _wrap((raw(self.low) + raw(self.high)) / 2)

    @property
    def variance(self):
        return _wrap((raw(self.high) - raw(self.low)) ** 2 / 12)

    def sample(self, shape=(), seed=0):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        lo, hi = raw(self.low), raw(self.high)
        full = tuple(check_shape(shape)) + _shape_of(lo, hi)
        return _wrap(lo + _uniform(full, lo) * (hi - lo))

    def log_prob(self, value):
        v = value_like(self.low, value)
        lo, hi = raw(self.low), raw(self.high)
        inside = ((lo < v) & (v < hi)).to(v.dtype)
        return _wrap(inside.log() - (hi - lo).log())

    def probs(self, value):
        v = value_like(self.low, value)
        lo, hi = raw(self.low), raw(self.high)
        inside = ((lo < v) & (v < hi)).to(v.dtype)
        return _wrap(inside / (hi - lo))

    prob = probs

    def cdf(self, value):
        v = value_like(self.low, value)
        lo, hi = raw(self.low), raw(self.high)
        return _wrap(((v - lo) / (hi - lo)).clamp(0, 1))

    def entropy(self):
        return _wrap((raw(self.high) - raw(self.low)).log())


# =============================================================================================== Laplace
class Laplace(Distribution):
    def __init__(self, loc, scale):
        self.loc, self.scale = params(loc, scale)
        super().__init__(_shape_of(self.loc, self.scale))

    @property
    def mean(self):
        return self.loc

    @property
    def stddev(self):
        return _wrap(math.sqrt(2) * raw(self.scale))

    @property
    def variance(self):
        return _wrap(2 * raw(self.scale) ** 2)

    def log_prob(self, value):
        v = value_like(self.loc, value)
        s = raw(self.scale)
        return _wrap(-(2 * s).log() - (v - raw(self.loc)).abs() / s)

    def entropy(self):
        return _wrap(1 + (2 * raw(self.scale)).log())

    def cdf(self, value):
        v = value_like(self.loc, value)
        z = v - raw(self.loc)
        return _wrap(0.5 - 0.5 * z.sign() * torch.expm1(-z.abs() / raw(self.scale)))

    def icdf(self, value):
        v = value_like(self.loc, value)
        t = v - 0.5
        return _wrap(raw(self.loc) - raw(self.scale) * t.sign() * torch.log1p(-2 * t.abs()))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape):
        loc, s = raw(self.loc), raw(self.scale)
        full = tuple(check_shape(shape)) + self.batch_shape
        u = _uniform(full, loc, -1 + _eps(loc.dtype), 1.0)
        return _wrap(loc - s * u.sign() * torch.log1p(-u.abs()))

    def kl_divergence(self, other):
        d = (raw(self.loc) - raw(other.loc)).abs()
        s1, s2 = raw(self.scale), raw(other.scale)
        return _wrap((s2 / s1).log() + d / s2 + s1 / s2 * torch.exp(-d / s1) - 1)


# =============================================================================================== Cauchy
class Cauchy(Distribution):
    def __init__(self, loc, scale, name=None):
        self.name = name or "Cauchy"
        self.loc, self.scale = params(loc, scale)
        super().__init__(_shape_of(self.loc, self.scale))

    @property
    def mean(self):
        raise ValueError("Cauchy distribution has no mean.")

    @property
    def variance(self):
        raise ValueError("Cauchy distribution has no variance.")

    @property
    def stddev(self):
        raise ValueError("Cauchy distribution has no stddev.")

    def sample(self, shape, name=None):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape, name=None):
        loc, s = raw(self.loc), raw(self.scale)
        full = tuple(check_shape(shape)) + self.batch_shape
        u = _uniform(full, loc)
        return _wrap(loc + s * torch.tan(math.pi * (u - 0.5)))

    def log_prob(self, value):
        v = value_like(self.loc, value)
        s = raw(self.scale)
        return _wrap(-math.log(math.pi) - s.log() - torch.log1p(((v - raw(self.loc)) / s) ** 2))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def cdf(self, value):
        v = value_like(self.loc, value)
        return _wrap(torch.atan((v - raw(self.loc)) / raw(self.scale)) / math.pi + 0.5)

    def entropy(self):
        return _wrap((4 * math.pi * raw(self.scale)).log())

    def kl_divergence(self, other):
        s1, s2 = raw(self.scale), raw(other.scale)
        d = raw(self.loc) - raw(other.loc)
        return _wrap((((s1 + s2) ** 2 + d ** 2) / (4 * s1 * s2)).log())


# =============================================================================================== Exponential
class Exponential(ExponentialFamily):
    def __init__(self, rate):
        (self.rate,) = params(rate)
        super().__init__(tuple(raw(self.rate).shape))

    @property
    def mean(self):
        return _wrap(raw(self.rate).reciprocal())

    @property
    def variance(self):
        return _wrap(raw(self.rate).pow(-2))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        r = raw(self.rate)
        full = tuple(check_shape(shape)) + self.batch_shape
        u = _uniform(full, r, _tiny(r.dtype), 1.0)
        return _wrap(-u.log() / r)

    def prob(self, value):
        v = value_like(self.rate, value)
        r = raw(self.rate)
        return _wrap(r * torch.exp(-r * v))

    def log_prob(self, value):
        v = value_like(self.rate, value)
        r = raw(self.rate)
        return _wrap(r.log() - r * v)

    def entropy(self):
        return _wrap(1.0 - raw(self.rate).log())

    def cdf(self, value):
        v = value_like(self.rate, value)
        return _wrap(1 - torch.exp(-raw(self.rate) * v))

    def icdf(self, value):
        v = value_like(self.rate, value)
        return _wrap(-torch.log1p(-v) / raw(self.rate))

    def kl_divergence(self, other):
        r = raw(self.rate) / raw(other.rate)
        return _wrap(r.log() + 1 / r - 1)

    def _natural_parameters(self):
        return (-raw(self.rate),)

    def _log_normalizer(self, x):
        return -torch.log(-x)


# =============================================================================================== Gamma / Chi2
class Gamma(ExponentialFamily):
    def __init__(self, concentration, rate):
        self.concentration, self.rate = params(concentration, rate)
        super().__init__(_shape_of(self.concentration, self.rate))

    @property
    def mean(self):
        return _wrap(raw(self.concentration) / raw(self.rate))

    @property
    def variance(self):
        return _wrap(raw(self.concentration) / raw(self.rate).pow(2))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def log_prob(self, value):
        v = value_like(self.concentration, value)
        c, r = raw(self.concentration), raw(self.rate)
        return _wrap(torch.xlogy(c, r) + torch.xlogy(c - 1, v) - r * v - torch.lgamma(c))

    def entropy(self):
        c, r = raw(self.concentration), raw(self.rate)
        return _wrap(c - r.log() + torch.lgamma(c) + (1.0 - c) * torch.digamma(c))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        c, r = raw(self.concentration), raw(self.rate)
        full = tuple(check_shape(shape)) + self.batch_shape
        g = torch._standard_gamma(c.expand(full).contiguous())
        return _wrap(g.clamp_min(_tiny(g.dtype)) / r)

    def kl_divergence(self, other):
        c1, r1 = raw(self.concentration), raw(self.rate)
        c2, r2 = raw(other.concentration), raw(other.rate)
        return _wrap((c1 - c2) * torch.digamma(c1) - torch.lgamma(c1) + torch.lgamma(c2)
                     + c2 * (r1.log() - r2.log()) + c1 * (r2 - r1) / r1)

    def _natural_parameters(self):
        return (raw(self.concentration) - 1, -raw(self.rate))

    def _log_normalizer(self, x, y):
        return torch.lgamma(x + 1) + (x + 1) * torch.log(-y.reciprocal())


class Chi2(Gamma):
    def __init__(self, df):
        (self.df,) = params(df)
        super().__init__(_wrap(0.5 * raw(self.df)), _wrap(torch.full_like(raw(self.df), 0.5)))


# =============================================================================================== Beta / Dirichlet
class Beta(ExponentialFamily):
    def __init__(self, alpha, beta):
        self.alpha, self.beta = params(alpha, beta)
        super().__init__(_shape_of(self.alpha, self.beta))

    @property
    def mean(self):
        a, b = raw(self.alpha), raw(self.beta)
        return _wrap(a / (a + b))

    @property
    def variance(self):
        a, b = raw(self.alpha), raw(self.beta)
        s = a + b
        return _wrap(a * b / (s.pow(2) * (s + 1)))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def log_prob(self, value):
        v = value_like(self.alpha, value)
        a, b = raw(self.alpha), raw(self.beta)
        return _wrap(torch.xlogy(a - 1, v) + torch.xlogy(b - 1, 1 - v) - _lbeta(a, b))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        a, b = raw(self.alpha), raw(self.beta)
        full = tuple(check_shape(shape)) + self.batch_shape
        x = torch._standard_gamma(a.expand(full).contiguous())
        y = torch._standard_gamma(b.expand(full).contiguous())
        return _wrap(x / (x + y))

    def entropy(self):
        a, b = raw(self.alpha), raw(self.beta)
        return _wrap(_lbeta(a, b) - (a - 1) * torch.digamma(a) - (b - 1) * torch.digamma(b)
                     + (a + b - 2) * torch.digamma(a + b))

    def _natural_parameters(self):
        return (raw(self.alpha), raw(self.beta))

    def _log_normalizer(self, x, y):
        return torch.lgamma(x) + torch.lgamma(y) - torch.lgamma(x + y)


def _lbeta(a, b):
    return torch.lgamma(a) + torch.lgamma(b) - torch.lgamma(a + b)


class Dirichlet(ExponentialFamily):
    def __init__(self, concentration):
        if hasattr(concentration, "_t"):
            self.concentration = concentration
        else:
            (self.concentration,) = params(concentration)
        c = raw(self.concentration)
        if c.dim() < 1:
            raise ValueError("`concentration` parameter must be at least one dimensional")
        super().__init__(tuple(c.shape[:-1]), tuple(c.shape[-1:]))

    @property
    def mean(self):
        c = raw(self.concentration)
        return _wrap(c / c.sum(-1, keepdim=True))

    @property
    def variance(self):
        c = raw(self.concentration)
        s = c.sum(-1, keepdim=True)
        return _wrap(c * (s - c) / (s.pow(2) * (s + 1)))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        c = raw(self.concentration)
        full = tuple(check_shape(shape)) + tuple(c.shape)
        g = torch._standard_gamma(c.expand(full).contiguous()).clamp_min(_tiny(c.dtype))
        return _wrap(g / g.sum(-1, keepdim=True))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def log_prob(self, value):
        v = value_like(self.concentration, value)
        c = raw(self.concentration)
        return _wrap(torch.xlogy(c - 1, v).sum(-1) + torch.lgamma(c.sum(-1)) - torch.lgamma(c).sum(-1))

    def entropy(self):
        c = raw(self.concentration)
        k = c.shape[-1]
        s = c.sum(-1)
        return _wrap(torch.lgamma(c).sum(-1) - torch.lgamma(s) - (k - s) * torch.digamma(s)
                     - ((c - 1.0) * torch.digamma(c)).sum(-1))

    def _natural_parameters(self):
        return (raw(self.concentration),)

    def _log_normalizer(self, x):
        return torch.lgamma(x).sum(-1) - torch.lgamma(x.sum(-1))


# =============================================================================================== StudentT
class StudentT(Distribution):
    def __init__(self, df, loc, scale, name=None):
        self.name = name or "StudentT"
        self.df, self.loc, self.scale = params(df, loc, scale)
        if bool((raw(self.df) <= 0).any()):
            raise ValueError("Every element of input parameter `df` should be nonnegative.")
        if bool((raw(self.scale) <= 0).any()):
            raise ValueError("Every element of input parameter `scale` should be nonnegative.")
        self._chi2 = Chi2(self.df)
        super().__init__(_shape_of(self.df, self.loc, self.scale))

    @property
    def mean(self):
        df, loc = raw(self.df), raw(self.loc)
        return _wrap(torch.where(df > 1.0, loc.expand(self.batch_shape),
                                 torch.full(self.batch_shape, float("nan"), dtype=loc.dtype, device=loc.device)))

    @property
    def variance(self):
        df, s = raw(self.df), raw(self.scale)
        shape = self.batch_shape
        var = torch.where(df > 2.0, (s.pow(2) * df / (df - 2.0)).expand(shape),
                          torch.full(shape, float("nan"), dtype=s.dtype, device=s.device))
        return _wrap(torch.where((df <= 2.0) & (df > 1.0), torch.full(shape, float("inf"), dtype=s.dtype,
                                                                         device=s.device), var))

    def sample(self, shape=()):
        with torch.no_grad():
            df, loc, s = raw(self.df), raw(self.loc), raw(self.scale)
            full = tuple(check_shape(shape)) + self.batch_shape
            z = torch.randn(full, dtype=loc.dtype, device=loc.device)
            chi2 = raw(self._chi2.sample(check_shape(shape))).expand(full)
            return _wrap(loc + s * z * torch.rsqrt(chi2 / df))

    def entropy(self):
        df, s = raw(self.df), raw(self.scale)
        lbeta = torch.lgamma(0.5 * df) + math.lgamma(0.5) - torch.lgamma(0.5 * (df + 1))
        return _wrap(s.log() + 0.5 * (df + 1) * (torch.digamma(0.5 * (df + 1)) - torch.digamma(0.5 * df))
                     + 0.5 * df.log() + lbeta)

    def log_prob(self, value):
        v = value_like(self.loc, value)
        df, loc, s = raw(self.df), raw(self.loc), raw(self.scale)
        y = (v - loc) / s
        z = s.log() + 0.5 * df.log() + 0.5 * math.log(math.pi) + torch.lgamma(0.5 * df) - torch.lgamma(0.5 * (df + 1))
        return _wrap(-0.5 * (df + 1.0) * torch.log1p(y * y / df) - z)

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())


# =============================================================================================== ContinuousBernoulli
class ContinuousBernoulli(Distribution):
    """CB(probs) on [0, 1]; the normalizer is Taylor-expanded inside ``lims`` around 0.5."""

    def __init__(self, probs, lims=(0.499, 0.501)):
        (p,) = params(probs)
        pt = raw(p)
        eps = _eps(pt.dtype)
        self.probs = _wrap(pt.clamp(eps, 1 - eps))
        self.lims = _wrap(torch.as_tensor(lims, dtype=pt.dtype))
        super().__init__(tuple(pt.shape))

    def _outside(self):
        p = raw(self.probs)
        lo, hi = raw(self.lims)[0], raw(self.lims)[1]
        return (p < lo) | (p > hi)

    def _cut_probs(self):
        p = raw(self.probs)
        return torch.where(self._outside(), p, raw(self.lims)[0] * torch.ones_like(p))

    def _tanh_inverse(self, value):
        return 0.5 * (torch.log1p(value) - torch.log1p(-value))

    def _log_constant(self):
        p = raw(self.probs)
        cut = self._cut_probs()
        cut_below = torch.where(cut <= 0.5, cut, torch.zeros_like(cut))
        cut_above = torch.where(cut >= 0.5, cut, torch.ones_like(cut))
        log_norm = (torch.abs(torch.log1p(-cut) - cut.log())).log() - torch.where(
            cut <= 0.5, torch.log1p(-2.0 * cut_below), torch.log(2.0 * cut_above - 1.0))
        x = (p - 0.5) ** 2
        taylor = math.log(2.0) + (4.0 / 3.0 + 104.0 / 45.0 * x) * x
        return torch.where(self._outside(), log_norm, taylor)

    @property
    def mean(self):
        p = raw(self.probs)
        cut = self._cut_probs()
        mus = cut / (2.0 * cut - 1.0) + 1.0 / (torch.log1p(-cut) - cut.log())
        x = p - 0.5
        taylor = 0.5 + (1.0 / 3.0 + 16.0 / 45.0 * x.pow(2)) * x
        return _wrap(torch.where(self._outside(), mus, taylor))

    @property
    def variance(self):
        p = raw(self.probs)
        cut = self._cut_probs()
        vars_ = cut * (cut - 1.0) / (1.0 - 2.0 * cut).pow(2) + 1.0 / (torch.log1p(-cut) - cut.log()).pow(2)
        x = (p - 0.5).pow(2)
        taylor = 1.0 / 12.0 - (1.0 / 15.0 - 128.0 / 945.0 * x) * x
        return _wrap(torch.where(self._outside(), vars_, taylor))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        p = raw(self.probs)
        full = tuple(check_shape(shape)) + self.batch_shape
        u = _uniform(full, p)
        return self.icdf(_wrap(u))

    def log_prob(self, value):
        v = value_like(self.probs, value)
        p = raw(self.probs)
        return _wrap(torch.xlogy(v, p) + torch.xlogy(1 - v, 1 - p) + self._log_constant())

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def entropy(self):
        p = raw(self.probs)
        lp0, lp1 = torch.log1p(-p), p.log()
        return _wrap(raw(self.mean) * (lp0 - lp1) - self._log_constant() - lp0)

    def cdf(self, value):
        v = value_like(self.probs, value)
        cut = self._cut_probs()
        cdfs = (cut.pow(v) * (1.0 - cut).pow(1.0 - v) + cut - 1.0) / (2.0 * cut - 1.0)
        unb = torch.where(self._outside(), cdfs, v)
        return _wrap(torch.where(v <= 0.0, torch.zeros_like(unb), torch.where(v >= 1.0, torch.ones_like(unb), unb)))

    def icdf(self, value):
        v = value_like(self.probs, value)
        cut = self._cut_probs()
        out = (torch.log1p(-cut + v * (2.0 * cut - 1.0)) - torch.log1p(-cut)) / (cut.log() - torch.log1p(-cut))
        return _wrap(torch.where(self._outside(), out, v))

    def kl_divergence(self, other):
        q = raw(other.probs)
        return _wrap(-raw(self.entropy()) - raw(self.mean) * (q.log() - torch.log1p(-q)) - torch.log1p(-q)
                     - other._log_constant())


# =============================================================================================== Gumbel / LogNormal
class Gumbel(TransformedDistribution):
    """Gumbel(loc, scale): loc - scale * log(-log U)."""

    def __init__(self, loc, scale):
        self.loc, self.scale = params(loc, scale)
        if bool((raw(self.scale) <= 0).any()):
            raise ValueError("scale must be positive")
        from .transform import AffineTransform

        self._base_u = Uniform(_wrap(torch.full_like(raw(self.loc), _tiny(raw(self.loc).dtype))),
                               _wrap(torch.ones_like(raw(self.loc)) - _eps(raw(self.loc).dtype)))
        super().__init__(self._base_u, [AffineTransform(_wrap(torch.zeros_like(raw(self.loc))),
                                                        _wrap(torch.ones_like(raw(self.loc))))])
        self._batch_shape = _shape_of(self.loc, self.scale)
        self._event_shape = ()

    @property
    def mean(self):
        return _wrap(raw(self.loc) + raw(self.scale) * EULER)

    @property
    def variance(self):
        return _wrap(raw(self.scale).pow(2) * math.pi ** 2 / 6)

    @property
    def stddev(self):
        return _wrap(raw(self.variance).sqrt())

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def log_prob(self, value):
        v = value_like(self.loc, value)
        z = (raw(self.loc) - v) / raw(self.scale)
        return _wrap(z - z.exp() - raw(self.scale).log())

    def cdf(self, value):
        v = value_like(self.loc, value)
        return _wrap(torch.exp(-torch.exp(-(v - raw(self.loc)) / raw(self.scale))))

    def entropy(self):
        return _wrap(raw(self.scale).log() + 1 + EULER)

    def sample(self, shape):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape):
        loc = raw(self.loc)
        full = tuple(check_shape(shape)) + self.batch_shape
        u = _uniform(full, loc, _tiny(loc.dtype), 1.0 - _eps(loc.dtype))
        return _wrap(loc - raw(self.scale) * torch.log(-u.log()))


class LogNormal(TransformedDistribution):
    def __init__(self, loc, scale):
        self._base = Normal(loc=loc, scale=scale)
        self.loc, self.scale = self._base.loc, self._base.scale
        super().__init__(self._base, [ExpTransform()])

    @property
    def mean(self):
        return _wrap(torch.exp(raw(self.loc) + raw(self.scale).pow(2) / 2))

    @property
    def variance(self):
        l, s = raw(self.loc), raw(self.scale)  # noqa: E741
        return _wrap(torch.expm1(s.pow(2)) * torch.exp(2 * l + s.pow(2)))

    def entropy(self):
        return _wrap(raw(self._base.entropy()) + raw(self.loc))

    def probs(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    prob = probs

    def kl_divergence(self, other):
        return self._base.kl_divergence(other._base)


# =============================================================================================== MultivariateNormal
class MultivariateNormal(Distribution):
    """N(loc, Sigma) with Sigma given as covariance, precision or lower Cholesky factor."""

    def __init__(self, loc, covariance_matrix=None, precision_matrix=None, scale_tril=None):
        given = [m is not None for m in (covariance_matrix, precision_matrix, scale_tril)]
        if sum(given) != 1:
            raise ValueError("Exactly one of covariance_matrix or precision_matrix or scale_tril may be specified.")
        (self.loc,) = params(loc) if not hasattr(loc, "_t") else (loc,)
        mu = raw(self.loc)
        if mu.dim() < 1:
            raise ValueError("loc must be at least one-dimensional.")
        if scale_tril is not None:
            L = raw(scale_tril)
            if L.dim() < 2:
                raise ValueError("scale_tril matrix must be at least two-dimensional, with optional leading batch "
                                 "dimensions")
        elif covariance_matrix is not None:
            C = raw(covariance_matrix)
            if C.dim() < 2:
                raise ValueError("covariance_matrix must be at least two-dimensional, with optional leading batch "
                                 "dimensions")
            L = torch.linalg.cholesky(C)
        else:
            P = raw(precision_matrix)
            if P.dim() < 2:
                raise ValueError("precision_matrix must be at least two-dimensional, with optional leading batch "
                                 "dimensions")
            L = _precision_to_scale_tril(P)
        batch = torch.broadcast_shapes(tuple(L.shape[:-2]), tuple(mu.shape[:-1]))
        self._L = L.expand(tuple(batch) + tuple(L.shape[-2:]))
        self.scale_tril = _wrap(self._L)
        self.covariance_matrix = _wrap(self._L @ self._L.transpose(-1, -2))
        self.precision_matrix = _wrap(torch.cholesky_inverse(self._L) if self._L.dim() == 2 else
                                      torch.linalg.inv(self._L @ self._L.transpose(-1, -2)))
        self._mu = mu.expand(tuple(batch) + tuple(mu.shape[-1:]))
        super().__init__(tuple(batch), tuple(mu.shape[-1:]))

    @property
    def mean(self):
        return _wrap(self._mu)

    @property
    def variance(self):
        return _wrap(self._L.pow(2).sum(-1).expand(self.batch_shape + self.event_shape))

    def sample(self, shape=()):
        with torch.no_grad():
            return self.rsample(shape)

    def rsample(self, shape=()):
        full = tuple(check_shape(shape)) + self.batch_shape + self.event_shape
        eps = torch.randn(full, dtype=self._mu.dtype, device=self._mu.device)
        return _wrap(self._mu + (self._L @ eps.unsqueeze(-1)).squeeze(-1))

    def log_prob(self, value):
        v = value_like(self.loc, value)
        diff = v - self._mu
        m = _batch_mahalanobis(self._L, diff)
        half_log_det = self._L.diagonal(dim1=-2, dim2=-1).log().sum(-1)
        return _wrap(-0.5 * (self.event_shape[0] * LOG_2PI + m) - half_log_det)

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def entropy(self):
        half_log_det = self._L.diagonal(dim1=-2, dim2=-1).log().sum(-1)
        h = 0.5 * self.event_shape[0] * (1.0 + LOG_2PI) + half_log_det
        return _wrap(h.expand(self.batch_shape) if self.batch_shape else h)

    def kl_divergence(self, other):
        if self.event_shape != other.event_shape:
            raise ValueError("KL-divergence between two Multivariate Normals with different event shapes cannot "
                             "be computed")
        L1, L2 = self._L, other._L
        hld1 = L1.diagonal(dim1=-2, dim2=-1).log().sum(-1)
        hld2 = L2.diagonal(dim1=-2, dim2=-1).log().sum(-1)
        n = self.event_shape[0]
        # tr(S2^-1 S1) = ||L2^-1 L1||_F^2
        M = torch.linalg.solve_triangular(L2, L1.expand(torch.broadcast_shapes(L1.shape, L2.shape)), upper=False)
        tr = M.pow(2).sum((-2, -1))
        maha = _batch_mahalanobis(L2, other._mu - self._mu)
        return _wrap(hld2 - hld1 + 0.5 * (tr + maha - n))


def _precision_to_scale_tril(P):
    Lf = torch.linalg.cholesky(torch.flip(P, (-2, -1)))
    L_inv = torch.transpose(torch.flip(Lf, (-2, -1)), -2, -1)
    Id = torch.eye(P.shape[-1], dtype=P.dtype, device=P.device)
    return torch.linalg.solve_triangular(L_inv, Id, upper=False)


def _batch_mahalanobis(L, x):
    """x^T (L L^T)^-1 x over broadcast batches."""
    shape = torch.broadcast_shapes(L.shape[:-2], x.shape[:-1])
    Lb = L.expand(tuple(shape) + tuple(L.shape[-2:]))
    xb = x.expand(tuple(shape) + tuple(x.shape[-1:]))
    sol = torch.linalg.solve_triangular(Lb, xb.unsqueeze(-1), upper=False).squeeze(-1)
    return sol.pow(2).sum(-1)


precision_to_scale_tril = _precision_to_scale_tril
batch_mahalanobis = _batch_mahalanobis


# =============================================================================================== LKJCholesky
def mvlgamma(a, p):
    """Multivariate log-gamma: log Gamma_p(a)."""
    a = raw(a)
    j = torch.arange(p, dtype=a.dtype, device=a.device)
    return p * (p - 1) / 4 * math.log(math.pi) + torch.lgamma(a.unsqueeze(-1) - j / 2).sum(-1)


class LKJCholesky(Distribution):
    """Cholesky factors of LKJ(eta)-distributed correlation matrices; ``onion`` or ``cvine`` sampling."""

    def __init__(self, dim=2, concentration=1.0, sample_method="onion"):
        if not isinstance(dim, int) or dim < 2:
            raise ValueError(f"Expected dim to be an integer greater than or equal to 2. Found dim={dim}.")
        if sample_method not in ("onion", "cvine"):
            raise ValueError("`method` should be one of 'cvine' or 'onion'.")
        self.dim = dim
        self.sample_method = sample_method
        (self.concentration,) = params(concentration) if not hasattr(concentration, "_t") else (concentration,)
        c = raw(self.concentration)
        super().__init__(tuple(c.shape), (dim, dim))

    def _beta_sample(self, a, b, shape):
        x = torch._standard_gamma(a.expand(shape).contiguous())
        y = torch._standard_gamma(b.expand(shape).contiguous())
        return x / (x + y)

    def _onion(self, sample_shape):
        c = raw(self.concentration)
        D = self.dim
        off = torch.arange(D - 1, dtype=c.dtype, device=c.device)
        conc1 = off + 0.5
        conc0 = c.unsqueeze(-1) + 0.5 * (D - 2) - 0.5 * off
        shp = tuple(sample_shape) + tuple(c.shape) + (D - 1,)
        y = self._beta_sample(conc1.expand(shp), conc0.expand(shp), shp).unsqueeze(-1)   # [..., D-1, 1]
        u = torch.randn(tuple(sample_shape) + tuple(c.shape) + (D - 1, D - 1), dtype=c.dtype, device=c.device)
        u = torch.tril(u, diagonal=0)   # row k (0-based within the D-1 rows) keeps k+1 entries
        u = u / u.norm(dim=-1, keepdim=True).clamp_min(_tiny(c.dtype))
        w = y.clamp_min(0).sqrt() * u
        eps = _tiny(c.dtype)
        diag = (1 - w.pow(2).sum(-1)).clamp_min(eps).sqrt()
        L = torch.zeros(tuple(sample_shape) + tuple(c.shape) + (D, D), dtype=c.dtype, device=c.device)
        L[..., 1:, :-1] = w
        L = L + torch.diag_embed(torch.cat([torch.ones_like(diag[..., :1]), diag], -1))
        return L

    def _cvine(self, sample_shape):
        c = raw(self.concentration)
        D = self.dim
        shp = tuple(sample_shape) + tuple(c.shape)
        # partial correlations of row i (0-based) ~ 2 Beta(b_i, b_i) - 1 with b_i = eta + (D - 2 - i) / 2
        i = torch.arange(D - 1, dtype=c.dtype, device=c.device)
        beta = (c.unsqueeze(-1) + 0.5 * (D - 2) - 0.5 * i).unsqueeze(-1).expand(tuple(c.shape) + (D - 1, D))
        z = 2 * self._beta_sample(beta.expand(shp + (D - 1, D)), beta.expand(shp + (D - 1, D)),
                                  shp + (D - 1, D)) - 1      # z[..., i, j] used for j > i
        L = torch.zeros(shp + (D, D), dtype=c.dtype, device=c.device)
        L[..., 0, 0] = 1.0
        for j in range(1, D):
            rem = torch.ones(shp, dtype=c.dtype, device=c.device)
            for k in range(j):
                L[..., j, k] = z[..., k, j] * rem.sqrt()
                rem = rem - L[..., j, k].pow(2)
            L[..., j, j] = rem.clamp_min(0).sqrt()
        return L

    def sample(self, sample_shape=()):
        with torch.no_grad():
            ss = tuple(check_shape(sample_shape))
            return _wrap(self._onion(ss) if self.sample_method == "onion" else self._cvine(ss))

    def log_prob(self, value):
        L = raw(value)
        c = raw(self.concentration)
        D = self.dim
        diag = L.diagonal(dim1=-2, dim2=-1)[..., 1:]
        order = torch.arange(2, D + 1, dtype=c.dtype, device=c.device)
        order = 2 * (c - 1).unsqueeze(-1) + D - order
        unnorm = (order * diag.log()).sum(-1)
        dm1 = D - 1
        alpha = c + 0.5 * dm1
        denom = torch.lgamma(alpha) * dm1
        numer = mvlgamma(alpha - 0.5, dm1)
        norm = 0.5 * dm1 * math.log(math.pi) + numer - denom
        return _wrap(unnorm - norm)
