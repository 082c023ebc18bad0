"""paddle.distribution (reference: python/paddle/distribution/): probability distributions with sampling,
(log-)densities, moments, entropy and KL divergence, bijective transforms and transformed distributions.

Module layout: ``distribution`` (base + parameter conversion), ``continuous`` / ``discrete`` (the families),
``exponential_family`` (Bregman entropy), ``transform`` / ``transformed_distribution`` / ``variable`` /
``constraint``, ``kl`` (registry)."""
from . import constraint, transform, variable  # noqa: F401
from .continuous import (Beta, Cauchy, Chi2, ContinuousBernoulli, Dirichlet, Exponential, Gamma, Gumbel,  # noqa: F401
                         Laplace, LKJCholesky, LogNormal, MultivariateNormal, Normal, StudentT, Uniform)
from .discrete import Bernoulli, Binomial, Categorical, Geometric, Multinomial, Poisson  # noqa: F401
from .distribution import Distribution  # noqa: F401
from .exponential_family import ExponentialFamily  # noqa: F401
from .kl import kl_divergence, register_kl  # noqa: F401
from .transform import (AbsTransform, AffineTransform, ChainTransform, ExpTransform,  # noqa: F401
                        IndependentTransform, PowerTransform, ReshapeTransform, SigmoidTransform, SoftmaxTransform,
                        StackTransform, StickBreakingTransform, TanhTransform, Transform)
from .transformed_distribution import Independent, TransformedDistribution  # noqa: F401

__all__ = ["Bernoulli", "Beta", "Binomial", "Categorical", "Cauchy", "Chi2", "ContinuousBernoulli", "Dirichlet",
           "Distribution", "Exponential", "ExponentialFamily", "Gamma", "Geometric", "Gumbel", "Independent",
           "LKJCholesky", "Laplace", "LogNormal", "Multinomial", "MultivariateNormal", "Normal", "Poisson",
           "StudentT", "TransformedDistribution", "Uniform", "kl_divergence", "register_kl", "AbsTransform",
           "AffineTransform", "ChainTransform", "ExpTransform", "IndependentTransform", "PowerTransform",
           "ReshapeTransform", "SigmoidTransform", "SoftmaxTransform", "StackTransform", "StickBreakingTransform",
           "TanhTransform", "Transform"]
