"""TransformedDistribution and Independent (reference: python/paddle/distribution/transformed_distribution.py,
independent.py)."""
from __future__ import annotations

from .distribution import Distribution, _wrap, raw, sum_rightmost


class Independent(Distribution):
    """Reinterpret the rightmost ``reinterpreted_batch_rank`` batch axes of ``base`` as event axes."""

    def __init__(self, base, reinterpreted_batch_rank):
        if not isinstance(base, Distribution):
            raise TypeError(f"Expected type of 'base' is Distribution, but got {type(base)}")
        if not (0 < reinterpreted_batch_rank <= len(base.batch_shape)):
            raise ValueError(f"Expected 0 < reinterpreted_batch_rank <= {len(base.batch_shape)}, but got "
                             f"{reinterpreted_batch_rank}")
        self._base = base
        self._reinterpreted_batch_rank = reinterpreted_batch_rank
        shape = tuple(base.batch_shape) + tuple(base.event_shape)
        k = len(base.batch_shape) - reinterpreted_batch_rank
        super().__init__(shape[:k], shape[k:])

    @property
    def mean(self):
        return self._base.mean

    @property
    def variance(self):
        return self._base.variance

    def sample(self, shape=()):
        return self._base.sample(shape)

    def rsample(self, shape=()):
        return self._base.rsample(shape)

    def log_prob(self, value):
        return _wrap(sum_rightmost(raw(self._base.log_prob(value)), self._reinterpreted_batch_rank))

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())

    def entropy(self):
        return _wrap(sum_rightmost(raw(self._base.entropy()), self._reinterpreted_batch_rank))


class TransformedDistribution(Distribution):
    """Y = T_n(...T_1(X)) for X ~ base; log p(y) adds the inverse log-det-Jacobians."""

    def __init__(self, base, transforms):
        from .transform import ChainTransform, Transform

        if not isinstance(base, Distribution):
            raise TypeError(f"Expected type of 'base' is Distribution, but got {type(base)}.")
        if not isinstance(transforms, (list, tuple)):
            raise TypeError(f"Expected type of 'transforms' is Sequence[Transform] or Chain, but got "
                            f"{type(transforms)}.")
        if not all(isinstance(t, Transform) for t in transforms):
            raise TypeError("All element of transforms must be Transform type.")
        self._base = base
        self._transforms = list(transforms)
        if not transforms:
            super().__init__(base.batch_shape, base.event_shape)
            return
        chain = ChainTransform(transforms)
        base_shape = tuple(base.batch_shape) + tuple(base.event_shape)
        if len(base_shape) < chain._domain.event_rank:
            raise ValueError(f"'base' needs to have shape with size at least {chain._domain.event_rank}, bug got "
                             f"{len(base_shape)}.")
        if chain._domain.event_rank > len(base.event_shape):
            base = Independent(base, chain._domain.event_rank - len(base.event_shape))
        out_shape = chain.forward_shape(tuple(base.batch_shape) + tuple(base.event_shape))
        ev = chain._codomain.event_rank + max(len(base.event_shape) - chain._domain.event_rank, 0)
        super().__init__(out_shape[:len(out_shape) - ev], out_shape[len(out_shape) - ev:])

    def sample(self, shape=()):
        x = self._base.sample(shape)
        for t in self._transforms:
            x = t.forward(x)
        return x

    def rsample(self, shape=()):
        x = self._base.rsample(shape)
        for t in self._transforms:
            x = t.forward(x)
        return x

    def log_prob(self, value):
        lp = 0.0
        y = value
        event_rank = len(self.event_shape)
        for t in reversed(self._transforms):
            x = t.inverse(y)
            event_rank += t._domain.event_rank - t._codomain.event_rank
            lp = lp - sum_rightmost(raw(t.forward_log_det_jacobian(x)), event_rank - t._domain.event_rank)
            y = x
        lp = lp + sum_rightmost(raw(self._base.log_prob(y)), event_rank - len(self._base.event_shape))
        return _wrap(lp)

    def prob(self, value):
        return _wrap(raw(self.log_prob(value)).exp())
