"""Gradient clipping (reference: python/paddle/nn/clip.py).

``ClipGradByGlobalNorm`` runs the multi-tensor sum-of-squares and scale HIP kernels on the GPU
(one launch each for the whole parameter set, no host sync — the clip coefficient stays on
device), matching the reference's squared_l2_norm + scale kernels per parameter.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor


class ClipGradBase:
    def __call__(self, params_grads):
        return self._dygraph_clip(params_grads)


class ClipGradByValue(ClipGradBase):
    def __init__(self, max, min=None):
        self.max = float(max)
        self.min = -self.max if min is None else float(min)

    def _dygraph_clip(self, params_grads):
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                continue
            g._t.clamp_(self.min, self.max)
        return params_grads


class ClipGradByNorm(ClipGradBase):
    def __init__(self, clip_norm):
        self.clip_norm = float(clip_norm)

    def _dygraph_clip(self, params_grads):
        for p, g in params_grads:
            if g is None or not getattr(p, "need_clip", True):
                continue
            n = torch.linalg.vector_norm(g._t.float())
            coef = torch.clamp(self.clip_norm / torch.clamp(n, min=1e-6), max=1.0)
            g._t.mul_(coef.to(g._t.dtype))
        return params_grads


class ClipGradByGlobalNorm(ClipGradBase):
    def __init__(self, clip_norm, group_name="default_group", auto_skip_clip=False):
        self.clip_norm = float(clip_norm)
        self.group_name = group_name
        self._tables = {}

    def _table(self, grads):
        """Cached multi-tensor table for a grad list (keyed on pointers/sizes; rebuilt if they move)."""
        from ..optimizer.multi_tensor import MultiTensorTable

        key = tuple((g.data_ptr(), g.numel(), g.dtype) for g in grads)
        t = self._tables.get(key)
        if t is None:
            if len(self._tables) > 8:
                self._tables.clear()
            t = self._tables[key] = MultiTensorTable.for_grads(grads)
        return t

    def _sq_norm(self, grads):
        """Sum of squares over ``grads`` (fp32 device scalar, one multi-tensor launch on GPU)."""
        if not grads:
            return None
        if grads[0].device.type == "cuda":
            return self._table(grads).sqnorm()
        return sum((g.float() ** 2).sum() for g in grads).reshape(1)

    def _total_sq(self, params_grads):
        """Global sum of squares of all clippable grads (overridden by HybridParallelClipGrad)."""
        grads = [g._t for p, g in params_grads if g is not None and getattr(p, "need_clip", True)]
        sq = self._sq_norm(grads)
        return None if sq is None else self._reduce_global(sq)

    def _coef(self, sq):
        norm = torch.sqrt(sq)
        return torch.clamp(self.clip_norm / torch.clamp(norm, min=1e-6), max=1.0).float().reshape(1)

    # The fused optimizers take the clip coefficient as a device scalar and fold it into their
    # single pass over the gradients (no separate scale pass over 2x the grad bytes).
    _fusable = True

    def global_coef(self, params_grads):
        """Device fp32 [1] tensor min(1, clip_norm / ||g||) over clippable grads (no host sync)."""
        n_clip = sum(1 for p, g in params_grads if g is not None and getattr(p, "need_clip", True))
        if n_clip == 0 or n_clip != len(params_grads):
            return None  # some grads excluded from clipping: fall back to the explicit scale pass
        sq = self._total_sq(params_grads)
        return None if sq is None else self._coef(sq)

    def _dygraph_clip(self, params_grads):
        grads = [g._t for p, g in params_grads if g is not None and getattr(p, "need_clip", True)]
        if not grads:
            return params_grads
        coef = self._coef(self._total_sq(params_grads))
        if grads[0].device.type == "cuda":
            self._table(grads).scale(coef)
        else:
            for g in grads:
                g.mul_(coef.to(g.dtype))
        return params_grads

    def _reduce_global(self, sq):
        """Hook for cross-rank norm reduction (overridden by hybrid-parallel clipping)."""
        return sq


GradientClipByGlobalNorm = ClipGradByGlobalNorm
GradientClipByNorm = ClipGradByNorm
GradientClipByValue = ClipGradByValue


def clip_grad_norm_(parameters, max_norm, norm_type=2.0, error_if_nonfinite=False):
    if isinstance(parameters, Tensor):
        parameters = [parameters]
    grads = [p._t.grad for p in parameters if p._t.grad is not None]
    if not grads:
        return Tensor._wrap(torch.tensor(0.0))
    total = torch.nn.utils.clip_grad_norm_([p._t for p in parameters if p._t.grad is not None], max_norm, norm_type,
                                           error_if_nonfinite)
    return Tensor._wrap(total)


def clip_grad_value_(parameters, clip_value):
    if isinstance(parameters, Tensor):
        parameters = [parameters]
    torch.nn.utils.clip_grad_value_([p._t for p in parameters], clip_value)
