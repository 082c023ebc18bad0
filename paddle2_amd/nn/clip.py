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
        self._cache = None

    def _global_sq_norm(self, grads):
        """Sum of squares over all grads (fp32 device scalar)."""
        from ..optimizer.multi_tensor import MultiTensorTable

        dev = grads[0].device
        if dev.type == "cuda":
            key = tuple((g.data_ptr(), g.numel(), g.dtype) for g in grads)
            if self._cache is None or self._cache[0] != key:
                self._cache = (key, MultiTensorTable.for_grads(grads))
            return self._cache[1].sqnorm()
        return sum((g.float() ** 2).sum() for g in grads)

    # The fused optimizers take the clip coefficient as a device scalar and fold it into their
    # single pass over the gradients (no separate scale pass over 2x the grad bytes).
    _fusable = True

    def global_coef(self, params_grads):
        """Device fp32 [1] tensor min(1, clip_norm / ||g||) over clippable grads (no host sync)."""
        grads = [g._t for p, g in params_grads if g is not None and getattr(p, "need_clip", True)]
        if not grads:
            return None
        if len(grads) != len(params_grads):
            return None  # some grads excluded from clipping: fall back to the explicit scale pass
        sq = self._reduce_global(self._global_sq_norm(grads))
        norm = torch.sqrt(sq)
        return torch.clamp(self.clip_norm / torch.clamp(norm, min=1e-6), max=1.0).float().reshape(1)

    def _dygraph_clip(self, params_grads):
        grads = [g._t for p, g in params_grads if g is not None and getattr(p, "need_clip", True)]
        if not grads:
            return params_grads
        sq = self._global_sq_norm(grads)
        sq = self._reduce_global(sq)
        norm = torch.sqrt(sq)
        coef = torch.clamp(self.clip_norm / torch.clamp(norm, min=1e-6), max=1.0).float().reshape(1)
        if grads[0].device.type == "cuda":
            self._cache[1].scale(coef)
        else:
            for g in grads:
                g.mul_(coef.to(g.dtype))
        return params_grads

    def _reduce_global(self, sq):
        """Hook for hybrid-parallel global norm (overridden by HybridParallelClipGrad)."""
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
