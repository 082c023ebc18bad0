"""fp32 ``main_grad`` accumulation for bf16/fp16 params (reference: fleet/utils/mix_precision_utils.py —
``MixPrecisionLayer`` :35-71 registers grad hooks that add each low-precision grad into an fp32
``main_grad`` and drop the bf16 grad; ``MixPrecisionOptimizer`` :97-199 steps on ``main_grad``).

Our optimizers already read ``main_grad`` when present (paddle2_amd.optimizer.optimizer._grad_of),
so the optimizer wrapper only has to manage clearing.
"""
from __future__ import annotations

import torch

from ....framework.tensor import Tensor
from ....nn.layer.layers import Layer


class MixPrecisionLayer(Layer):
    def __init__(self, layers, dtype="float16"):
        super().__init__()
        self._layers = layers
        self._dtype = dtype
        for p in layers.parameters():
            if p._t.dtype in (torch.float16, torch.bfloat16) and not p.stop_gradient:
                p.main_grad = None
                p._t.register_post_accumulate_grad_hook(self._make_hook(p))

    @staticmethod
    def _make_hook(p):
        def hook(t):
            g = t.grad
            if g is None:
                return
            if p.main_grad is None:
                p.main_grad = Tensor._wrap(g.float())
            else:
                p.main_grad._t.add_(g.float())
            t.grad = None

        return hook

    def forward(self, *inputs, **kwargs):
        return self._layers(*inputs, **kwargs)

    def state_dict(self, *a, **k):
        return self._layers.state_dict(*a, **k)

    def set_state_dict(self, *a, **k):
        return self._layers.set_state_dict(*a, **k)


class MixPrecisionOptimizer:
    def __init__(self, optimizer):
        self._inner_opt = optimizer

    def step(self):
        self._inner_opt.step()

    def clear_grad(self, set_to_zero=True):
        for p in self._inner_opt._parameter_list:
            if getattr(p, "main_grad", None) is not None:
                if set_to_zero:
                    p.main_grad._t.zero_()
                else:
                    p.main_grad = None
            if p._t.grad is not None:
                p._t.grad = None

    clear_gradients = clear_grad

    def __getattr__(self, name):
        return getattr(self._inner_opt, name)


class MixPrecisionScaler:
    def __init__(self, scaler):
        self._inner = scaler

    def __getattr__(self, name):
        return getattr(self._inner, name)
