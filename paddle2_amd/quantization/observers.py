"""paddle.quantization.observers (reference: python/paddle/quantization/observers/abs_max.py, groupwise.py).

* AbsmaxObserver: the running max |x| of every calibration batch -> one per-tensor scale;
* GroupWiseWeightObserver: per (group of ``group_size`` input rows, output channel) max |W| for weight-only
  int8 / int4 quantization (the scales the weight-only GEMMs consume).
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from .base_observer import BaseObserver
from .factory import QuanterFactory

_w = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


class AbsmaxObserverLayer(BaseObserver):
    def __init__(self, layer, quant_bits=8):
        super().__init__()
        self._quant_bits = quant_bits
        self.abs_max_val = torch.tensor(1e-7)

    def forward(self, input):
        x = _t(input)
        self.abs_max_val = torch.maximum(self.abs_max_val.to(x.device), x.detach().abs().max().float())
        return input

    def cal_thresholds(self):
        self.thresholds = self.abs_max_val

    def bit_length(self):
        return self._quant_bits

    def quant_axis(self):
        return -1

    def scales(self):
        return _w(self.abs_max_val.reshape(()).clone())

    def zero_points(self):
        return None


class AbsmaxObserver(QuanterFactory):
    def __init__(self, quant_bits=8):
        super().__init__(quant_bits=quant_bits)

    def _get_class(self):
        return AbsmaxObserverLayer


class GroupWiseWeightObserverLayer(BaseObserver):
    """Per-(group of input rows, output channel) abs-max for weight-only quantization."""

    def __init__(self, layer, quant_bits=8, group_size=128):
        super().__init__()
        self._quant_bits, self.group_size = quant_bits, group_size
        self._max = None

    def forward(self, input):
        x = _t(input).detach().float()
        if x.dim() == 2 and x.shape[0] % self.group_size == 0:
            m = x.reshape(-1, self.group_size, x.shape[1]).abs().amax(1)
        else:
            m = x.abs().amax(0, keepdim=True)
        self._max = m if self._max is None else torch.maximum(self._max, m)
        return input

    def cal_thresholds(self):
        pass

    def bit_length(self):
        return self._quant_bits

    def quant_axis(self):
        return -1

    def scales(self):
        return _w(self._max) if self._max is not None else None

    def zero_points(self):
        return None


class GroupWiseWeightObserver(QuanterFactory):
    def __init__(self, quant_bits=8, group_size=128):
        super().__init__(quant_bits=quant_bits, group_size=group_size)

    def _get_class(self):
        return GroupWiseWeightObserverLayer


__all__ = ["AbsmaxObserver", "GroupWiseWeightObserver"]
