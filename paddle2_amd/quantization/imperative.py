"""Legacy dygraph quantization API (reference: python/paddle/quantization/imperative/qat.py
ImperativeQuantAware, ptq.py ImperativePTQ, ptq_config.py PTQConfig, ptq_quantizer.py
Absmax/PerChannelAbsmax/Hist/KL quantizers, ptq_registry.py PTQRegistry)."""
from __future__ import annotations

import copy
import math

import numpy as np
import torch

from ..framework.tensor import Tensor


def _t(x):
    return x._t if isinstance(x, Tensor) else x


class ImperativeQuantAware:
    """Swap quantizable layers (Linear / Conv2D by default) for fake-quant QuantizedLinear /
    QuantizedConv2D with the chosen weight / activation quantize types."""

    def __init__(self, quantizable_layer_type=("Conv2D", "Linear"), weight_quantize_type="abs_max",
                 activation_quantize_type="moving_average_abs_max", weight_bits=8, activation_bits=8,
                 moving_rate=0.9, fuse_conv_bn=False, weight_preprocess_layer=None, act_preprocess_layer=None,
                 weight_quantize_layer=None, act_quantize_layer=None, onnx_format=False):
        self._types = set(t if isinstance(t, str) else t.__name__ for t in quantizable_layer_type)
        self._kw = dict(weight_bits=weight_bits, activation_bits=activation_bits, moving_rate=moving_rate,
                        weight_quantize_type=weight_quantize_type, activation_quantize_type=activation_quantize_type,
                        weight_pre_layer=weight_preprocess_layer, act_pre_layer=act_preprocess_layer,
                        weight_quant_layer=weight_quantize_layer, act_quant_layer=act_quantize_layer)

    def quantize(self, model):
        from ..nn.quant.quant_layers import QuantizedConv2D, QuantizedLinear

        for name, child in list(model.named_children()):
            tn = type(child).__name__
            if tn in self._types and tn in ("Linear", "Conv2D"):
                cls = QuantizedLinear if tn == "Linear" else QuantizedConv2D
                model._sub_layers[name] = cls(child, **self._kw)
            else:
                self.quantize(child)
        return model

    def save_quantized_model(self, layer, path, input_spec=None, **config):
        from .. import jit

        jit.save(layer, path, input_spec=input_spec, **config)


# ----------------------------------------------------------------------------- PTQ quantizers
class BaseQuantizer:
    def __init__(self, quant_bits=8):
        self.quant_bits = quant_bits
        self.thresholds = []
        self.abs_max_vals = []

    def sample_data(self, layer, tensors):
        raise NotImplementedError

    def cal_thresholds(self):
        raise NotImplementedError


class AbsmaxQuantizer(BaseQuantizer):
    def sample_data(self, layer, tensors):
        vals = [float(_t(t).detach().abs().max()) for t in tensors]
        self.abs_max_vals = vals if not self.abs_max_vals else [max(a, b) for a, b in zip(self.abs_max_vals, vals)]

    def cal_thresholds(self):
        self.thresholds = list(self.abs_max_vals)


class PerChannelAbsmaxQuantizer(BaseQuantizer):
    def sample_data(self, layer, tensors):
        vals = []
        for t in tensors:
            x = _t(t).detach().float()
            axis = 1 if type(layer).__name__ == "Linear" and x.dim() == 2 else 0
            dims = [d for d in range(x.dim()) if d != axis]
            vals.append(x.abs().amax(dim=dims).cpu().numpy())
        self.abs_max_vals = vals if not self.abs_max_vals else [np.maximum(a, b) for a, b in
                                                                zip(self.abs_max_vals, vals)]

    def cal_thresholds(self):
        self.thresholds = list(self.abs_max_vals)


class _HistBase(BaseQuantizer):
    def __init__(self, quant_bits=8, bins=1024, upsample_bins=64):
        super().__init__(quant_bits)
        self.bins, self.upsample_bins = bins, upsample_bins
        self.hists = []

    def sample_data(self, layer, tensors):
        if not self.abs_max_vals:
            self.abs_max_vals = [float(_t(t).detach().abs().max()) for t in tensors]
            self.hists = [None] * len(tensors)
        for i, t in enumerate(tensors):
            x = _t(t).detach().abs().float().flatten().cpu()
            mx = max(self.abs_max_vals[i], 1e-8)
            h = torch.histc(x.clamp(max=mx), bins=self.bins, min=0, max=mx).numpy()
            self.hists[i] = h if self.hists[i] is None else self.hists[i] + h


class HistQuantizer(_HistBase):
    """Threshold = the ``hist_percent`` quantile of |x|."""

    def __init__(self, quant_bits=8, bins=1024, hist_percent=0.99999):
        super().__init__(quant_bits, bins)
        self.hist_percent = hist_percent

    def cal_thresholds(self):
        self.thresholds = []
        for h, mx in zip(self.hists, self.abs_max_vals):
            c = np.cumsum(h) / max(h.sum(), 1)
            idx = min(int(np.searchsorted(c, self.hist_percent)), self.bins - 1)
            self.thresholds.append((idx + 1) * mx / self.bins)


class KLQuantizer(_HistBase):
    """Threshold minimising the KL divergence between the clipped reference histogram and its
    ``2^(bits-1)``-level quantized version (TensorRT-style calibration)."""

    def cal_thresholds(self):
        self.thresholds = []
        levels = 2 ** (self.quant_bits - 1)
        for h, mx in zip(self.hists, self.abs_max_vals):
            best, best_i = math.inf, self.bins
            for i in range(levels, self.bins + 1, max(1, self.bins // 128)):
                p = h[:i].astype(np.float64).copy()
                p[i - 1] += h[i:].sum()
                if p.sum() == 0:
                    continue
                chunks = np.array_split(h[:i].astype(np.float64), levels)
                q = np.concatenate([np.full(len(c), c.sum() / max((c > 0).sum(), 1)) * (c > 0) for c in chunks])
                p, q = p / p.sum(), q / max(q.sum(), 1e-12)
                m = p > 0
                kl = float(np.sum(p[m] * np.log(p[m] / np.maximum(q[m], 1e-12))))
                if kl < best:
                    best, best_i = kl, i
            self.thresholds.append(best_i * mx / self.bins)


SUPPORT_ACT_QUANTIZERS = [AbsmaxQuantizer, HistQuantizer, KLQuantizer]
SUPPORT_WT_QUANTIZERS = [AbsmaxQuantizer, PerChannelAbsmaxQuantizer]


class PTQConfig:
    def __init__(self, activation_quantizer, weight_quantizer):
        assert type(activation_quantizer) in SUPPORT_ACT_QUANTIZERS
        assert type(weight_quantizer) in SUPPORT_WT_QUANTIZERS
        self.in_act_quantizer = copy.deepcopy(activation_quantizer)
        self.out_act_quantizer = copy.deepcopy(activation_quantizer)
        self.wt_quantizer = copy.deepcopy(weight_quantizer)
        self.quant_hook_handle = None
        self.enable_in_act_quantizer = False


default_ptq_config = PTQConfig(KLQuantizer(), PerChannelAbsmaxQuantizer())


class PTQRegistry:
    _SUPPORTED = {"Conv2D": ["weight"], "Linear": ["weight"], "Conv2DTranspose": ["weight"]}

    @classmethod
    def is_supported_layer(cls, layer):
        return type(layer).__name__ in cls._SUPPORTED

    @classmethod
    def is_simulated_quant_layer(cls, layer):
        return type(layer).__name__.startswith("Quantized")

    @classmethod
    def layer_info(cls, layer):
        return cls._SUPPORTED.get(type(layer).__name__)


class ImperativePTQ:
    """Post-training quantization: ``quantize`` hooks supported layers so calibration forwards
    sample activations/weights; ``save_quantized_model`` computes thresholds and exports."""

    def __init__(self, quant_config=default_ptq_config):
        self._cfg = quant_config

    def quantize(self, model, inplace=False, fuse=False, fuse_list=None):
        m = model if inplace else copy.deepcopy(model)
        for name, layer in m.named_sublayers():
            if PTQRegistry.is_supported_layer(layer):
                cfg = copy.deepcopy(self._cfg)
                layer._quant_config = cfg

                def hook(l, inputs, outputs, cfg=cfg):
                    cfg.in_act_quantizer.sample_data(l, [i for i in inputs if isinstance(i, Tensor)])
                    outs = outputs if isinstance(outputs, (list, tuple)) else [outputs]
                    cfg.out_act_quantizer.sample_data(l, outs)
                    if not cfg.wt_quantizer.abs_max_vals:
                        cfg.wt_quantizer.sample_data(l, [l.weight])

                cfg.quant_hook_handle = layer.register_forward_post_hook(hook)
        return m

    def _calc(self, model):
        for _, layer in model.named_sublayers():
            cfg = getattr(layer, "_quant_config", None)
            if cfg is None:
                continue
            for q in (cfg.in_act_quantizer, cfg.out_act_quantizer, cfg.wt_quantizer):
                if q.abs_max_vals:
                    q.cal_thresholds()
            if cfg.quant_hook_handle is not None:
                cfg.quant_hook_handle.remove()
                cfg.quant_hook_handle = None

    def save_quantized_model(self, model, path, input_spec=None, **config):
        from .. import jit

        self._calc(model)
        jit.save(model, path, input_spec=input_spec, **config)
