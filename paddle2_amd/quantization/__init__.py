"""paddle.quantization — QAT / PTQ (reference: python/paddle/quantization/ — config.py:67 QuantConfig,
factory.py:78 quanter, qat.py:27 QAT, ptq.py:29 PTQ, quantize.py:28 Quantization.convert,
quanters/abs_max.py FakeQuanterWithAbsMaxObserver, observers/abs_max.py AbsmaxObserver,
observers/groupwise.py GroupWiseWeightObserver, wrapper.py ObserveWrapper, imperative/ legacy API).

Flow: a QuantConfig maps layers (by instance, name prefix or type) to (activation, weight)
quanter *factories*; ``QAT.quantize`` swaps quantifiable layers for their QAT counterparts
(Linear -> QuantedLinear, Conv2D -> QuantedConv2D) whose quanters fake-quantize in forward with a
straight-through gradient; ``PTQ.quantize`` additionally wraps observed layers so calibration
batches record scales; ``convert`` turns quanters into deployable quant/dequant layers
(LinearQuanterDequanter) and stores weights on the integer grid.
"""
from __future__ import annotations

import abc
import copy

import torch

from ..framework.tensor import Tensor
from ..nn.layer.layers import Layer

_w = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else x


from .base_quanter import BaseQuanter  # noqa: E402
from .base_observer import BaseObserver  # noqa: E402
from .factory import ClassWithArguments, ObserverFactory, QuanterFactory, quanter  # noqa: E402,F401
from .observers import (AbsmaxObserver, AbsmaxObserverLayer, GroupWiseWeightObserver,  # noqa: E402,F401
                        GroupWiseWeightObserverLayer)
from .quanters import FakeQuanterWithAbsMaxObserver, FakeQuanterWithAbsMaxObserverLayer  # noqa: E402,F401


class ObserveWrapper(Layer):
    def __init__(self, observer, observed, observe_input=True):
        super().__init__()
        self._observer, self._observed, self._observe_input = observer, observed, observe_input

    def forward(self, *inputs, **kwargs):
        if self._observe_input:
            out = self._observer(*inputs, **kwargs)
            return self._observed(out, **kwargs)
        out = self._observed(*inputs, **kwargs)
        return self._observer(out, **kwargs)


# ----------------------------------------------------------------------------- config
class SingleLayerConfig:
    def __init__(self, activation, weight):
        self._activation, self._weight = activation, weight

    @property
    def activation(self):
        return self._activation

    @property
    def weight(self):
        return self._weight

    def __str__(self):
        return f"activation: {self._activation}\nweight: {self._weight}"


def _default_qat_mapping():
    from ..nn import Conv2D, Linear
    from ..nn.quant.qat import QuantedConv2D, QuantedLinear

    return {Linear: QuantedLinear, Conv2D: QuantedConv2D}


class QuantConfig:
    def __init__(self, activation, weight):
        self._global_config = None if (activation is None and weight is None) else SingleLayerConfig(activation,
                                                                                                      weight)
        self._layer2config, self._prefix2config, self._type2config = {}, {}, {}
        self._model = None
        self._qat_layer_mapping = _default_qat_mapping()
        self._customized_qat_layer_mapping = {}
        self._customized_leaves = []

    def add_layer_config(self, layer, activation=None, weight=None):
        # keyed by the layer's unique full name, which survives the deepcopy in quantize()
        for l in (layer if isinstance(layer, (list, tuple)) else [layer]):
            self.add_name_config(l.full_name(), activation, weight)

    def add_name_config(self, layer_name, activation=None, weight=None):
        for n in (layer_name if isinstance(layer_name, (list, tuple)) else [layer_name]):
            self._prefix2config[n] = SingleLayerConfig(activation, weight)

    def add_type_config(self, layer_type, activation=None, weight=None):
        for t in (layer_type if isinstance(layer_type, (list, tuple)) else [layer_type]):
            self._type2config[t] = SingleLayerConfig(activation, weight)

    def add_qat_layer_mapping(self, source, target):
        self._qat_layer_mapping[source] = target
        self._customized_qat_layer_mapping[source] = target

    def add_customized_leaf(self, layer_type):
        self._customized_leaves.append(layer_type)

    @property
    def customized_leaves(self):
        return self._customized_leaves

    @property
    def qat_layer_mappings(self):
        return self._qat_layer_mapping

    @property
    def default_qat_layer_mapping(self):
        return _default_qat_mapping()

    @property
    def global_config(self):
        return self._global_config

    def _specify(self, model):
        """Resolve every sub-layer's config: global < parent's < type < full name / name prefix."""
        self._model = model
        self._resolved = {id(model): self._global_config}
        named = dict((id(l), n) for n, l in model.named_sublayers())

        def visit(parent):
            for child in parent.children():
                cfg = self._resolved.get(id(parent), self._global_config)
                cfg = self._type2config.get(type(child), cfg)
                sname = named.get(id(child), "")
                for key, c in self._prefix2config.items():
                    if key == child.full_name() or sname == key or sname.startswith(key + "."):
                        cfg = c
                self._resolved[id(child)] = cfg
                visit(child)

        visit(model)

    def _get_config_by_layer(self, layer):
        return getattr(self, "_resolved", {}).get(id(layer), self._global_config)

    def _is_leaf(self, layer):
        return not layer._sub_layers or type(layer) in self._customized_leaves

    def _is_quantifiable(self, layer):
        return self._get_config_by_layer(layer) is not None

    def _get_qat_layer(self, layer):
        return self._qat_layer_mapping[type(layer)](layer, self._get_config_by_layer(layer))

    def _need_observe(self, layer):
        cfg = self._get_config_by_layer(layer)
        return (self._is_leaf(layer) and cfg is not None and cfg.activation is not None
                and type(layer) not in self._qat_layer_mapping.values())

    def _get_observe_wrapper(self, layer):
        cfg = self._get_config_by_layer(layer)
        return ObserveWrapper(cfg.activation._instance(layer), layer)

    def details(self):
        lines = []
        model = self._model
        if model is None:
            return str(self)
        for name, layer in list(model.named_sublayers()):
            cfg = self._get_config_by_layer(layer)
            lines.append(f"{name}({type(layer).__name__}): {cfg.activation if cfg else None}, "
                         f"{cfg.weight if cfg else None}")
        return "\n".join(lines)

    def __str__(self):
        return f"Global config:\n{self._global_config}" if self._global_config else "Global config: None"


# ----------------------------------------------------------------------------- QAT / PTQ
class Quantization(metaclass=abc.ABCMeta):
    def __init__(self, config):
        self._config = copy.deepcopy(config)

    @abc.abstractmethod
    def quantize(self, model, inplace=False):
        ...

    def convert(self, model, inplace=False, remain_weight=False):
        from ..nn.quant import ConvertibleQuantedLayer, LinearQuanterDequanter

        m = model if inplace else copy.deepcopy(model)
        repl = {}
        for name, child in m.named_children():
            if isinstance(child, ConvertibleQuantedLayer):
                if child.converted:
                    continue
                wq = getattr(child, "weight_quanter", None)
                if wq is not None and wq.scales() is None:
                    continue
                child._convert(remain_weight=remain_weight)
            elif isinstance(child, BaseQuanter):
                repl[name] = LinearQuanterDequanter.from_quanter(child)
            else:
                self.convert(child, inplace=True, remain_weight=remain_weight)
        for k, v in repl.items():
            m._sub_layers[k] = v
            object.__setattr__(m, k, v) if k in m.__dict__ else None
        return m

    @staticmethod
    def _replace_children(layer, make, descend):
        """Post-order rewrite of the layer tree: a child for which ``make(child)`` returns a layer is swapped for
        it (in place, by name); otherwise the walk enters the child when ``descend(child)`` allows."""
        swaps = []
        for name, child in layer.named_children():
            new = make(child)
            if new is not None:
                swaps.append((name, new))
            elif descend(child):
                Quantization._replace_children(child, make, descend)
        for name, new in swaps:
            layer._sub_layers[name] = new

    def _convert_to_quant_layers(self, model, config):
        # quantifiable layers with a QAT mapping become their quantized counterparts
        self._replace_children(
            model,
            lambda c: config._get_qat_layer(c) if config._is_quantifiable(c) and type(c) in
            config.qat_layer_mappings else None,
            lambda c: True)

    def _insert_activation_observers(self, model, config):
        # observed layers get their observe wrapper; already-quantized layers are leaves
        qat_types = tuple(config.qat_layer_mappings.values())
        self._replace_children(
            model,
            lambda c: config._get_observe_wrapper(c) if config._need_observe(c) else None,
            lambda c: type(c) not in qat_types)

    def _details(self):
        return self._config.details()

    def __str__(self):
        return self._details()

    __repr__ = __str__


class QAT(Quantization):
    def quantize(self, model, inplace=False):
        assert model.training, "QAT.quantize expects a model in training mode"
        m = model if inplace else copy.deepcopy(model)
        self._config._specify(m)
        self._convert_to_quant_layers(m, self._config)
        self._insert_activation_observers(m, self._config)
        return m


class PTQ(Quantization):
    def quantize(self, model, inplace=False):
        m = model if inplace else copy.deepcopy(model)
        m.eval()
        self._config._specify(m)
        self._convert_to_quant_layers(m, self._config)
        self._insert_activation_observers(m, self._config)
        return m


from .imperative import (SUPPORT_ACT_QUANTIZERS, SUPPORT_WT_QUANTIZERS, AbsmaxQuantizer,  # noqa: E402,F401
                         BaseQuantizer, HistQuantizer, ImperativePTQ, ImperativeQuantAware, KLQuantizer,
                         PerChannelAbsmaxQuantizer, PTQConfig, PTQRegistry, default_ptq_config)

__all__ = ["QuantConfig", "BaseQuanter", "BaseObserver", "quanter", "QAT", "PTQ"]
