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


# ----------------------------------------------------------------------------- bases
class BaseQuanter(Layer, metaclass=abc.ABCMeta):
    def __init__(self):
        super().__init__()

    @abc.abstractmethod
    def forward(self, input):
        ...

    @abc.abstractmethod
    def scales(self):
        ...

    @abc.abstractmethod
    def zero_points(self):
        ...

    @abc.abstractmethod
    def quant_axis(self):
        ...

    @abc.abstractmethod
    def bit_length(self):
        ...


class BaseObserver(BaseQuanter, metaclass=abc.ABCMeta):
    def __init__(self):
        super().__init__()

    @abc.abstractmethod
    def cal_thresholds(self):
        ...


class ClassWithArguments(metaclass=abc.ABCMeta):
    def __init__(self, **kwargs):
        self._kwargs = kwargs

    @property
    def args(self):
        return self._kwargs

    @abc.abstractmethod
    def _get_class(self):
        ...

    def __str__(self):
        args = ",".join(f"{k}={v}" for k, v in self._kwargs.items())
        return f"{self.__class__.__name__}({args})"

    __repr__ = __str__


class QuanterFactory(ClassWithArguments):
    """Holds constructor arguments; ``_instance(layer)`` builds one quanter per quantized layer."""

    def __init__(self, **kwargs):
        super().__init__(**kwargs)
        self.partial_class = None

    def _instance(self, layer):
        return self._get_class()(layer, **self._kwargs)


ObserverFactory = QuanterFactory


def quanter(class_name):
    """Decorator: ``@quanter("MyQuanter")`` on a BaseQuanter subclass ``MyQuanterLayer`` registers a
    factory class named ``MyQuanter`` in the caller's module."""

    def deco(target):
        import inspect

        frm = inspect.stack()[1]
        mod = inspect.getmodule(frm[0])
        factory = type(class_name, (QuanterFactory,), {
            "__init__": lambda self, *a, **k: QuanterFactory.__init__(self, **k),
            "_get_class": lambda self: target})
        if mod is not None:
            setattr(mod, class_name, factory)
        return target

    return deco


# ----------------------------------------------------------------------------- observers / quanters
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


class FakeQuanterWithAbsMaxObserverLayer(BaseQuanter):
    """Moving-average abs-max fake quanter: scale = accum/state, accum = rate*accum + max|x|."""

    def __init__(self, layer, name=None, moving_rate=0.9, bit_length=8, dtype="float32"):
        super().__init__()
        self._moving_rate, self._bit_length = moving_rate, bit_length
        self.register_buffer("_scale", _w(torch.full((1,), 1e-3)))
        self.register_buffer("_state", _w(torch.zeros(1)))
        self.register_buffer("_accum", _w(torch.zeros(1)))

    def forward(self, input):
        from ..nn.quant.quant_layers import fake_quant_dequant

        x = _t(input)
        if self.training:
            with torch.no_grad():
                cur = x.detach().abs().max().float().reshape(1).to(self._accum._t.device)
                self._accum._t.mul_(self._moving_rate).add_(cur)
                self._state._t.mul_(self._moving_rate).add_(1.0)
                self._scale._t.copy_(self._accum._t / self._state._t)
        return _w(fake_quant_dequant(x, self._scale._t.to(x.device).reshape(()), self._bit_length))

    def bit_length(self):
        return self._bit_length

    def quant_axis(self):
        return -1

    def scales(self):
        return self._scale

    def zero_points(self):
        return None


class FakeQuanterWithAbsMaxObserver(QuanterFactory):
    def __init__(self, moving_rate=0.9, bit_length=8, dtype="float32", name=None):
        super().__init__(name=name, moving_rate=moving_rate, bit_length=bit_length, dtype=dtype)

    def _get_class(self):
        return FakeQuanterWithAbsMaxObserverLayer


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
