"""Quanter factories (reference: python/paddle/quantization/factory.py): a QuantConfig holds factories — the
constructor arguments of a quanter — and instantiates one quanter per quantized layer; ``@quanter`` registers a
factory for a user-written BaseQuanter subclass."""
from __future__ import annotations

import abc


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
