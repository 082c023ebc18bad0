"""paddle.onnx.export (reference: python/paddle/onnx/export.py:35, which drives paddle2onnx).

Here the Layer is traced through torch's ONNX exporter: a thin ``torch.nn.Module`` adapter calls the
Layer on wrapped tensors, parameters are frozen for the trace, and ``{path}.onnx`` is written.  The
exporter needs the ``onnx`` package; without it a clear ImportError is raised.
"""
from __future__ import annotations

import os

import torch

from ..framework.tensor import Tensor


class _Adapter(torch.nn.Module):
    def __init__(self, layer):
        super().__init__()
        self._layer = layer

    def forward(self, *xs):
        out = self._layer(*[Tensor._wrap(x) for x in xs])
        if isinstance(out, (list, tuple)):
            return tuple(o._t if isinstance(o, Tensor) else o for o in out)
        return out._t if isinstance(out, Tensor) else out


def _example(spec):
    if isinstance(spec, Tensor):
        return spec._t
    if isinstance(spec, torch.Tensor):
        return spec
    from ..framework.dtype import convert_dtype

    shape = [1 if (d is None or d < 0) else int(d) for d in spec.shape]
    dt = convert_dtype(spec.dtype)
    return torch.zeros(shape, dtype=dt) if not dt.is_floating_point else torch.randn(shape).to(dt)


def export(layer, path, input_spec=None, opset_version=9, **configs):
    try:
        import onnx  # noqa: F401
    except ImportError as e:
        raise ImportError("paddle.onnx.export needs the 'onnx' package, which is not installed") from e
    if input_spec is None:
        raise ValueError("input_spec is required to trace the Layer")
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    params = list(layer.parameters())
    flags = [p._t.requires_grad for p in params]
    was_training = getattr(layer, "training", False)
    layer.eval()
    try:
        for p in params:
            p._t.requires_grad_(False)
        names = [getattr(s, "name", None) or f"x{i}" for i, s in enumerate(input_spec)]
        dyn = {}
        for n, s in zip(names, input_spec):
            shp = getattr(s, "shape", None) or []
            axes = {i: f"{n}_d{i}" for i, v in enumerate(shp) if v is None or (isinstance(v, int) and v < 0)}
            if axes:
                dyn[n] = axes
        with torch.no_grad():
            torch.onnx.export(_Adapter(layer), tuple(_example(s) for s in input_spec), path + ".onnx",
                              input_names=names, opset_version=max(int(opset_version), 9),
                              dynamic_axes=dyn or None, dynamo=False)
    finally:
        for p, f in zip(params, flags):
            p._t.requires_grad_(f)
        if was_training:
            layer.train()
