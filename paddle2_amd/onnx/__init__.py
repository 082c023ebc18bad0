"""paddle.onnx.export (reference: python/paddle/onnx/export.py:35, which drives paddle2onnx over a ProgramDesc).

The Layer is recorded into the framework's static Program and converted op by op to an ONNX opset-17 graph,
serialized with the framework's own protobuf codec (``onnx/exporter.py``) — no ``onnx`` / ``torch.onnx``
dependency.  ``{path}.onnx`` is written; dynamic (None / -1) input dims are recorded at size 1.
"""
from __future__ import annotations

from .exporter import export_layer, export_program, load_model_dict, run_reference  # noqa: F401


def export(layer, path, input_spec=None, opset_version=17, **configs):
    if input_spec is None:
        raise ValueError("input_spec is required to record the Layer")
    return export_layer(layer, path, input_spec)
