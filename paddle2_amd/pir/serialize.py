"""PIR program serialization: ``save(program, path)`` / ``load(path)``.

Reference: paddle/fluid/pir/serialize_deserialize (pir::WriteModule / ReadModule: a versioned JSON document of
the program's ops — name, operand value ids, typed results, attributes with their types — and
``paddle.static.save`` of the parameters).  Here the document is JSON with a format version; every attribute is
stored with a type tag so bools / ints / floats / strings / dtypes / nested lists round-trip exactly, and the
parameter tensors go to a safetensors file beside it (loaded without executing anything from the file).
"""
from __future__ import annotations

import json
import os

import torch

from . import Operation, Program

FORMAT = "paddle2_amd.pir"
VERSION = 1

_DT = {torch.float32: "f32", torch.float16: "f16", torch.bfloat16: "bf16", torch.float64: "f64", torch.int64: "i64",
       torch.int32: "i32", torch.int16: "i16", torch.int8: "i8", torch.uint8: "u8", torch.bool: "b"}
_DT_INV = {v: k for k, v in _DT.items()}


def _enc(v):
    if isinstance(v, bool):
        return {"t": "b", "v": v}
    if isinstance(v, int):
        return {"t": "i", "v": v}
    if isinstance(v, float):
        return {"t": "f", "v": repr(v)}          # repr keeps every bit of a double
    if isinstance(v, str):
        return {"t": "s", "v": v}
    if v is None:
        return {"t": "n"}
    if isinstance(v, torch.dtype):
        return {"t": "dt", "v": _DT[v]}
    if isinstance(v, (list, tuple)):
        return {"t": "l" if isinstance(v, list) else "tu", "v": [_enc(x) for x in v]}
    if isinstance(v, dict):
        return {"t": "d", "v": {k: _enc(x) for k, x in v.items()}}
    raise TypeError(f"attribute of type {type(v).__name__} is not serializable")


def _dec(e):
    t = e["t"]
    if t in ("b", "i", "s"):
        return e["v"]
    if t == "f":
        return float(e["v"])
    if t == "n":
        return None
    if t == "dt":
        return _DT_INV[e["v"]]
    if t == "l":
        return [_dec(x) for x in e["v"]]
    if t == "tu":
        return tuple(_dec(x) for x in e["v"])
    if t == "d":
        return {k: _dec(x) for k, x in e["v"].items()}
    raise ValueError(f"unknown attribute tag {t!r}")


def to_dict(program):
    ops = []
    for op in program.global_block().ops:
        ops.append({"name": op.name(), "operands": [v.id for v in op.operands()],
                    "results": [{"id": r.id, "shape": r.shape, "dtype": _DT.get(r.dtype, "f32")} for r in op.results()],
                    "attrs": {k: _enc(v) for k, v in op.attrs_.items()}})
    return {"format": FORMAT, "version": VERSION, "ops": ops}


def from_dict(doc, params=None):
    if doc.get("format") != FORMAT:
        raise ValueError(f"not a {FORMAT} document")
    if doc.get("version", 0) > VERSION:
        raise ValueError(f"document version {doc['version']} is newer than this reader ({VERSION})")
    prog = Program()
    vals = {}
    for o in doc["ops"]:
        operands = [vals[i] for i in o["operands"]]
        rtypes = [(r["shape"], _DT_INV[r["dtype"]]) for r in o["results"]]
        op = prog.global_block().append(Operation(o["name"], operands, rtypes,
                                                  {k: _dec(v) for k, v in o["attrs"].items()}))
        for r, rd in zip(op.results(), o["results"]):
            vals[rd["id"]] = r
        if o["name"] == "builtin.parameter" and params is not None:
            prog.params[op.result(0).id] = params[op.attrs_["parameter_name"]]
    return prog


def save(program, path):
    """Write ``path`` (JSON program) and, if the program has parameters, ``path + '.safetensors'``."""
    doc = to_dict(program)
    tensors = {}
    for op in program.global_block().ops:
        if op.name() == "builtin.parameter":
            t = program.params.get(op.result(0).id)
            if t is not None:
                tensors[op.attrs_["parameter_name"]] = t.detach().cpu().contiguous()
    doc["has_params"] = bool(tensors)
    with open(path, "w") as f:
        json.dump(doc, f)
    if tensors:
        from safetensors.torch import save_file

        save_file(tensors, path + ".safetensors")


def load(path):
    with open(path) as f:
        doc = json.load(f)
    params = None
    if doc.get("has_params") and os.path.exists(path + ".safetensors"):
        from safetensors.torch import load_file

        params = load_file(path + ".safetensors")
    return from_dict(doc, params)
