"""Paddle data types on top of torch dtypes.

Paddle exposes ``paddle.float32`` etc. (phi/common/data_type.h; python/paddle/framework/dtype.py).
Here the dtype objects *are* torch dtypes so tensors carry no conversion cost on the hot path;
strings, numpy dtypes and Paddle-style names are normalised through :func:`convert_dtype`.
"""
from __future__ import annotations

import numpy as np
import torch

bool_ = torch.bool
uint8 = torch.uint8
int8 = torch.int8
int16 = torch.int16
int32 = torch.int32
int64 = torch.int64
float16 = torch.float16
bfloat16 = torch.bfloat16
float32 = torch.float32
float64 = torch.float64
complex64 = torch.complex64
complex128 = torch.complex128
# OCP fp8 (gfx950 MFMA native formats; NOT the MI300 fnuz variants)
float8_e4m3fn = torch.float8_e4m3fn
float8_e5m2 = torch.float8_e5m2

_STR2DT = {
    "bool": bool_, "uint8": uint8, "int8": int8, "int16": int16, "int32": int32, "int64": int64,
    "float16": float16, "half": float16, "fp16": float16,
    "bfloat16": bfloat16, "bf16": bfloat16, "uint16": bfloat16,  # paddle encodes bf16 as uint16 in numpy
    "float32": float32, "float": float32, "fp32": float32,
    "float64": float64, "double": float64, "fp64": float64,
    "complex64": complex64, "complex128": complex128,
    "float8_e4m3fn": float8_e4m3fn, "float8_e5m2": float8_e5m2,
}

_DT2STR = {
    bool_: "bool", uint8: "uint8", int8: "int8", int16: "int16", int32: "int32", int64: "int64",
    float16: "float16", bfloat16: "bfloat16", float32: "float32", float64: "float64",
    complex64: "complex64", complex128: "complex128",
    float8_e4m3fn: "float8_e4m3fn", float8_e5m2: "float8_e5m2",
}

_NP2DT = {
    np.dtype("bool"): bool_, np.dtype("uint8"): uint8, np.dtype("int8"): int8,
    np.dtype("int16"): int16, np.dtype("int32"): int32, np.dtype("int64"): int64,
    np.dtype("float16"): float16, np.dtype("float32"): float32, np.dtype("float64"): float64,
    np.dtype("complex64"): complex64, np.dtype("complex128"): complex128,
}

_DT2NP = {v: k for k, v in _NP2DT.items()}

_default_dtype = float32


def convert_dtype(dtype) -> torch.dtype:
    """Normalise any Paddle/numpy/str dtype spelling to a torch dtype."""
    if dtype is None:
        return None
    if isinstance(dtype, torch.dtype):
        return dtype
    if isinstance(dtype, str):
        key = dtype.lower().replace("paddle.", "").replace("torch.", "")
        if key in _STR2DT:
            return _STR2DT[key]
        raise TypeError(f"unsupported dtype string {dtype!r}")
    if dtype is bool:
        return bool_
    if dtype is int:
        return int64
    if dtype is float:
        return _default_dtype
    try:
        return _NP2DT[np.dtype(dtype)]
    except Exception as e:  # pragma: no cover - defensive
        raise TypeError(f"unsupported dtype {dtype!r}") from e


def dtype_name(dtype) -> str:
    return _DT2STR[convert_dtype(dtype)]


def to_numpy_dtype(dtype):
    dt = convert_dtype(dtype)
    if dt == bfloat16:
        return np.dtype("uint16")
    return _DT2NP[dt]


def set_default_dtype(d):
    global _default_dtype
    d = convert_dtype(d)
    if d not in (float16, bfloat16, float32, float64):
        raise TypeError("default dtype must be a floating type")
    _default_dtype = d
    torch.set_default_dtype(d if d in (float32, float64) else float32)


def get_default_dtype():
    return _DT2STR[_default_dtype]


def default_float_dtype() -> torch.dtype:
    return _default_dtype


def is_floating_point_dtype(dtype) -> bool:
    return convert_dtype(dtype).is_floating_point


def is_integer_dtype(dtype) -> bool:
    d = convert_dtype(dtype)
    return d in (uint8, int8, int16, int32, int64)


def finfo(dtype):
    return torch.finfo(convert_dtype(dtype))


def iinfo(dtype):
    return torch.iinfo(convert_dtype(dtype))
