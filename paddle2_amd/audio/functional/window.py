"""Window functions (reference: python/paddle/audio/functional/window.py:396 get_window).

Windows are computed in float64 on the host (scipy.signal's definitions, which the reference's
implementations follow) and returned as tensors; ``fftbins=True`` gives the periodic form.
"""
from __future__ import annotations

import torch

from ...framework.dtype import convert_dtype
from ...framework.tensor import Tensor

_NAMES = ("hamming", "hann", "gaussian", "general_gaussian", "exponential", "triang", "bohman", "blackman",
          "cosine", "tukey", "taylor", "bartlett", "kaiser", "nuttall")


def get_window(window, win_length, fftbins=True, dtype="float64"):
    from scipy import signal as _sig

    name = window[0] if isinstance(window, tuple) else window
    if name not in _NAMES:
        raise ValueError(f"unknown window {name!r}; expected one of {_NAMES}")
    if name in ("gaussian", "kaiser", "general_gaussian") and not isinstance(window, tuple):
        raise ValueError(f"window {name!r} needs parameters, e.g. ('{name}', 7)")
    w = _sig.get_window(window, int(win_length), fftbins=fftbins)
    return Tensor._wrap(torch.as_tensor(w, dtype=torch.float64).to(convert_dtype(dtype)))
