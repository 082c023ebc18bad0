"""RNG state (reference: phi/core/generator.h:32 — Philox seed/offset per device).

The MI355X kernels that need randomness (dropout inside our fused kernels) take an explicit
(seed, offset) pair drawn from :func:`next_philox` so results are reproducible and graph-capture
safe; everything else uses torch's per-device Philox generators.
"""
from __future__ import annotations

import random as _py_random

import numpy as np
import torch

_seed = 0
_philox_offset = 0


def seed(s: int):
    """paddle.seed."""
    global _seed, _philox_offset
    _seed = int(s)
    _philox_offset = 0
    torch.manual_seed(_seed)
    _py_random.seed(_seed)
    np.random.seed(_seed % (2**32))
    return torch.default_generator


def get_rng_state(device=None):
    if device is not None and "gpu" in str(device) and torch.cuda.is_available():
        return [torch.cuda.get_rng_state(i) for i in range(torch.cuda.device_count())]
    return [torch.get_rng_state()]


def set_rng_state(state, device=None):
    if device is not None and "gpu" in str(device) and torch.cuda.is_available():
        for i, s in enumerate(state):
            torch.cuda.set_rng_state(s, i)
    else:
        torch.set_rng_state(state[0])


def get_cuda_rng_state():
    if not torch.cuda.is_available():
        return []
    return [torch.cuda.get_rng_state(i) for i in range(torch.cuda.device_count())]


def set_cuda_rng_state(state):
    for i, s in enumerate(state):
        torch.cuda.set_rng_state(s, i)


def next_philox(increment: int):
    """Return (seed, offset) and advance the global Philox offset (``IncrementOffset``)."""
    global _philox_offset
    off = _philox_offset
    _philox_offset += int(increment)
    return _seed, off
