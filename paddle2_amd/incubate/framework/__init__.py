"""paddle.incubate.framework (reference: python/paddle/incubate/framework/random.py): RNG state of every device
generator as a list (or, with ``use_index``, as indices of registered states)."""
from __future__ import annotations

import torch

__all__ = ["get_rng_state", "set_rng_state", "register_rng_state_as_index"]

_INDEXED = []


def get_rng_state(device=None, use_index=False):
    """-> [state per generator]: the CPU generator, then one per GPU (or just ``device``'s)."""
    if device is None:
        states = [torch.get_rng_state()]
        if torch.cuda.is_available():
            states += [torch.cuda.get_rng_state(i) for i in range(torch.cuda.device_count())]
    elif str(device).startswith("gpu") or str(device).startswith("cuda"):
        idx = int(str(device).split(":")[1]) if ":" in str(device) else 0
        states = [torch.cuda.get_rng_state(idx)]
    else:
        states = [torch.get_rng_state()]
    if use_index:
        return [register_rng_state_as_index(s) for s in states]
    return states


def set_rng_state(state_list, device=None, use_index=False):
    states = [_INDEXED[i] for i in state_list] if use_index else list(state_list)
    if device is None:
        torch.set_rng_state(states[0])
        for i, s in enumerate(states[1:]):
            torch.cuda.set_rng_state(s, i)
    elif str(device).startswith("gpu") or str(device).startswith("cuda"):
        idx = int(str(device).split(":")[1]) if ":" in str(device) else 0
        torch.cuda.set_rng_state(states[0], idx)
    else:
        torch.set_rng_state(states[0])


def register_rng_state_as_index(state_list=None):
    """Keep a state and return its index (the reference's generator-state registry)."""
    s = torch.get_rng_state() if state_list is None else state_list
    _INDEXED.append(s.clone() if isinstance(s, torch.Tensor) else s)
    return len(_INDEXED) - 1
