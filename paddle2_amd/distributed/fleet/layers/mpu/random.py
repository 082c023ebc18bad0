"""Model-parallel RNG tracker (reference: fleet/layers/mpu/random.py — ``RNGStatesTracker``,
``get_rng_state_tracker``, ``model_parallel_random_seed``, ``dropout`` with ``rng_name``).

Each named state is a private torch Philox generator state for the current device.  Inside
``tracker.rng_state(name)`` the device generator is swapped to that state and swapped back on
exit, so dropout inside TP-sharded regions (``"local_seed"``, different per mp rank) stays
decorrelated while replicated regions (``"global_seed"``, identical on the mp group) match.
"""
from __future__ import annotations

import contextlib

import numpy as np
import torch

from .....framework import random as _R
from .....framework.place import current_torch_device

MODEL_PARALLEL_RNG = "model_parallel_rng"


def _dev_get_state():
    d = current_torch_device()
    if d.type == "cuda":
        return torch.cuda.get_rng_state(d.index)
    return torch.get_rng_state()


def _dev_set_state(s):
    d = current_torch_device()
    if d.type == "cuda":
        torch.cuda.set_rng_state(s, d.index)
    else:
        torch.set_rng_state(s)


def _dev_seed(seed):
    d = current_torch_device()
    if d.type == "cuda":
        torch.cuda.manual_seed(seed)
    else:
        torch.manual_seed(seed)


class RNGStatesTracker:
    def __init__(self):
        self.states_ = {}
        self.seeds_ = set()

    def reset(self):
        self.states_ = {}
        self.seeds_ = set()

    def add(self, name, seed):
        if seed in self.seeds_:
            raise ValueError(f"seed {seed} already exists")
        if name in self.states_:
            raise ValueError(f"state {name} already exists")
        self.seeds_.add(seed)
        orig = _dev_get_state()
        _dev_seed(seed)
        self.states_[name] = _dev_get_state()
        _dev_set_state(orig)

    def get_states_tracker(self):
        return {k: v.clone() for k, v in self.states_.items()}

    def set_states_tracker(self, states):
        self.states_ = {k: v.clone() for k, v in states.items()}

    @contextlib.contextmanager
    def rng_state(self, name=MODEL_PARALLEL_RNG):
        if name not in self.states_:
            raise ValueError(f"state {name} does not exist")
        orig = _dev_get_state()
        _dev_set_state(self.states_[name])
        try:
            yield
        finally:
            self.states_[name] = _dev_get_state()
            _dev_set_state(orig)


_RNG_STATE_TRACKER = RNGStatesTracker()


def get_rng_state_tracker():
    return _RNG_STATE_TRACKER


def model_parallel_random_seed(seed=None):
    """Global seed identical across mp ranks; local seed distinct per mp rank (random.py:98)."""
    from ..... import distributed as dist
    from .... import fleet

    hcg = fleet.get_hybrid_communicate_group()
    rank = hcg.get_model_parallel_rank() if hcg is not None else 0
    pp_rank = hcg.get_stage_id() if hcg is not None else 0
    if seed:
        global_seed = seed
        local_seed = seed * 1024 + rank * 100 + pp_rank
    else:
        global_seed = np.random.randint(0, 10000) if dist.get_world_size() == 1 else 2048
        local_seed = global_seed + 1024 + rank * 100 + pp_rank * 7
    _RNG_STATE_TRACKER.reset()
    _RNG_STATE_TRACKER.add(MODEL_PARALLEL_RNG, local_seed)
    _RNG_STATE_TRACKER.add("global_seed", global_seed)
    _RNG_STATE_TRACKER.add("local_seed", local_seed + 1)
    _R.seed(global_seed)


def determinate_seed(rng_name):
    assert rng_name is not None and rng_name != ""
    return int(torch.randint(0, 2**31 - 1, (1,)).item())


def dropout(x, p=0.5, axis=None, rng_name=None, training=True, mode="upscale_in_train", name=None):
    """Dropout drawing from a named tracker state (random.py:144)."""
    from .....nn import functional as F

    if rng_name is None or not training or p == 0.0:
        return F.dropout(x, p, axis, training, mode)
    with _RNG_STATE_TRACKER.rng_state(rng_name):
        return F.dropout(x, p, axis, training, mode)
