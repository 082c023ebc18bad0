"""Activation recomputation (reference: fleet/recompute/recompute.py — ``RecomputeFunction`` :124
(reentrant PyLayer with RNG replay :112), non-reentrant path via ``saved_tensors_hooks``
:319-449, ``recompute`` :455, ``recompute_sequential`` :622; recompute_hybrid.py:265).

Two implementations on the torch autograd tape:

* reentrant: a ``torch.autograd.Function`` runs the block under ``no_grad`` and saves only its
  inputs; backward restores the forward RNG state (CPU + current HIP device), re-runs the block
  with grad enabled and back-propagates through the fresh sub-graph (param grads accumulate as
  a side effect, exactly like Paddle's reentrant recompute);
* non-reentrant (default in Paddle ≥2.5 when ``use_reentrant=False``): saved-tensor hooks replace
  every activation the block saves with a slot index; the first unpack in backward replays the
  block once under the recorded RNG state, refilling the slots in the same order.

The RNG replay covers dropout inside the block, and the fleet RNG tracker states are replayed
too so TP-local dropout masks match between the two passes.
"""
from __future__ import annotations

import contextlib

import torch

from ....framework.place import current_torch_device
from ....framework.tensor import Tensor

_wrap = Tensor._wrap


def _is_t(x):
    return isinstance(x, Tensor)


class _RngSnapshot:
    def __init__(self, preserve):
        self.preserve = preserve
        if not preserve:
            return
        self.cpu = torch.get_rng_state()
        d = current_torch_device()
        self.dev = d
        self.gpu = torch.cuda.get_rng_state(d.index) if d.type == "cuda" else None
        from ..layers.mpu.random import get_rng_state_tracker

        self.tracker = get_rng_state_tracker().get_states_tracker()

    @contextlib.contextmanager
    def replay(self):
        if not self.preserve:
            yield
            return
        from ..layers.mpu.random import get_rng_state_tracker

        tr = get_rng_state_tracker()
        cpu, gpu, trk = torch.get_rng_state(), (
            torch.cuda.get_rng_state(self.dev.index) if self.gpu is not None else None), tr.get_states_tracker()
        torch.set_rng_state(self.cpu)
        if self.gpu is not None:
            torch.cuda.set_rng_state(self.gpu, self.dev.index)
        tr.set_states_tracker(self.tracker)
        try:
            yield
        finally:
            torch.set_rng_state(cpu)
            if gpu is not None:
                torch.cuda.set_rng_state(gpu, self.dev.index)
            tr.set_states_tracker(trk)


def _flatten_out(out):
    """Tensor | tuple/list of (Tensor | other) -> (list of torch tensors, rebuild fn)."""
    if _is_t(out):
        return [out._t], lambda ts: _wrap(ts[0])
    if isinstance(out, (tuple, list)):
        idx = [i for i, o in enumerate(out) if _is_t(o)]

        def rebuild(ts, out=out, idx=idx):
            lst = list(out)
            for i, t in zip(idx, ts):
                lst[i] = _wrap(t)
            return type(out)(lst) if isinstance(out, tuple) else lst

        return [out[i]._t for i in idx], rebuild
    raise TypeError("recompute: function must return Tensor(s)")


class _RecomputeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, run, preserve, n_args, *flat):
        # flat = tensor args (torch) in positional order; non-tensors are baked into ``run``
        ctx.run = run
        ctx.rng = _RngSnapshot(preserve)
        ctx.save_for_backward(*flat)
        with torch.no_grad():
            outs = run(*flat)
        ctx.n_out = len(outs)
        return tuple(o.detach() if isinstance(o, torch.Tensor) else o for o in outs)

    @staticmethod
    def backward(ctx, *grads):
        inputs = ctx.saved_tensors
        det = []
        for x in inputs:
            d = x.detach()
            d.requires_grad_(x.requires_grad)
            det.append(d)
        with ctx.rng.replay(), torch.enable_grad():
            outs = ctx.run(*det)
        pairs = [(o, g) for o, g in zip(outs, grads) if isinstance(o, torch.Tensor) and o.requires_grad and g is not None]
        if pairs:
            torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
        return (None, None, None) + tuple(d.grad if d.requires_grad else None for d in det)


def _recompute_reentrant(function, preserve, args, kwargs):
    t_pos = [i for i, a in enumerate(args) if _is_t(a)]
    holder = {}

    def run(*ts):
        a = list(args)
        for i, t in zip(t_pos, ts):
            a[i] = _wrap(t)
        out = function(*a, **kwargs)
        flat, rebuild = _flatten_out(out)
        holder["rebuild"] = rebuild
        return flat

    outs = _RecomputeFn.apply(run, preserve, len(t_pos), *[args[i]._t for i in t_pos])
    return holder["rebuild"](list(outs))


def _recompute_non_reentrant(function, preserve, args, kwargs):
    rng = _RngSnapshot(preserve)
    slots: list = []
    state = {"done": False}

    def replay():
        inner = []

        def ipack(x):
            inner.append(x)
            return len(inner) - 1

        def iunpack(i):
            return inner[i]

        with rng.replay(), torch.enable_grad(), torch.autograd.graph.saved_tensors_hooks(ipack, iunpack):
            a = [(_wrap(x._t.detach().requires_grad_(x._t.requires_grad)) if _is_t(x) else x) for x in args]
            function(*a, **kwargs)
        slots[:] = inner
        state["done"] = True

    counter = [0]

    def pack(x):
        i = counter[0]
        counter[0] += 1
        return i

    def unpack(i):
        if not state["done"]:
            replay()
        return slots[i]

    with torch.autograd.graph.saved_tensors_hooks(pack, unpack):
        return function(*args, **kwargs)


def recompute(function, *args, **kwargs):
    """paddle.distributed.fleet.utils.recompute(function, *args, preserve_rng_state=True,
    use_reentrant=True, **kwargs)."""
    preserve = kwargs.pop("preserve_rng_state", True)
    use_reentrant = kwargs.pop("use_reentrant", True)
    kwargs.pop("offload_indices", None)
    if not torch.is_grad_enabled():
        return function(*args, **kwargs)
    if use_reentrant:
        return _recompute_reentrant(function, preserve, args, kwargs)
    return _recompute_non_reentrant(function, preserve, args, kwargs)


def recompute_sequential(ctx, functions, *args, **kwargs):
    """Split a Sequential into ``ctx['segments']`` chunks and recompute each (recompute.py:622)."""
    segments = int(ctx.get("segments", 1))
    preserve = ctx.get("preserve_rng_state", True)
    layers = list(functions.children()) if hasattr(functions, "children") else list(functions)
    per = (len(layers) + segments - 1) // segments

    def run_seg(lo, hi):
        def f(x):
            for l in layers[lo:hi]:
                x = l(x)
            return x

        return f

    x = args[0] if len(args) == 1 else args
    for s in range(0, len(layers), per):
        hi = min(s + per, len(layers))
        if hi == len(layers):
            for l in layers[s:hi]:
                x = l(x)
        else:
            x = recompute(run_seg(s, hi), x, preserve_rng_state=preserve, **kwargs)
    return x


def recompute_hybrid(ctx, function, *args, **kwargs):
    """Hybrid-parallel recompute (recompute_hybrid.py:265).  The reference optionally partitions the
    saved inputs across the mp group and offloads them to host; with 288 GB of HBM per MI355X we keep
    them resident and recompute in place."""
    kwargs.setdefault("preserve_rng_state", True)
    return recompute(function, *args, **kwargs)
