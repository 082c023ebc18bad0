"""NaN/Inf checker (reference: paddle/fluid/eager/nan_inf_utils.cc:84 ``CheckTensorHasNanOrInf``,
``FLAGS_check_nan_inf`` / ``FLAGS_check_nan_inf_level`` flags.cc:79).

The reference scans every op output inside the generated ``<op>_ad_func``.  Here two granularities run
together when the flag is on:
  * per OP: a torch dispatch mode sees every ATen kernel the program runs — forward AND backward ops
    (autograd's backward kernels dispatch through it too) — and scans each floating output, naming the
    op (``aten.mm.default``) that produced the first NaN/Inf;
  * per LAYER: every ``Layer.__call__`` output is scanned and a gradient hook scans the gradient flowing
    back into it, which also covers the fused HIP nodes (their kernels write into buffers the dispatch mode
    only sees allocated, so freshly allocated ``empty`` outputs are never scanned).

Levels (reference semantics): 0 = raise on the first NaN/Inf; 1 = log and continue;
2 = also log fp32 stats (min/max/mean) of offending tensors; 3 = log stats of every checked tensor.
Off (the default) costs one module-level bool test per layer call.
"""
from __future__ import annotations

import sys

import torch

enabled = False
level = 0
_log = []   # (where, name, n_nan, n_inf) records for levels >= 1


def _sync_from_flags():
    global enabled, level
    from . import flags

    enabled = bool(flags.flag("FLAGS_check_nan_inf", False))
    level = int(flags.flag("FLAGS_check_nan_inf_level", 0))
    _set_op_mode(enabled)


_SKIP = ("empty", "empty_like", "empty_strided", "new_empty", "new_empty_strided", "set_", "_local_scalar_dense",
         "isfinite", "isnan", "isinf", "detach", "alias", "view", "_to_copy", "lift_fresh", "lift",
         "lift_fresh_copy", "scalar_tensor", "copy_", "clone")  # allocation / data-movement, not compute


def _make_mode():
    from torch.utils._python_dispatch import TorchDispatchMode

    class _OpChecker(TorchDispatchMode):
        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            out = func(*args, **(kwargs or {}))
            name = func.overloadpacket.__name__
            if name not in _SKIP and not _busy[0]:
                _busy[0] = True
                try:
                    phase = "backward op" if torch._C._current_graph_task_id() != -1 else "op"
                    for i, t in enumerate(_tensors(out)):
                        if t.device.type != "meta":
                            check_tensor(t, f"{phase} {func}", f"output[{i}]")
                finally:
                    _busy[0] = False
            return out

    return _OpChecker()


_mode = [None]
_busy = [False]


def _set_op_mode(on):
    if on and _mode[0] is None:
        m = _make_mode()
        m.__enter__()
        _mode[0] = m
    elif not on and _mode[0] is not None:
        m, _mode[0] = _mode[0], None
        m.__exit__(None, None, None)


def _tensors(out):
    from .tensor import Tensor

    if isinstance(out, Tensor):
        yield out._t
    elif isinstance(out, torch.Tensor):
        yield out
    elif isinstance(out, (list, tuple)):
        for o in out:
            yield from _tensors(o)
    elif isinstance(out, dict):
        for o in out.values():
            yield from _tensors(o)


def check_tensor(t: torch.Tensor, where: str, name: str = ""):
    if not (t.is_floating_point() or t.is_complex()) or t.numel() == 0:
        return
    ok = bool(torch.isfinite(t).all())
    if ok and level < 3:
        return
    n_nan = int(torch.isnan(t).sum()) if not ok else 0
    n_inf = int(torch.isinf(t).sum()) if not ok else 0
    msg = f"[check_nan_inf] {where} {name}: shape={list(t.shape)} dtype={t.dtype} nan={n_nan} inf={n_inf}"
    if level >= 2 or (level >= 3 and ok):
        f = t.float()
        fin = f[torch.isfinite(f)]
        if fin.numel():
            msg += f" min={float(fin.min()):.4g} max={float(fin.max()):.4g} mean={float(fin.mean()):.4g}"
    if not ok and level == 0:
        raise RuntimeError(msg + " (set FLAGS_check_nan_inf_level>=1 to log instead of raising)")
    _log.append((where, name, n_nan, n_inf))
    print(msg, file=sys.stderr)


def check_layer(layer, out):
    lname = getattr(layer, "_full_name", None) or type(layer).__name__
    for i, t in enumerate(_tensors(out)):
        check_tensor(t, f"forward {lname}", f"output[{i}]")
        if t.requires_grad:
            t.register_hook(lambda g, _n=lname, _i=i: (check_tensor(g, f"backward {_n}", f"grad(output[{_i}])"),
                                                        None)[1])


def records():
    return list(_log)
