"""paddle.incubate.autograd (reference: python/paddle/incubate/autograd/ — functional.py vjp / jvp / Jacobian /
Hessian, primapi.py forward_grad / grad, utils.py enable_prim / disable_prim / prim_enabled).

* ``vjp`` / ``jvp`` — functional products of a Python function over framework Tensors (reverse mode; the JVP by
  the double-backward trick: J v = d/du <u, J^T ...>, as the reference's ``_double_backward_trick``);
* ``Jacobian`` / ``Hessian`` — lazily evaluated, row-cached matrices with the reference's flattening rules:
  inputs and outputs are flattened and concatenated (per sample when ``is_batched``), indexing ``J[i, j]`` /
  ``J[:, i, j]`` evaluates only the rows it touches;
* ``forward_grad`` / ``grad`` — forward- and reverse-mode gradients of already computed outputs;
  ``enable_prim`` / ``disable_prim`` switch the primitive (decomposed) mode flag that ``paddle2_amd.decomposition``
  consults (static programs are lowered to primitives and differentiated by the primitive VJP rules).
"""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor

__all__ = ["vjp", "jvp", "Jacobian", "Hessian", "enable_prim", "disable_prim", "forward_grad", "grad",
           "prim_enabled"]

_PRIM = {"on": False}


def enable_prim():
    _PRIM["on"] = True


def disable_prim():
    _PRIM["on"] = False


def prim_enabled():
    return _PRIM["on"]


def _as_list(xs):
    return (list(xs), False) if isinstance(xs, (list, tuple)) else ([xs], True)


def _raw(x):
    return x._t if isinstance(x, Tensor) else x


def _prep_inputs(xs):
    """Fresh leaves that require grad (the function is re-run on them)."""
    lst, single = _as_list(xs)
    leaves = [_raw(x).detach().clone().requires_grad_(True) for x in lst]
    return leaves, single


def _call(func, leaves, single):
    args = [Tensor._wrap(t) for t in leaves]
    out = func(args[0]) if single else func(*args)
    outs, osingle = _as_list(out)
    return out, [_raw(o) for o in outs], osingle


def _grads(ys, xs, vs, create_graph=False):
    gs = torch.autograd.grad(ys, xs, vs, allow_unused=True, create_graph=create_graph)
    return [torch.zeros_like(x) if g is None else g for g, x in zip(gs, xs)]


def vjp(func, xs, v=None):
    """-> (func(xs), v^T J) — v defaults to ones like the outputs."""
    with torch.enable_grad():
        leaves, single = _prep_inputs(xs)
        out, ys, _ = _call(func, leaves, single)
        vs = [torch.ones_like(y) for y in ys] if v is None else [_raw(t) for t in _as_list(v)[0]]
        gs = _grads(ys, leaves, vs)
    res = [Tensor._wrap(g) for g in gs]
    return out, (res[0] if single else tuple(res))


def jvp(func, xs, v=None):
    """-> (func(xs), J v) — v defaults to ones like the inputs."""
    with torch.enable_grad():
        leaves, single = _prep_inputs(xs)
        out, ys, osingle = _call(func, leaves, single)
        vs = [torch.ones_like(x) for x in leaves] if v is None else [_raw(t) for t in _as_list(v)[0]]
        us = [torch.zeros_like(y, requires_grad=True) for y in ys]
        gx = torch.autograd.grad(ys, leaves, us, allow_unused=True, create_graph=True)
        pairs = [(g, vv) for g, vv in zip(gx, vs) if g is not None]
        if pairs:
            jv = torch.autograd.grad([g for g, _ in pairs], us, [vv for _, vv in pairs], allow_unused=True)
        else:
            jv = [None] * len(us)
    res = [Tensor._wrap(torch.zeros_like(y) if j is None else j.detach()) for j, y in zip(jv, ys)]
    return out, (res[0] if osingle else tuple(res))


class _Jac:
    """Row-lazy Jacobian of the flattened, concatenated outputs w.r.t. the flattened, concatenated inputs."""

    def __init__(self, func, xs, is_batched):
        self.batched = is_batched
        with torch.enable_grad():
            self.leaves, single = _prep_inputs(xs)
            _, ys, _ = _call(func, self.leaves, single)
        if is_batched:
            self.B = ys[0].shape[0]
            self.flat_y = torch.cat([y.reshape(self.B, -1) for y in ys], 1)
            self.nx = sum(x[0].numel() for x in self.leaves)
            self.shape = [self.B, self.flat_y.shape[1], self.nx]
        else:
            self.flat_y = torch.cat([y.reshape(-1) for y in ys])
            self.nx = sum(x.numel() for x in self.leaves)
            self.shape = [self.flat_y.numel(), self.nx]
        self._rows = {}

    def _row(self, i):
        r = self._rows.get(i)
        if r is None:
            with torch.enable_grad():
                tgt = self.flat_y[:, i].sum() if self.batched else self.flat_y[i]
                gs = torch.autograd.grad(tgt, self.leaves, retain_graph=True, allow_unused=True)
            gs = [torch.zeros_like(x) if g is None else g for g, x in zip(gs, self.leaves)]
            if self.batched:
                r = torch.cat([g.reshape(self.B, -1) for g in gs], 1)   # [B, nx]
            else:
                r = torch.cat([g.reshape(-1) for g in gs])              # [nx]
            self._rows[i] = r
        return r

    def __getitem__(self, idx):
        if not isinstance(idx, tuple):
            idx = (idx,)
        if any(i is Ellipsis for i in idx):
            raise IndexError("Ellipsis index is not supported")
        ax = 1 if self.batched else 0
        idx = idx + (slice(None),) * (len(self.shape) - len(idx))
        rows = range(self.shape[ax])[idx[ax]] if isinstance(idx[ax], slice) else [idx[ax] % self.shape[ax]]
        mats = torch.stack([self._row(i) for i in rows], ax)   # [.., len(rows), .., nx]
        sel = list(idx)
        sel[ax] = slice(None) if isinstance(idx[ax], slice) else 0
        return Tensor._wrap(mats[tuple(sel)].detach())


class Jacobian:
    """reference functional.py:214 — ``Jacobian(func, xs, is_batched=False)[index]``."""

    def __init__(self, func, xs, is_batched=False):
        self._jacobian = _Jac(func, xs, is_batched)

    def __getitem__(self, indexes):
        return self._jacobian[indexes]

    @property
    def shape(self):
        return list(self._jacobian.shape)


class Hessian(Jacobian):
    """reference functional.py:308 — the Jacobian of the gradient of a scalar (per sample when batched) func."""

    def __init__(self, func, xs, is_batched=False):
        def grad_fn(*args):
            with torch.enable_grad():
                raw = [_raw(a) for a in args]
                y = _raw(func(*args) if len(args) > 1 else func(args[0]))
                if (y.numel() if not is_batched else y.reshape(y.shape[0], -1).shape[1]) != 1:
                    raise ValueError("Hessian needs a scalar function (one value per sample when batched)")
                gs = torch.autograd.grad(y.sum(), raw, create_graph=True, allow_unused=True)
            gs = [torch.zeros_like(r) if g is None else g for g, r in zip(gs, raw)]
            if is_batched:
                return Tensor._wrap(torch.cat([g.reshape(g.shape[0], -1) for g in gs], 1))
            return Tensor._wrap(torch.cat([g.reshape(-1) for g in gs]))

        super().__init__(grad_fn, xs, is_batched)


def grad(outputs, inputs, grad_outputs=None):
    """Reverse-mode gradients of computed ``outputs`` w.r.t. ``inputs`` (reference primapi.grad)."""
    outs, _ = _as_list(outputs)
    ins, single = _as_list(inputs)
    gos = None if grad_outputs is None else [_raw(g) for g in _as_list(grad_outputs)[0]]
    ys = [_raw(o) for o in outs]
    if gos is None:
        gos = [torch.ones_like(y) for y in ys]
    gs = _grads(ys, [_raw(x) for x in ins], gos, create_graph=True)
    res = [Tensor._wrap(g) for g in gs]
    return res[0] if single else res


def forward_grad(outputs, inputs, grad_inputs=None):
    """Forward-mode (JVP) gradients of computed ``outputs`` along ``grad_inputs`` (ones by default) w.r.t.
    ``inputs`` (reference primapi.forward_grad), by the double-backward trick over the recorded graph."""
    outs, osingle = _as_list(outputs)
    ins, _ = _as_list(inputs)
    ys = [_raw(o) for o in outs]
    xs = [_raw(x) for x in ins]
    vs = [torch.ones_like(x) for x in xs] if grad_inputs is None else [_raw(g) for g in _as_list(grad_inputs)[0]]
    with torch.enable_grad():
        us = [torch.zeros_like(y, requires_grad=True) for y in ys]
        gx = torch.autograd.grad(ys, xs, us, allow_unused=True, create_graph=True, retain_graph=True)
        pairs = [(g, v) for g, v in zip(gx, vs) if g is not None]
        jv = torch.autograd.grad([g for g, _ in pairs], us, [v for _, v in pairs], allow_unused=True) if pairs \
            else [None] * len(us)
    res = [Tensor._wrap(torch.zeros_like(y) if j is None else j) for j, y in zip(jv, ys)]
    return res[0] if osingle else res
