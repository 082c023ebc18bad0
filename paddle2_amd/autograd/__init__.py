"""paddle.autograd (reference: python/paddle/autograd/ — grad, backward, PyLayer, saved_tensors_hooks).

The tape is torch's native autograd engine (C++, multithreaded); Paddle semantics are mapped on:
``paddle.grad`` -> ``torch.autograd.grad``; ``PyLayer`` -> ``torch.autograd.Function`` with a
context object exposing ``save_for_backward`` / ``saved_tensor()``.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor

_wrap = Tensor._wrap


def _u(x):
    return x._t if isinstance(x, Tensor) else x


def _w(x):
    if isinstance(x, torch.Tensor):
        return _wrap(x)
    if isinstance(x, (list, tuple)):
        return type(x)(_w(i) for i in x)
    return x


def grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False, only_inputs=True,
         allow_unused=False, no_grad_vars=None):
    single = isinstance(inputs, Tensor)
    outs = [outputs] if isinstance(outputs, Tensor) else list(outputs)
    ins = [inputs] if single else list(inputs)
    gos = None
    if grad_outputs is not None:
        gos = [grad_outputs] if isinstance(grad_outputs, Tensor) else list(grad_outputs)
        gos = [None if g is None else g._t for g in gos]
    res = torch.autograd.grad([o._t for o in outs], [i._t for i in ins], grad_outputs=gos,
                              retain_graph=retain_graph, create_graph=create_graph, allow_unused=True)
    if not allow_unused and any(r is None for r in res):
        raise ValueError("some inputs are unreachable from outputs; set allow_unused=True")
    res = [None if r is None else _wrap(r) for r in res]
    return res


def backward(tensors, grad_tensors=None, retain_graph=False):
    ts = [tensors] if isinstance(tensors, Tensor) else list(tensors)
    gs = None
    if grad_tensors is not None:
        gs = [grad_tensors] if isinstance(grad_tensors, Tensor) else list(grad_tensors)
        gs = [None if g is None else g._t for g in gs]
    torch.autograd.backward([t._t for t in ts], gs, retain_graph=retain_graph)


class PyLayerContext:
    def __init__(self, tctx):
        object.__setattr__(self, "_tctx", tctx)
        object.__setattr__(self, "_saved", ())
        object.__setattr__(self, "_non_diff", set())
        object.__setattr__(self, "_materialize", True)

    def save_for_backward(self, *tensors):
        object.__setattr__(self, "_saved", tensors)
        ts = [t._t for t in tensors if isinstance(t, Tensor)]
        self._tctx.save_for_backward(*ts)

    def saved_tensor(self):
        ts = list(self._tctx.saved_tensors)
        out = []
        for t in self._saved:
            out.append(_wrap(ts.pop(0)) if isinstance(t, Tensor) else t)
        return tuple(out)

    saved_tensors = property(saved_tensor)

    def mark_not_inplace(self, *args):
        pass

    def mark_non_differentiable(self, *tensors):
        self._tctx.mark_non_differentiable(*[t._t for t in tensors])

    def set_materialize_grads(self, value):
        self._tctx.set_materialize_grads(value)

    def __setattr__(self, k, v):
        object.__setattr__(self, k, v)


class _PyLayerMeta(type):
    """Builds one torch.autograd.Function per PyLayer subclass (reference: eager/pylayer/)."""

    def __init__(cls, name, bases, attrs):
        super().__init__(name, bases, attrs)
        if name == "PyLayer":
            return
        user = cls

        class _Fn(torch.autograd.Function):
            @staticmethod
            def forward(tctx, kwargs, *args):
                tctx._n_inputs = len(args)
                ctx = PyLayerContext(tctx)
                tctx._pctx = ctx
                wargs = [_wrap(a) if isinstance(a, torch.Tensor) else a for a in args]
                out = user.forward(ctx, *wargs, **kwargs)
                tctx._multi = isinstance(out, (tuple, list))
                outs = out if tctx._multi else (out,)
                res = tuple(o._t if isinstance(o, Tensor) else o for o in outs)
                return res if tctx._multi else res[0]

            @staticmethod
            def backward(tctx, *grads):
                ctx = tctx._pctx
                wg = [None if g is None else _wrap(g) for g in grads]
                r = user.backward(ctx, *wg)
                rs = r if isinstance(r, (tuple, list)) else (r,)
                out = [None if x is None else (x._t if isinstance(x, Tensor) else x) for x in rs]
                n_in = tctx._n_inputs
                out = out[:n_in] + [None] * max(0, n_in - len(out))
                return (None,) + tuple(out)

        cls._fn = _Fn


class PyLayer(metaclass=_PyLayerMeta):
    @staticmethod
    def forward(ctx, *args, **kwargs):
        raise NotImplementedError

    @staticmethod
    def backward(ctx, *args):
        raise NotImplementedError

    @classmethod
    def apply(cls, *args, **kwargs):
        targs = [a._t if isinstance(a, Tensor) else a for a in args]
        out = cls._fn.apply(kwargs, *targs)
        if isinstance(out, tuple):
            return tuple(_wrap(o) if isinstance(o, torch.Tensor) else o for o in out)
        return _wrap(out) if isinstance(out, torch.Tensor) else out


LegacyPyLayer = PyLayer
EagerPyLayer = PyLayer


class saved_tensors_hooks:
    def __init__(self, pack_hook, unpack_hook):
        self._cm = torch.autograd.graph.saved_tensors_hooks(lambda t: pack_hook(_wrap(t)),
                                                            lambda x: _u(unpack_hook(x)))

    def __enter__(self):
        self._cm.__enter__()
        return self

    def __exit__(self, *a):
        return self._cm.__exit__(*a)


def jacobian(ys, xs, batch_axis=None):
    """Dense Jacobian of ``ys`` w.r.t. ``xs`` (reference: autograd/autograd.py jacobian)."""
    single_x = isinstance(xs, Tensor)
    xs_l = [xs] if single_x else list(xs)
    y = ys._t.reshape(-1)
    rows = []
    for i in range(y.numel()):
        g = torch.autograd.grad(y[i], [x._t for x in xs_l], retain_graph=True, allow_unused=True)
        rows.append([torch.zeros_like(x._t).reshape(-1) if gi is None else gi.reshape(-1) for gi, x in zip(g, xs_l)])
    jac = [_wrap(torch.stack([r[j] for r in rows])) for j in range(len(xs_l))]
    return jac[0] if single_x else jac


def hessian(ys, xs, batch_axis=None):
    """Hessian of scalar ``ys`` w.r.t. a single ``xs`` by double backward (xs must be a leaf in ys' graph)."""
    x = xs._t
    (g,) = torch.autograd.grad(ys._t.reshape(()), [x], create_graph=True)
    g = g.reshape(-1)
    rows = [torch.autograd.grad(g[i], [x], retain_graph=True, allow_unused=True)[0] for i in range(g.numel())]
    rows = [torch.zeros_like(x) if r is None else r for r in rows]
    return _wrap(torch.stack([r.reshape(-1) for r in rows]))


def no_grad(func=None):
    from ..framework.grad_mode import no_grad as _ng

    return _ng()(func) if func is not None else _ng()
