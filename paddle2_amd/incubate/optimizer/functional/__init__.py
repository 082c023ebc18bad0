"""paddle.incubate.optimizer.functional: minimize_bfgs / minimize_lbfgs (reference:
python/paddle/incubate/optimizer/functional/{bfgs,lbfgs,line_search,utils}.py).

Functional quasi-Newton minimisers of ``objective_func(x) -> scalar`` over a 1-D position: the gradient comes from
autograd, the step from a strong-Wolfe line search (the cubic-interpolation search shared with
``paddle.optimizer.LBFGS``), BFGS keeps the dense inverse-Hessian estimate H (Nocedal & Wright Alg. 6.1: H+ =
(I - rho s y^T) H (I - rho y s^T) + rho s s^T), L-BFGS the last ``history_size`` (s, y) pairs and the two-loop
recursion (Alg. 7.4 / 7.5).  Results follow the reference tuples:

    minimize_bfgs  -> (is_converge, num_func_calls, position, objective_value, objective_gradient,
                       inverse_hessian_estimate)
    minimize_lbfgs -> (is_converge, num_func_calls, position, objective_value, objective_gradient)
"""
from __future__ import annotations

import torch

from ....framework.tensor import Tensor
from ....optimizer.lbfgs import _strong_wolfe

__all__ = ["minimize_bfgs", "minimize_lbfgs"]


def _dtype(dtype):
    if dtype not in ("float32", "float64"):
        raise ValueError(f"dtype must be 'float32' or 'float64', got {dtype!r}")
    return torch.float32 if dtype == "float32" else torch.float64


def _value_and_grad(f, x):
    """f at x (a 1-D torch tensor) and its gradient, the objective seeing a framework Tensor."""
    with torch.enable_grad():
        xv = x.detach().clone().requires_grad_(True)
        y = f(Tensor._wrap(xv))
        yt = y._t if isinstance(y, Tensor) else torch.as_tensor(y)
        if yt.numel() != 1:
            raise ValueError("objective_func must return a scalar")
        (g,) = torch.autograd.grad(yt.reshape(()), xv)
    return yt.detach().reshape(()).to(x.dtype), g.detach().to(x.dtype)


def _check(line_search_fn, x0):
    if line_search_fn != "strong_wolfe":
        raise NotImplementedError("only line_search_fn='strong_wolfe' is supported (as in the reference)")
    if x0.dim() != 1:
        raise ValueError("initial_position must be a 1-D tensor")


def _search(f, x, d, fx, g, step, max_ls, tol_change):
    calls = [0]

    def obj(x_, t, d_):
        calls[0] += 1
        v, gg = _value_and_grad(f, x_ + t * d_)
        return float(v), gg

    gtd = float(g.dot(d))
    f_new, g_new, t, _ = _strong_wolfe(obj, x, step, d, float(fx), g, gtd, tol_change=tol_change, max_ls=max_ls)
    return torch.as_tensor(f_new, dtype=x.dtype, device=x.device), g_new, t, calls[0]


def minimize_bfgs(objective_func, initial_position, max_iters=50, tolerance_grad=1e-7, tolerance_change=1e-9,
                  initial_inverse_hessian_estimate=None, line_search_fn="strong_wolfe", max_line_search_iters=50,
                  initial_step_length=1.0, dtype="float32", name=None):
    dt = _dtype(dtype)
    x = (initial_position._t if isinstance(initial_position, Tensor) else torch.as_tensor(initial_position))
    x = x.detach().to(dt)
    _check(line_search_fn, x)
    n = x.numel()
    if initial_inverse_hessian_estimate is None:
        H = torch.eye(n, dtype=dt, device=x.device)
    else:
        H = initial_inverse_hessian_estimate
        H = (H._t if isinstance(H, Tensor) else torch.as_tensor(H)).to(dt).clone()
        if not torch.allclose(H, H.t()) or bool((torch.linalg.eigvalsh(H) <= 0).any()):
            raise ValueError("initial_inverse_hessian_estimate must be symmetric positive definite")
    fx, g = _value_and_grad(objective_func, x)
    calls, converged = 1, bool(g.abs().max() <= tolerance_grad)
    eye = torch.eye(n, dtype=dt, device=x.device)
    for _ in range(max_iters):
        if converged:
            break
        d = -(H @ g)
        f_new, g_new, t, c = _search(objective_func, x, d, fx, g, initial_step_length, max_line_search_iters,
                                     tolerance_change)
        calls += c
        s = t * d
        y = g_new - g
        x = x + s
        change = float(s.abs().max())
        fx, g = f_new, g_new
        if bool(g.abs().max() <= tolerance_grad):
            converged = True
            break
        if change <= tolerance_change:
            converged = True
            break
        ys = float(y.dot(s))
        if ys > 0:
            rho = 1.0 / ys
            V = eye - rho * torch.outer(s, y)
            H = V @ H @ V.t() + rho * torch.outer(s, s)
    w = Tensor._wrap
    return (w(torch.tensor(converged)), w(torch.tensor(calls)), w(x), w(fx), w(g), w(H))


def minimize_lbfgs(objective_func, initial_position, history_size=100, max_iters=50, tolerance_grad=1e-8,
                   tolerance_change=1e-8, initial_inverse_hessian_estimate=None, line_search_fn="strong_wolfe",
                   max_line_search_iters=50, initial_step_length=1.0, dtype="float32", name=None):
    dt = _dtype(dtype)
    x = (initial_position._t if isinstance(initial_position, Tensor) else torch.as_tensor(initial_position))
    x = x.detach().to(dt)
    _check(line_search_fn, x)
    H0 = None
    if initial_inverse_hessian_estimate is not None:
        H0 = initial_inverse_hessian_estimate
        H0 = (H0._t if isinstance(H0, Tensor) else torch.as_tensor(H0)).to(dt)
        if not torch.allclose(H0, H0.t()) or bool((torch.linalg.eigvalsh(H0) <= 0).any()):
            raise ValueError("initial_inverse_hessian_estimate must be symmetric positive definite")
    fx, g = _value_and_grad(objective_func, x)
    calls, converged = 1, bool(g.abs().max() <= tolerance_grad)
    S, Y, R = [], [], []
    for _ in range(max_iters):
        if converged:
            break
        # two-loop recursion: d = -H_k g
        q = g.clone()
        alphas = []
        for s, y, rho in zip(reversed(S), reversed(Y), reversed(R)):
            a = rho * float(s.dot(q))
            alphas.append(a)
            q = q - a * y
        if H0 is not None:
            r = H0 @ q
        elif S:
            r = q * (float(S[-1].dot(Y[-1])) / float(Y[-1].dot(Y[-1])))
        else:
            r = q
        for (s, y, rho), a in zip(zip(S, Y, R), reversed(alphas)):
            b = rho * float(y.dot(r))
            r = r + s * (a - b)
        d = -r
        f_new, g_new, t, c = _search(objective_func, x, d, fx, g, initial_step_length, max_line_search_iters,
                                     tolerance_change)
        calls += c
        s = t * d
        y = g_new - g
        x = x + s
        change = float(s.abs().max())
        fx, g = f_new, g_new
        if bool(g.abs().max() <= tolerance_grad) or change <= tolerance_change:
            converged = True
            break
        ys = float(y.dot(s))
        if ys > 0:
            S.append(s)
            Y.append(y)
            R.append(1.0 / ys)
            if len(S) > history_size:
                S.pop(0)
                Y.pop(0)
                R.pop(0)
    w = Tensor._wrap
    return (w(torch.tensor(converged)), w(torch.tensor(calls)), w(x), w(fx), w(g))
