"""L-BFGS (reference surface: python/paddle/optimizer/lbfgs.py ``LBFGS``: closure-driven ``step``,
``history_size``, ``tolerance_grad/change``, ``line_search_fn='strong_wolfe'``).

Implementation: two-loop recursion over a flat fp32 view of all parameters (one fused vector per
step instead of per-parameter lists — the direction, history and line search each run as a few
large device ops); strong-Wolfe line search with cubic interpolation (Nocedal & Wright, Alg. 3.5/3.6).
"""
from __future__ import annotations

import torch

from .optimizer import Optimizer


def _cubic_min(x1, f1, g1, x2, f2, g2, lo=None, hi=None):
    lo, hi = (min(x1, x2), max(x1, x2)) if lo is None else (lo, hi)
    d1 = g1 + g2 - 3 * (f1 - f2) / (x1 - x2)
    sq = d1 * d1 - g1 * g2
    if sq >= 0:
        d2 = sq ** 0.5
        if x1 <= x2:
            t = x2 - (x2 - x1) * ((g2 + d2 - d1) / (g2 - g1 + 2 * d2))
        else:
            t = x1 - (x1 - x2) * ((g1 + d2 - d1) / (g1 - g2 + 2 * d2))
        return min(max(t, lo), hi)
    return (lo + hi) / 2.0


def _strong_wolfe(obj, x, t, d, f, g, gtd, c1=1e-4, c2=0.9, tol_change=1e-9, max_ls=25):
    """Returns (f_new, g_new, t, n_evals)."""
    dmax = float(d.abs().max())
    f_new, g_new = obj(x, t, d)
    evals, gtd_new = 1, float(g_new.dot(d))
    t_prev, f_prev, g_prev, gtd_prev = 0.0, f, g, gtd
    done, it = False, 0
    while it < max_ls:
        if f_new > f + c1 * t * gtd or (it > 1 and f_new >= f_prev):
            br, brf, brg, brgtd = [t_prev, t], [f_prev, f_new], [g_prev, g_new.clone()], [gtd_prev, gtd_new]
            break
        if abs(gtd_new) <= -c2 * gtd:
            br, brf, brg = [t], [f_new], [g_new]
            done = True
            break
        if gtd_new >= 0:
            br, brf, brg, brgtd = [t_prev, t], [f_prev, f_new], [g_prev, g_new.clone()], [gtd_prev, gtd_new]
            break
        lo, hi = t + 0.01 * (t - t_prev), t * 10
        t_next = _cubic_min(t_prev, f_prev, gtd_prev, t, f_new, gtd_new, lo, hi)
        t_prev, f_prev, g_prev, gtd_prev = t, f_new, g_new.clone(), gtd_new
        t = t_next
        f_new, g_new = obj(x, t, d)
        evals += 1
        gtd_new = float(g_new.dot(d))
        it += 1
    else:
        br, brf, brg = [0.0, t], [f, f_new], [g, g_new]
        brgtd = [gtd, gtd_new]
    # zoom
    insuf = False
    lo_i, hi_i = (0, 1) if len(br) == 2 and brf[0] <= brf[-1] else (1, 0)
    while not done and it < max_ls and len(br) == 2:
        if abs(br[1] - br[0]) * dmax < tol_change:
            break
        t = _cubic_min(br[0], brf[0], brgtd[0], br[1], brf[1], brgtd[1])
        eps = 0.1 * (max(br) - min(br))
        if min(max(br) - t, t - min(br)) < eps:
            if insuf or t >= max(br) or t <= min(br):
                t = max(br) - eps if abs(t - max(br)) < abs(t - min(br)) else min(br) + eps
                insuf = False
            else:
                insuf = True
        else:
            insuf = False
        f_new, g_new = obj(x, t, d)
        evals += 1
        gtd_new = float(g_new.dot(d))
        it += 1
        if f_new > f + c1 * t * gtd or f_new >= brf[lo_i]:
            br[hi_i], brf[hi_i], brg[hi_i], brgtd[hi_i] = t, f_new, g_new.clone(), gtd_new
            lo_i, hi_i = (0, 1) if brf[0] <= brf[1] else (1, 0)
        else:
            if abs(gtd_new) <= -c2 * gtd:
                done = True
            elif gtd_new * (br[hi_i] - br[lo_i]) >= 0:
                br[hi_i], brf[hi_i], brg[hi_i], brgtd[hi_i] = br[lo_i], brf[lo_i], brg[lo_i], brgtd[lo_i]
            br[lo_i], brf[lo_i], brg[lo_i], brgtd[lo_i] = t, f_new, g_new.clone(), gtd_new
    i = 0 if len(br) == 1 else lo_i
    return brf[i], brg[i], br[i], evals


class LBFGS(Optimizer):
    def __init__(self, learning_rate=1.0, max_iter=20, max_eval=None, tolerance_grad=1e-7, tolerance_change=1e-9,
                 history_size=100, line_search_fn=None, parameters=None, weight_decay=None, grad_clip=None,
                 name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        if line_search_fn not in (None, "strong_wolfe"):
            raise ValueError(f"only 'strong_wolfe' line search is supported, got {line_search_fn!r}")
        self.max_iter = max_iter
        self.max_eval = max_eval if max_eval is not None else max_iter * 5 // 4
        self.tol_grad, self.tol_change = tolerance_grad, tolerance_change
        self.history_size, self.line_search_fn = history_size, line_search_fn
        self.state = {"func_evals": 0, "n_iter": 0}

    # flat views ---------------------------------------------------------------------------
    def _params(self):
        return [p for p in self._parameter_list if not p.stop_gradient]

    def _flat_grad(self):
        out = []
        for p in self._params():
            g = p._t.grad
            g = torch.zeros_like(p._t) if g is None else self._reg_grad(p, g)
            out.append(g.reshape(-1).float())
        return torch.cat(out)

    def _add(self, t, d):
        off = 0
        with torch.no_grad():
            for p in self._params():
                n = p._t.numel()
                p._t.add_(d[off:off + n].view_as(p._t).to(p._t.dtype), alpha=t)
                off += n

    def _get(self):
        return [p._t.detach().clone() for p in self._params()]

    def _set(self, vals):
        with torch.no_grad():
            for p, v in zip(self._params(), vals):
                p._t.copy_(v)

    def step(self, closure=None):
        if closure is None:
            raise ValueError("LBFGS.step needs a closure that clears grads, recomputes the loss and calls backward")

        def evaluate():
            with torch.enable_grad():
                loss = closure()
            return float(loss.detach() if hasattr(loss, "detach") else loss)

        st = self.state
        lr = self.get_lr()
        orig_loss = evaluate()
        f = orig_loss
        evals = 1
        st["func_evals"] += 1
        g = self._flat_grad()
        if float(g.abs().max()) <= self.tol_grad:
            return orig_loss
        d, t = st.get("d"), st.get("t")
        old_dirs, old_stps, ro = st.get("old_dirs", []), st.get("old_stps", []), st.get("ro", [])
        H_diag, prev_g, prev_f = st.get("H_diag", 1.0), st.get("prev_flat_grad"), st.get("prev_loss")
        n_iter = 0
        while n_iter < self.max_iter:
            n_iter += 1
            st["n_iter"] += 1
            if st["n_iter"] == 1:
                d, old_dirs, old_stps, ro, H_diag = -g, [], [], [], 1.0
            else:
                y = g - prev_g
                s = d * t
                ys = float(y.dot(s))
                if ys > 1e-10:
                    if len(old_dirs) == self.history_size:
                        old_dirs.pop(0), old_stps.pop(0), ro.pop(0)
                    old_dirs.append(y)
                    old_stps.append(s)
                    ro.append(1.0 / ys)
                    H_diag = ys / float(y.dot(y))
                q = -g
                al = [0.0] * len(old_dirs)
                for i in range(len(old_dirs) - 1, -1, -1):
                    al[i] = float(old_stps[i].dot(q)) * ro[i]
                    q.add_(old_dirs[i], alpha=-al[i])
                d = q * H_diag
                for i in range(len(old_dirs)):
                    be = float(old_dirs[i].dot(d)) * ro[i]
                    d.add_(old_stps[i], alpha=al[i] - be)
            prev_g = g.clone()
            prev_f = f
            t = min(1.0, 1.0 / float(g.abs().sum())) * lr if st["n_iter"] == 1 else lr
            gtd = float(g.dot(d))
            if gtd > -self.tol_change:
                break
            ls_evals = 0
            if self.line_search_fn == "strong_wolfe":
                x0 = self._get()

                def obj(x, step, direction):
                    self._add(step, direction)
                    fv = evaluate()
                    gv = self._flat_grad()
                    self._set(x)
                    return fv, gv

                f, g, t, ls_evals = _strong_wolfe(obj, x0, t, d, f, g, gtd, tol_change=self.tol_change)
                self._add(t, d)
            else:
                self._add(t, d)
                if n_iter != self.max_iter:
                    f = evaluate()
                    g = self._flat_grad()
                    ls_evals = 1
            evals += ls_evals
            st["func_evals"] += ls_evals
            if n_iter == self.max_iter or evals >= self.max_eval:
                break
            if float(g.abs().max()) <= self.tol_grad:
                break
            if float((d * t).abs().max()) <= self.tol_change or abs(f - prev_f) < self.tol_change:
                break
        st.update(d=d, t=t, old_dirs=old_dirs, old_stps=old_stps, ro=ro, H_diag=H_diag, prev_flat_grad=prev_g,
                  prev_loss=prev_f)
        self._step += 1
        return orig_loss

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        raise NotImplementedError("LBFGS needs a closure: call step(closure)")

    def state_dict(self):
        sd = super().state_dict()
        sd["lbfgs_state"] = {k: v for k, v in self.state.items() if isinstance(v, (int, float))}
        return sd
