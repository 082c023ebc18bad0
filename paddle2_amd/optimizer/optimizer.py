"""Optimizers (reference: python/paddle/optimizer/{optimizer,adamw,adam,sgd,momentum,...}.py).

State-dict layout follows Paddle: one entry per accumulator named ``{param.name}_{acc}_0``
(``moment1``, ``moment2``, ``beta1_pow_acc``, ``beta2_pow_acc``, ``velocity`` ...), plus
``master_weights`` and ``LR_Scheduler``.  On the MI355X the Adam family runs as ONE fused
multi-tensor HIP launch per dtype group (csrc/kernels/optim.hip) instead of the reference's one
``adamw_`` launch per parameter (adamw.py:495).
"""
from __future__ import annotations

import collections
import math

import numpy as np
import torch

from ..framework.tensor import Tensor
from ..ops import _native as N
from .lr import LRScheduler
from ..framework.tensor_types import SelectedRows
from .multi_tensor import MultiTensorTable, aligned16

_wrap = Tensor._wrap


from ..regularizer import L1Decay, L2Decay, as_regularizer  # noqa: E402,F401  (re-exported by paddle.optimizer)


def _grad_of(p):
    mg = getattr(p, "main_grad", None)
    if mg is not None:
        return mg._t if isinstance(mg, Tensor) else mg
    return p._t.grad


class Optimizer:
    _acc_names = ()

    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None, name=None):
        if parameters is None:
            raise ValueError("parameters must be given in dygraph mode")
        params = list(parameters)
        if params and isinstance(params[0], dict):
            self._param_groups = []
            for g in params:
                g = dict(g)
                g["params"] = list(g["params"])
                self._param_groups.append(g)
        else:
            self._param_groups = [{"params": params}]
        self._parameter_list = [p for g in self._param_groups for p in g["params"]]
        self._learning_rate = learning_rate
        self.regularization = weight_decay
        self._grad_clip = grad_clip
        self._name = name
        self._accumulators = collections.defaultdict(dict)   # acc name -> {param name: torch.Tensor}
        self._master_weights = {}                             # param name -> fp32 torch.Tensor
        self._step = 0
        self._multi_precision = False
        self._mt_cache = None

    # ------------------------------------------------------------ lr
    def get_lr(self):
        lr = self._learning_rate
        return float(lr()) if isinstance(lr, LRScheduler) else float(lr)

    def set_lr(self, value):
        if isinstance(self._learning_rate, LRScheduler):
            raise RuntimeError("optimizer's learning rate is an LRScheduler; call scheduler.step() instead")
        self._learning_rate = float(value)

    def set_lr_scheduler(self, scheduler):
        self._learning_rate = scheduler

    # ------------------------------------------------------------ grads
    def clear_grad(self, set_to_zero=True):
        for p in self._parameter_list:
            if getattr(p, "main_grad", None) is not None:
                if set_to_zero:
                    (p.main_grad._t if isinstance(p.main_grad, Tensor) else p.main_grad).zero_()
                else:
                    p.main_grad = None
            g = p._t.grad
            if g is None:
                continue
            if set_to_zero and getattr(p, "_keep_grad_storage", False):
                g.zero_()  # grad is a view into a communication bucket: keep the storage
            else:
                # Lazy zero: drop the buffer so the next backward's AccumulateGrad adopts the fresh
                # gradient instead of launching a fill now and a read-modify-write add later (one
                # fill + one add per parameter per step); reading ``p.grad`` before that backward
                # materialises zeros, so set_to_zero semantics are unchanged.
                p._t.grad = None
                p._lazy_zero_grad = bool(set_to_zero)

    clear_gradients = clear_grad

    def _params_grads(self):
        out = []
        for p in self._parameter_list:
            if p.stop_gradient and getattr(p, "main_grad", None) is None:
                continue
            g = _grad_of(p)
            if g is None:
                continue
            out.append((p, _wrap(g)))
        return out

    def _group_of(self, p):
        for g in self._param_groups:
            for q in g["params"]:
                if q is p:
                    return g
        return self._param_groups[0]

    # ------------------------------------------------------------ accumulators
    def _acc(self, name, p, like=None, dtype=torch.float32, fill=0.0):
        d = self._accumulators[name]
        t = d.get(p.name)
        if t is None:
            ref = p._t if like is None else like
            t = torch.full_like(ref, fill, dtype=dtype)  # DistTensor params get DistTensor state
            d[p.name] = t
        return t

    def _master(self, p):
        if p._t.dtype in (torch.float16, torch.bfloat16) and self._multi_precision:
            m = self._master_weights.get(p.name)
            if m is None:
                m = p._t.detach().float().clone()
                self._master_weights[p.name] = m
            return m
        return None

    # ------------------------------------------------------------ step
    _fused_clip = False  # optimizers that consume a device-side clip coefficient in their update pass

    @torch.no_grad()
    def step(self):
        from ..profiler import _host_on, host_range

        if _host_on:
            with host_range(f"{type(self).__name__}.step", 4):
                return self._step_impl()
        return self._step_impl()

    def _step_impl(self):
        pg = self._params_grads()
        self._clip_coef = None
        sparse = [(p, g) for p, g in pg if g._t.is_sparse]
        if sparse:
            # row-sparse (SelectedRows) gradients, e.g. nn.Embedding(sparse=True): clipping needs the dense
            # norm, otherwise only the touched rows are updated
            pg = [(p, g) for p, g in pg if not g._t.is_sparse]
            if self._grad_clip is not None:
                pg += [(p, _wrap(g._t.to_dense())) for p, g in sparse]
                sparse = []
        if self._grad_clip is not None and pg:
            if self._fused_clip and getattr(self._grad_clip, "_fusable", False) and all(
                    g._t.device.type == "cuda" for _, g in pg):
                self._clip_coef = self._grad_clip.global_coef(pg)
                if self._clip_coef is None:
                    pg = self._grad_clip(pg)
            else:
                pg = self._grad_clip(pg)
        self._step += 1
        if pg:
            self._apply(pg)
        for p, g in sparse:
            self._apply_sparse(p, SelectedRows.from_torch_sparse(g._t).merge_add())

    def _apply_sparse(self, p, sr):
        """Update from a SelectedRows gradient; the default densifies it (exact for every optimizer)."""
        self._apply([(p, _wrap(sr.to_dense()))])

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from ..static.graph import SymTensor

        if isinstance(getattr(loss, "_t", None), SymTensor):
            # static graph: record backward + this optimizer's update into the loss's Program
            from .. import static as _static

            pg = _static.append_backward(loss, parameter_list=parameters)
            loss._t._program.append_special("optimize", optimizer=self)
            return [], pg
        pg = self._params_grads()
        self.step()
        return None, pg

    def _reg_grad(self, p, g):
        reg = as_regularizer(getattr(p, "regularizer", None) or self.regularization)
        return g if reg is None else reg.decay(p._t, g)

    def _apply(self, params_grads):
        raise NotImplementedError

    # ------------------------------------------------------------ state
    def state_dict(self):
        sd = collections.OrderedDict()
        for acc, d in self._accumulators.items():
            for pname, t in d.items():
                sd[f"{pname}_{acc}_0"] = _wrap(t)
        self._extra_state(sd)
        if self._master_weights:
            sd["master_weights"] = {k: _wrap(v) for k, v in self._master_weights.items()}
        if isinstance(self._learning_rate, LRScheduler):
            sd["LR_Scheduler"] = self._learning_rate.state_dict()
        return sd

    def _extra_state(self, sd):
        pass

    def set_state_dict(self, state_dict):
        names = {p.name: p for p in self._parameter_list}
        for k, v in state_dict.items():
            if k == "master_weights":
                for pn, t in v.items():
                    self._master_weights[pn] = _to_torch(t, names[pn]._t.device if pn in names else None).float()
                continue
            if k == "LR_Scheduler":
                if isinstance(self._learning_rate, LRScheduler):
                    self._learning_rate.set_state_dict(v)
                continue
            for pn, p in names.items():
                if k.startswith(pn + "_") and k.endswith("_0"):
                    acc = k[len(pn) + 1: -2]
                    self._load_acc(acc, p, _to_torch(v, p._t.device))
                    break
        self._mt_cache = None

    set_dict = set_state_dict

    def _load_acc(self, acc, p, t):
        self._accumulators[acc][p.name] = t.float() if t.is_floating_point() else t


def _to_torch(v, device):
    if isinstance(v, Tensor):
        t = v._t
    elif isinstance(v, np.ndarray):
        t = torch.from_numpy(np.ascontiguousarray(v))
    elif isinstance(v, torch.Tensor):
        t = v
    else:
        t = torch.as_tensor(v)
    return t.to(device) if device is not None else t


# ============================================================================== SGD / Momentum
class SGD(Optimizer):
    def __init__(self, learning_rate=0.001, parameters=None, weight_decay=None, grad_clip=None, multi_precision=False,
                 name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._multi_precision = multi_precision

    def _apply(self, pg):
        lr = self.get_lr()
        for p, g in pg:
            gl = self._group_of(p).get("learning_rate", 1.0) * p.optimize_attr.get("learning_rate", 1.0) \
                if hasattr(p, "optimize_attr") else 1.0
            gt = self._reg_grad(p, g._t)
            m = self._master(p)
            if m is not None:
                m.add_(gt.float(), alpha=-lr * gl)
                p._t.copy_(m)
            else:
                p._t.add_(gt.to(p._t.dtype), alpha=-lr * gl)

    def _apply_sparse(self, p, sr):
        """w[rows] -= lr * value: one index_add over the touched rows (reference sgd SelectedRows kernel)."""
        if (getattr(p, "regularizer", None) or self.regularization) is not None:
            return super()._apply_sparse(p, sr)
        lr = self.get_lr()
        gl = self._group_of(p).get("learning_rate", 1.0) * p.optimize_attr.get("learning_rate", 1.0) \
            if hasattr(p, "optimize_attr") else 1.0
        rows = sr._rows.to(p._t.device)
        m = self._master(p)
        tgt = m if m is not None else p._t
        tgt.index_add_(0, rows, sr._value.to(tgt.dtype), alpha=-lr * gl)
        if m is not None:
            p._t.copy_(m)


class Momentum(Optimizer):
    def __init__(self, learning_rate=0.001, momentum=0.9, parameters=None, use_nesterov=False, weight_decay=None,
                 grad_clip=None, multi_precision=False, rescale_grad=1.0, use_multi_tensor=False, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._momentum, self._nesterov, self._rescale = momentum, use_nesterov, rescale_grad
        self._multi_precision = multi_precision

    def _apply(self, pg):
        lr = self.get_lr()
        for p, g in pg:
            gt = self._reg_grad(p, g._t).float() * self._rescale
            v = self._acc("velocity", p)
            v.mul_(self._momentum).add_(gt)
            upd = gt + self._momentum * v if self._nesterov else v
            m = self._master(p)
            tgt = m if m is not None else p._t
            tgt.add_(upd.to(tgt.dtype), alpha=-lr)
            if m is not None:
                p._t.copy_(m)


# ============================================================================== Adam family
class Adam(Optimizer):
    """Adam with L2 ``weight_decay`` folded into the gradient (paddle semantics)."""

    _decoupled = False
    _fused_clip = True

    def _grad_mult(self):
        """Device scalar multiplying every gradient in the update: AMP 1/scale x global-norm clip coef."""
        a, b = self._inv_scale, getattr(self, "_clip_coef", None)
        if a is None:
            return b
        if b is None:
            return a
        return a * b

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None, weight_decay=None,
                 grad_clip=None, lazy_mode=False, multi_precision=False, use_multi_tensor=False, amsgrad=False,
                 name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._beta1, self._beta2, self._epsilon = float(beta1), float(beta2), float(epsilon)
        self._multi_precision = multi_precision
        self._amsgrad = amsgrad
        self._lazy_mode = lazy_mode
        self._found_inf = None   # set by GradScaler for fused skip
        self._inv_scale = None
        # L2 regularisation is added after clipping in Paddle, so it cannot share the fused multiplier
        self._fused_clip = weight_decay is None

    # per-parameter decoupled-decay coefficient and lr ratio
    def _decay_of(self, p):
        return 0.0

    def _lr_ratio_of(self, p):
        r = p.optimize_attr.get("learning_rate", 1.0) if hasattr(p, "optimize_attr") else 1.0
        return r * self._group_of(p).get("learning_rate", 1.0)

    def _apply(self, pg):
        lr = self.get_lr()
        b1, b2 = self._beta1, self._beta2
        bc1 = 1.0 - b1 ** self._step
        bc2 = 1.0 - b2 ** self._step
        if not self._decoupled and self.regularization is not None:
            pg = [(p, _wrap(self._reg_grad(p, g._t))) for p, g in pg]
        gpu = [(p, g) for p, g in pg if g._t.device.type == "cuda" and N.use_native(g._t)]
        cpu = [(p, g) for p, g in pg if not (g._t.device.type == "cuda" and N.use_native(g._t))]
        if gpu:
            self._apply_fused(gpu, lr, b1, b2, bc1, bc2)
        for p, g in cpu:
            self._apply_ref(p, g._t, lr, b1, b2, bc1, bc2)

    def _apply_sparse(self, p, sr):
        """lazy_mode: moments and weights of the touched rows only (reference adam SelectedRows kernel with
        lazy_mode); otherwise the dense update (untouched rows still decay their moments)."""
        if not self._lazy_mode or self._amsgrad or (not self._decoupled and self.regularization is not None):
            return super()._apply_sparse(p, sr)
        lr = self.get_lr()
        b1, b2 = self._beta1, self._beta2
        bc1, bc2 = 1.0 - b1 ** self._step, 1.0 - b2 ** self._step
        rows = sr._rows.to(p._t.device)
        m1 = self._acc("moment1", p)
        m2 = self._acc("moment2", p)
        g = sr._value.float()
        mult = self._grad_mult()
        if mult is not None:
            g = g * mult.to(g.device)
        r1 = m1.index_select(0, rows).mul_(b1).add_(g, alpha=1 - b1)
        r2 = m2.index_select(0, rows).mul_(b2).addcmul_(g, g, value=1 - b2)
        m1.index_copy_(0, rows, r1)
        m2.index_copy_(0, rows, r2)
        lr_t = lr * self._lr_ratio_of(p)
        mw = self._master(p)
        tgt = mw if mw is not None else p._t
        w = tgt.index_select(0, rows).float()
        w = w * (1 - lr_t * self._decay_of(p)) - (lr_t / bc1) * r1 / (r2.sqrt() / math.sqrt(bc2) + self._epsilon)
        tgt.index_copy_(0, rows, w.to(tgt.dtype))
        if mw is not None:
            p._t.copy_(mw)

    def _apply_ref(self, p, g, lr, b1, b2, bc1, bc2):
        m1 = self._acc("moment1", p)
        m2 = self._acc("moment2", p)
        gf = g.float()
        mult = self._grad_mult()
        if mult is not None:
            gf = gf * mult.to(gf.device)
        m1.mul_(b1).add_(gf, alpha=1 - b1)
        m2.mul_(b2).addcmul_(gf, gf, value=1 - b2)
        lr_t = lr * self._lr_ratio_of(p)
        mw = self._master(p)
        tgt = mw if mw is not None else p._t
        if self._amsgrad:
            mx = self._acc("moment2_max", p)
            torch.maximum(mx, m2, out=mx)
            denom = mx.sqrt() / math.sqrt(bc2) + self._epsilon
        else:
            denom = m2.sqrt() / math.sqrt(bc2) + self._epsilon
        upd = tgt.float() * (1 - lr_t * self._decay_of(p)) - (lr_t / bc1) * m1 / denom
        tgt.copy_(upd.to(tgt.dtype))
        if mw is not None:
            p._t.copy_(mw)

    def _apply_fused(self, pg, lr, b1, b2, bc1, bc2):
        if self._amsgrad or any(not aligned16(p._t) or not aligned16(g._t) for p, g in pg):
            for p, g in pg:
                self._apply_ref(p, g._t, lr, b1, b2, bc1, bc2)
            return
        key = tuple((id(p), g._t.data_ptr(), p._t.data_ptr()) for p, g in pg)
        if self._mt_cache is None or self._mt_cache[0] != key:
            groups = collections.OrderedDict()
            for p, g in pg:
                m = self._master(p)
                k = (p._t.dtype, g._t.dtype, m is not None)
                groups.setdefault(k, []).append((p, g, m))
            tables = []
            for (pdt, gdt, has_m), items in groups.items():
                if (pdt, gdt) not in ((torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16),
                                      (torch.bfloat16, torch.float32), (torch.float16, torch.float16),
                                      (torch.float16, torch.float32), (torch.float32, torch.bfloat16)):
                    tables.append(("ref", items))
                    continue
                ps = [p._t for p, g, m in items]
                gs = [g._t for p, g, m in items]
                m1 = [self._acc("moment1", p) for p, g, m in items]
                m2 = [self._acc("moment2", p) for p, g, m in items]
                ms = [m for p, g, m in items] if has_m else None
                lrr = [self._lr_ratio_of(p) for p, g, m in items]
                dec = [self._decay_of(p) for p, g, m in items]
                tables.append(("mt", MultiTensorTable(ps, gs, m1, m2, ms, lrr, dec)))
            self._mt_cache = (key, tables)
        mult = self._grad_mult()
        for kind, tab in self._mt_cache[1]:
            if kind == "mt":
                tab.adamw(lr, b1, b2, self._epsilon, bc1, bc2, self._found_inf, mult)
            else:
                for p, g, m in tab:
                    self._apply_ref(p, g._t, lr, b1, b2, bc1, bc2)

    def _extra_state(self, sd):
        for p in self._parameter_list:
            if p.name in self._accumulators.get("moment1", {}):
                dev = self._accumulators["moment1"][p.name].device
                sd[f"{p.name}_beta1_pow_acc_0"] = _wrap(torch.tensor([self._beta1 ** self._step], device=dev))
                sd[f"{p.name}_beta2_pow_acc_0"] = _wrap(torch.tensor([self._beta2 ** self._step], device=dev))

    def _load_acc(self, acc, p, t):
        if acc == "beta1_pow_acc":
            v = float(t.reshape(-1)[0])
            if 0 < v < 1:
                self._step = int(round(math.log(v) / math.log(self._beta1)))
            return
        if acc == "beta2_pow_acc":
            return
        super()._load_acc(acc, p, t)


class AdamW(Adam):
    """AdamW with decoupled decay, ``lr_ratio`` and ``apply_decay_param_fun`` (adamw.py)."""

    _decoupled = True

    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None, weight_decay=0.01,
                 lr_ratio=None, apply_decay_param_fun=None, grad_clip=None, lazy_mode=False, multi_precision=False,
                 amsgrad=False, name=None):
        super().__init__(learning_rate, beta1, beta2, epsilon, parameters, None, grad_clip, lazy_mode, multi_precision,
                         amsgrad=amsgrad, name=name)
        if isinstance(weight_decay, Tensor):
            weight_decay = float(weight_decay.item())
        self._coeff = 0.0 if weight_decay is None else float(weight_decay)
        self._lr_ratio = lr_ratio
        self._apply_decay_param_fun = apply_decay_param_fun

    def _decay_of(self, p):
        g = self._group_of(p)
        coeff = float(g.get("weight_decay", self._coeff))
        if self._apply_decay_param_fun is not None and not self._apply_decay_param_fun(p.name):
            return 0.0
        return coeff

    def _lr_ratio_of(self, p):
        r = super()._lr_ratio_of(p)
        if self._lr_ratio is not None:
            r *= float(self._lr_ratio(p))
        return r


class Adamax(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1e-8, parameters=None, weight_decay=None,
                 grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon

    def _apply(self, pg):
        lr = self.get_lr()
        for p, g in pg:
            gt = self._reg_grad(p, g._t).float()
            m = self._acc("moment", p)
            u = self._acc("inf_norm", p)
            m.mul_(self._b1).add_(gt, alpha=1 - self._b1)
            torch.maximum(u * self._b2, gt.abs() + self._eps, out=u)
            p._t.add_((m / u).to(p._t.dtype), alpha=-lr / (1 - self._b1 ** self._step))


class Adagrad(Optimizer):
    def __init__(self, learning_rate, epsilon=1e-6, parameters=None, weight_decay=None, grad_clip=None, name=None,
                 initial_accumulator_value=0.0):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._eps, self._init = epsilon, initial_accumulator_value

    def _apply(self, pg):
        lr = self.get_lr()
        for p, g in pg:
            gt = self._reg_grad(p, g._t).float()
            m = self._acc("moment", p, fill=self._init)
            m.addcmul_(gt, gt)
            p._t.add_((gt / (m.sqrt() + self._eps)).to(p._t.dtype), alpha=-lr)


class RMSProp(Optimizer):
    def __init__(self, learning_rate, rho=0.95, epsilon=1e-6, momentum=0.0, centered=False, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._rho, self._eps, self._mom, self._centered = rho, epsilon, momentum, centered

    def _apply(self, pg):
        lr = self.get_lr()
        for p, g in pg:
            gt = self._reg_grad(p, g._t).float()
            ms = self._acc("mean_square", p)
            mom = self._acc("momentum", p)
            ms.mul_(self._rho).addcmul_(gt, gt, value=1 - self._rho)
            if self._centered:
                mg = self._acc("mean_grad", p)
                mg.mul_(self._rho).add_(gt, alpha=1 - self._rho)
                denom = (ms - mg * mg + self._eps).sqrt()
            else:
                denom = (ms + self._eps).sqrt()
            mom.mul_(self._mom).add_(gt / denom, alpha=lr)
            p._t.sub_(mom.to(p._t.dtype))


class Adadelta(Optimizer):
    def __init__(self, learning_rate=0.001, epsilon=1.0e-6, rho=0.95, parameters=None, weight_decay=None,
                 grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._eps, self._rho = epsilon, rho

    def _apply(self, pg):
        lr = self.get_lr()
        for p, g in pg:
            gt = self._reg_grad(p, g._t).float()
            ag = self._acc("avg_squared_grad", p)
            au = self._acc("avg_squared_update", p)
            ag.mul_(self._rho).addcmul_(gt, gt, value=1 - self._rho)
            upd = -((au + self._eps).sqrt() / (ag + self._eps).sqrt()) * gt
            au.mul_(self._rho).addcmul_(upd, upd, value=1 - self._rho)
            p._t.add_(upd.to(p._t.dtype), alpha=lr)


class Lamb(Optimizer):
    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6,
                 parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None, multi_precision=False,
                 always_adapt=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name)
        self._wd, self._b1, self._b2, self._eps = lamb_weight_decay, beta1, beta2, epsilon
        self._exclude = exclude_from_weight_decay_fn
        self._multi_precision = multi_precision
        self._always_adapt = always_adapt

    def _apply(self, pg):
        lr = self.get_lr()
        for p, g in pg:
            gt = g._t.float()
            m = self._acc("moment1", p)
            v = self._acc("moment2", p)
            m.mul_(self._b1).add_(gt, alpha=1 - self._b1)
            v.mul_(self._b2).addcmul_(gt, gt, value=1 - self._b2)
            mh = m / (1 - self._b1 ** self._step)
            vh = v / (1 - self._b2 ** self._step)
            mw = self._master(p)
            w = mw if mw is not None else p._t.float()
            wd = 0.0 if (self._exclude is not None and self._exclude(p)) else self._wd
            r = mh / (vh.sqrt() + self._eps) + wd * w
            wn, rn = torch.linalg.vector_norm(w), torch.linalg.vector_norm(r)
            trust = torch.where((wn > 0) & (rn > 0), wn / rn, torch.ones_like(wn))
            neww = w - lr * trust * r
            if mw is not None:
                mw.copy_(neww)
            p._t.copy_(neww.to(p._t.dtype))


class NAdam(Optimizer):
    def __init__(self, learning_rate=0.002, beta1=0.9, beta2=0.999, epsilon=1.0e-8, momentum_decay=0.004,
                 parameters=None, weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps, self._md = beta1, beta2, epsilon, momentum_decay
        self._mu_prod = 1.0

    def _apply(self, pg):
        lr = self.get_lr()
        t = self._step
        mu = self._b1 * (1 - 0.5 * 0.96 ** (t * self._md))
        mu_next = self._b1 * (1 - 0.5 * 0.96 ** ((t + 1) * self._md))
        self._mu_prod *= mu
        for p, g in pg:
            gt = self._reg_grad(p, g._t).float()
            m = self._acc("moment1", p)
            v = self._acc("moment2", p)
            m.mul_(self._b1).add_(gt, alpha=1 - self._b1)
            v.mul_(self._b2).addcmul_(gt, gt, value=1 - self._b2)
            vh = v / (1 - self._b2 ** t)
            upd = (mu_next * m / (1 - self._mu_prod * mu_next) + (1 - mu) * gt / (1 - self._mu_prod)) / (vh.sqrt() + self._eps)
            p._t.add_(upd.to(p._t.dtype), alpha=-lr)


class RAdam(Optimizer):
    def __init__(self, learning_rate=0.001, beta1=0.9, beta2=0.999, epsilon=1.0e-8, parameters=None,
                 weight_decay=None, grad_clip=None, name=None):
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._b1, self._b2, self._eps = beta1, beta2, epsilon

    def _apply(self, pg):
        lr = self.get_lr()
        t = self._step
        rho_inf = 2 / (1 - self._b2) - 1
        rho_t = rho_inf - 2 * t * self._b2 ** t / (1 - self._b2 ** t)
        for p, g in pg:
            gt = self._reg_grad(p, g._t).float()
            m = self._acc("moment1", p)
            v = self._acc("moment2", p)
            m.mul_(self._b1).add_(gt, alpha=1 - self._b1)
            v.mul_(self._b2).addcmul_(gt, gt, value=1 - self._b2)
            mh = m / (1 - self._b1 ** t)
            if rho_t > 5:
                r = math.sqrt((rho_t - 4) * (rho_t - 2) * rho_inf / ((rho_inf - 4) * (rho_inf - 2) * rho_t))
                upd = r * mh * math.sqrt(1 - self._b2 ** t) / (v.sqrt() + self._eps)
            else:
                upd = mh
            p._t.add_(upd.to(p._t.dtype), alpha=-lr)


class ASGD(Optimizer):
    """Averaged SGD over a window of ``batch_num`` gradients (reference: optimizer/asgd.py:239,
    phi/kernels/cpu/asgd_kernel.cc): ``d += g - y[m % n]``, ``y[m % n] = g``,
    ``p -= lr / min(m + 1, n) * d``."""

    def __init__(self, learning_rate=0.001, batch_num=1, parameters=None, weight_decay=None, grad_clip=None,
                 multi_precision=False, name=None):
        if batch_num is None or batch_num <= 0:
            raise ValueError("batch_num should be a positive integer")
        super().__init__(learning_rate, parameters, weight_decay, grad_clip, name)
        self._n = int(batch_num)
        self._multi_precision = multi_precision

    def _apply(self, pg):
        lr = self.get_lr()
        for p, g in pg:
            gt = self._reg_grad(p, g._t).float()
            d = self._acc("d", p)
            m = self._acc("m", p, like=torch.zeros(1, device=p._t.device))
            ys = self._accumulators["y"].get(p.name)
            if ys is None:
                ys = torch.zeros((self._n,) + tuple(p._t.shape), dtype=torch.float32, device=p._t.device)
                self._accumulators["y"][p.name] = ys
            idx = int(m.item()) % self._n
            m.add_(1)
            d.sub_(ys[idx]).add_(gt)
            ys[idx].copy_(gt)
            mw = self._master(p)
            tgt = mw if mw is not None else p._t
            tgt.sub_((d * (lr / min(float(m.item()), self._n))).to(tgt.dtype))
            if mw is not None:
                p._t.copy_(mw)


class Rprop(Optimizer):
    def __init__(self, learning_rate=0.001, learning_rate_range=(1e-5, 50), parameters=None, etas=(0.5, 1.2),
                 grad_clip=None, multi_precision=False, name=None):
        super().__init__(learning_rate, parameters, None, grad_clip, name)
        self._range, self._etas = learning_rate_range, etas

    def _apply(self, pg):
        for p, g in pg:
            gt = g._t.float()
            prev = self._acc("prev", p)
            lrs = self._acc("learning_rate", p, fill=self.get_lr())
            s = gt * prev
            lrs.copy_(torch.where(s > 0, lrs * self._etas[1], torch.where(s < 0, lrs * self._etas[0], lrs)).clamp(*self._range))
            gt = torch.where(s < 0, torch.zeros_like(gt), gt)
            p._t.sub_((torch.sign(gt) * lrs).to(p._t.dtype))
            prev.copy_(gt)
