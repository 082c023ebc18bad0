"""paddle.amp: auto_cast (O1/O2), decorate, GradScaler (reference: python/paddle/amp/).

* ``auto_cast`` O1 casts inputs of white-list ops (matmul/linear/conv/attention) to the AMP dtype
  via torch's autocast on the ROCm device (bf16 by default on MI355X); O2 assumes parameters were
  cast by :func:`decorate` and keeps fp32 master weights in the optimizer (``multi_precision``).
* ``GradScaler`` runs ``check_finite_and_unscale`` as ONE multi-tensor HIP launch per grad dtype
  and hands ``found_inf`` / ``inv_scale`` device pointers to the fused AdamW kernel, so the
  skip-on-overflow decision never syncs the host (reference: grad_scaler.py:426, amp_kernel.cu).
"""
from __future__ import annotations

import contextlib

import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor

_amp_state = {"enable": False, "level": "O0", "dtype": torch.bfloat16, "white": frozenset(), "black": frozenset()}

# Default op lists (reference python/paddle/amp/amp_lists.py): white ops run in the AMP dtype, black ops
# in fp32.  torch.autocast applies the equivalent defaults to the ATen ops underneath; the lists matter
# for the ops the user moves with custom_white_list / custom_black_list, which ``amp_op`` enforces at
# this framework's op entry points (nn.functional / tensor APIs decorated with @amp_op).
WHITE_LIST = {"matmul", "linear", "conv2d", "conv1d", "conv3d", "einsum", "bmm", "mm", "flash_attn",
              "scaled_dot_product_attention"}
BLACK_LIST = {"exp", "log", "softmax", "log_softmax", "cross_entropy", "layer_norm", "batch_norm", "reduce_sum",
              "sum", "mean"}


def _effective_lists(custom_white, custom_black):
    cw, cb = set(custom_white or ()), set(custom_black or ()),
    if cw & cb:
        raise ValueError(f"auto_cast: ops in both custom_white_list and custom_black_list: {sorted(cw & cb)}")
    return frozenset((WHITE_LIST | cw) - cb), frozenset((BLACK_LIST | cb) - cw)


def op_policy(name):
    """'low' (run in the AMP dtype), 'fp32', or None (leave it to autocast) for op ``name`` now."""
    st = _amp_state
    if not st["enable"] or st["level"] not in ("O1", "O2"):
        return None
    if name in st["black"]:
        return "fp32"
    if name in st["white"]:
        return "low"
    return None


def amp_op(name):
    """Decorator for an op entry point: enforce the current auto_cast op lists for op ``name``
    (the custom lists override torch.autocast's built-in choice for that op)."""
    import functools

    def deco(fn):
        @functools.wraps(fn)
        def inner(*args, **kw):
            pol = op_policy(name)
            if pol is None:
                return fn(*args, **kw)
            dt = torch.float32 if pol == "fp32" else _amp_state["dtype"]

            def cast(a):
                t = a._t if isinstance(a, Tensor) else a
                if isinstance(t, torch.Tensor) and t.is_floating_point() and t.dtype != dt:
                    t = t.to(dt)
                    return Tensor._wrap(t) if isinstance(a, Tensor) else t
                return a

            args = tuple(cast(a) for a in args)
            kw = {k: cast(v) for k, v in kw.items()}
            from ..framework.place import current_torch_device

            with torch.autocast(device_type=current_torch_device().type, enabled=False):
                return fn(*args, **kw)

        return inner

    return deco


def is_float16_supported(device=None):
    return True


def is_bfloat16_supported(device=None):
    return True


def amp_state():
    return dict(_amp_state)


@contextlib.contextmanager
def auto_cast(enable=True, custom_white_list=None, custom_black_list=None, level="O1", dtype="bfloat16",
              use_promote=True):
    dt = _dt.convert_dtype(dtype)
    prev = dict(_amp_state)
    white, black = _effective_lists(custom_white_list, custom_black_list)
    _amp_state.update(enable=enable, level=level, dtype=dt, white=white, black=black)
    from ..framework.place import current_torch_device

    dev = current_torch_device().type
    try:
        if enable and level in ("O1", "O2"):
            with torch.autocast(device_type=dev, dtype=dt, enabled=True):
                yield
        else:
            yield
    finally:
        _amp_state.clear()
        _amp_state.update(prev)


amp_guard = auto_cast


def decorate(models, optimizers=None, level="O1", dtype="bfloat16", master_weight=None, save_dtype=None,
             master_grad=False, excluded_layers=None):
    """O2: cast model parameters to the AMP dtype (norm layers stay fp32) and enable master weights."""
    from ..nn import BatchNorm, BatchNorm1D, BatchNorm2D, BatchNorm3D, LayerNorm

    dt = _dt.convert_dtype(dtype)
    single_model = not isinstance(models, (list, tuple))
    ms = [models] if single_model else list(models)
    if level == "O2":
        keep = (BatchNorm, BatchNorm1D, BatchNorm2D, BatchNorm3D, LayerNorm)
        if excluded_layers is not None:
            ex = excluded_layers if isinstance(excluded_layers, (list, tuple)) else [excluded_layers]
            keep = keep + tuple(e for e in ex if isinstance(e, type))
        for m in ms:
            for l in m.sublayers(include_self=True):
                if isinstance(l, keep):
                    continue
                for k, p in l._parameters.items():
                    if p is not None and p._t.is_floating_point():
                        with torch.no_grad():
                            rg = p._t.requires_grad
                            p._t = p._t.detach().to(dt).requires_grad_(rg)
            m._casted_by_pure_fp16 = True
        if optimizers is not None:
            opts = optimizers if isinstance(optimizers, (list, tuple)) else [optimizers]
            for o in opts:
                o._multi_precision = True if master_weight is None else bool(master_weight)
                o._mt_cache = None
    if optimizers is None:
        return models if single_model else ms
    return (models if single_model else ms), optimizers


class GradScaler:
    """Dynamic loss scaling (reference: python/paddle/amp/grad_scaler.py:657)."""

    def __init__(self, enable=True, init_loss_scaling=2.0 ** 15, incr_ratio=2.0, decr_ratio=0.5,
                 incr_every_n_steps=1000, decr_every_n_nan_or_inf=2, use_dynamic_loss_scaling=True):
        self._enable = enable
        self._incr_ratio, self._decr_ratio = incr_ratio, decr_ratio
        self._incr_every_n, self._decr_every_n = incr_every_n_steps, decr_every_n_nan_or_inf
        self._dynamic = use_dynamic_loss_scaling
        from ..framework.place import current_torch_device

        dev = current_torch_device()
        self._scale = torch.tensor([float(init_loss_scaling)], dtype=torch.float32, device=dev)
        self._found_inf = torch.zeros(1, dtype=torch.float32, device=dev)
        self._good = torch.zeros(1, dtype=torch.int32, device=dev)
        self._bad = torch.zeros(1, dtype=torch.int32, device=dev)
        self._unscaled = False
        self._tables = None

    def is_enable(self):
        return self._enable

    def is_use_dynamic_loss_scaling(self):
        return self._dynamic

    def get_init_loss_scaling(self):
        return float(self._scale.item())

    def set_init_loss_scaling(self, v):
        self._scale.fill_(float(v))

    def scale(self, var):
        if not self._enable:
            return var
        return Tensor._wrap(var._t * self._scale.to(var._t.dtype))

    def _grads(self, optimizer):
        from ..optimizer.optimizer import _grad_of

        return [g for g in (_grad_of(p) for p in optimizer._parameter_list) if g is not None]

    def unscale_(self, optimizer):
        if not self._enable or self._unscaled:
            return
        self._found_inf.zero_()
        grads = self._grads(optimizer)
        if grads and grads[0].device.type == "cuda":
            from ..optimizer.multi_tensor import MultiTensorTable

            key = tuple(g.data_ptr() for g in grads)
            if self._tables is None or self._tables[0] != key:
                by_dt = {}
                for g in grads:
                    by_dt.setdefault(g.dtype, []).append(g)
                self._tables = (key, [MultiTensorTable.for_grads(gs) for gs in by_dt.values()])
            for t in self._tables[1]:
                t.unscale(self._scale, self._found_inf)
        else:
            inv = 1.0 / self._scale
            for g in grads:
                g.mul_(inv.to(g.dtype))
                if not torch.isfinite(g).all():
                    self._found_inf.fill_(1.0)
        self._unscaled = True

    def minimize(self, optimizer, *args, **kwargs):
        return self.step(optimizer)

    def step(self, optimizer):
        if not self._enable:
            return optimizer.step()
        self.unscale_(optimizer)
        # fused optimizers read found_inf on device and skip; others consult it (host sync)
        from ..optimizer.optimizer import Adam

        if isinstance(optimizer, Adam):
            optimizer._found_inf = self._found_inf
            try:
                optimizer.step()
            finally:
                optimizer._found_inf = None
        else:
            if float(self._found_inf.item()) == 0.0:
                optimizer.step()
            else:
                optimizer._step += 0
        self._unscaled = False

    def update(self):
        if not self._enable or not self._dynamic:
            return
        if self._scale.device.type == "cuda":
            from ..ops import _native as N

            N.require().update_loss_scaling(self._found_inf.data_ptr(), self._scale.data_ptr(), self._good.data_ptr(),
                                            self._bad.data_ptr(), self._incr_every_n, self._decr_every_n,
                                            self._incr_ratio, self._decr_ratio, N.stream())
        else:
            if float(self._found_inf.item()) != 0.0:
                self._good.zero_()
                self._bad += 1
                if int(self._bad.item()) == self._decr_every_n:
                    self._scale.mul_(self._decr_ratio).clamp_(min=1.0)
                    self._bad.zero_()
            else:
                self._bad.zero_()
                self._good += 1
                if int(self._good.item()) == self._incr_every_n:
                    self._scale.mul_(self._incr_ratio)
                    self._good.zero_()

    def state_dict(self):
        return {"scale": Tensor._wrap(self._scale.clone()), "incr_ratio": self._incr_ratio,
                "decr_ratio": self._decr_ratio, "incr_every_n_steps": self._incr_every_n,
                "decr_every_n_nan_or_inf": self._decr_every_n, "incr_count": int(self._good.item()),
                "decr_count": int(self._bad.item()), "use_dynamic_loss_scaling": self._dynamic}

    def load_state_dict(self, sd):
        self._scale.copy_(sd["scale"]._t if isinstance(sd["scale"], Tensor) else torch.as_tensor(sd["scale"]))
        self._good.fill_(int(sd.get("incr_count", 0)))
        self._bad.fill_(int(sd.get("decr_count", 0)))

    set_state_dict = load_state_dict


AmpScaler = GradScaler


class debugging:
    """paddle.amp.debugging — tensor checker (reference: amp/debugging.py:173)."""

    @staticmethod
    def check_numerics(tensor, op_type="", var_name="", debug_mode=None):
        t = tensor._t
        n_nan = int(torch.isnan(t).sum())
        n_inf = int(torch.isinf(t).sum())
        if n_nan or n_inf:
            raise RuntimeError(f"[check_numerics] {op_type}:{var_name} has {n_nan} NaN and {n_inf} Inf")
        return tensor

    @staticmethod
    def enable_tensor_checker(config=None):
        from ..framework import flags

        flags.set_flags({"FLAGS_check_nan_inf": True})

    @staticmethod
    def disable_tensor_checker():
        from ..framework import flags

        flags.set_flags({"FLAGS_check_nan_inf": False})
