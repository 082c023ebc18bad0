"""The eager ``paddle.Tensor``.

Design: a thin Python object that owns a ``torch.Tensor`` living on the MI355X
(torch device ``cuda`` under ROCm) or on the CPU.  Paddle semantics sit on top:

* ``stop_gradient`` (default ``True`` for plain tensors, ``False`` for parameters) maps onto
  torch's ``requires_grad``; autograd itself is torch's native multithreaded engine
  (reference: paddle/fluid/eager/backward.cc:105 ``RunBackward``).
* ``shape`` is a Python list, ``place`` is a :class:`Place`, ``size`` is the element count.
* Methods from ``paddle2_amd.tensor`` are patched on (like python/paddle/tensor/__init__.py:459
  ``tensor_method_func``).
"""
from __future__ import annotations

import numbers

import numpy as np
import torch

from . import dtype as _dt
from .place import CPUPlace, CUDAPlace, Place, current_torch_device, place_of_device


class Tensor:
    """Eager tensor (reference: paddle/fluid/pybind/eager.cc, eager_method.cc, eager_properties.cc)."""

    # class-level defaults keep instance creation cheap (only ``_t`` is set per instance)
    name = None
    persistable = False
    _is_param = False
    _dist_attr = None
    _process_mesh = None
    _placements = None

    __array_priority__ = 100

    def __init__(self, value=None, dtype=None, place=None, stop_gradient=True, name=None):
        if value is None:
            t = torch.empty(0)
        else:
            t = _to_torch(value, dtype=dtype, place=place)
        self._t = t
        if name is not None:
            self.name = name
        if not stop_gradient:
            self.stop_gradient = False

    # ------------------------------------------------------------------ basics
    @property
    def shape(self):
        return list(self._t.shape)

    @property
    def dtype(self):
        return self._t.dtype

    @property
    def place(self) -> Place:
        return place_of_device(self._t.device)

    @property
    def ndim(self):
        return self._t.dim()

    def dim(self):
        return self._t.dim()

    def ndimension(self):
        return self._t.dim()

    @property
    def size(self):
        return self._t.numel()

    def numel(self):
        return Tensor._wrap(torch.tensor(self._t.numel(), dtype=torch.int64))

    @property
    def T(self):
        return Tensor._wrap(self._t.permute(*reversed(range(self._t.dim()))))

    @property
    def mT(self):
        return Tensor._wrap(self._t.transpose(-1, -2))

    @property
    def is_leaf(self):
        return self._t.is_leaf

    @property
    def stop_gradient(self):
        return not self._t.requires_grad

    @stop_gradient.setter
    def stop_gradient(self, v: bool):
        v = bool(v)
        t = self._t
        if v:
            if t.requires_grad:
                if t.is_leaf:
                    t.requires_grad_(False)
                else:
                    self._t = t.detach()
        else:
            if not t.requires_grad:
                if t.is_floating_point() or t.is_complex():
                    if t.is_leaf:
                        t.requires_grad_(True)
                    else:  # produced under no_grad: re-root as a leaf
                        self._t = t.detach().requires_grad_(True)

    @property
    def grad(self):
        g = self._t.grad
        if g is None and getattr(self, "_lazy_zero_grad", False):
            # cleared with set_to_zero=True (optimizer.clear_grad): materialise the zeros on demand
            g = torch.zeros_like(self._t)
            self._t.grad = g
        return None if g is None else Tensor._wrap(g)

    @grad.setter
    def grad(self, value):
        self._t.grad = None if value is None else _unwrap(value)

    @property
    def data(self):
        return Tensor._wrap(self._t.detach())

    @data.setter
    def data(self, value):
        with torch.no_grad():
            self._t.data = _unwrap(value)

    def _is_initialized(self):
        return True

    def is_dense(self):
        return not self._t.is_sparse

    def is_dist(self):
        return self._dist_attr is not None

    def is_contiguous(self):
        return self._t.is_contiguous()

    def contiguous(self):
        return Tensor._wrap(self._t.contiguous())

    def element_size(self):
        return self._t.element_size()

    def value(self):
        return self

    def get_tensor(self):
        return self

    def _numel(self):
        return self._t.numel()

    def _md5sum(self):
        import hashlib

        return hashlib.md5(self.numpy().tobytes()).hexdigest()

    # ---------------------------------------------------------------- creation
    @staticmethod
    def _wrap(t: torch.Tensor) -> "Tensor":
        o = object.__new__(Tensor)
        o._t = t
        return o

    # --------------------------------------------------------------- transfers
    def numpy(self):
        t = self._t.detach()
        if t.device.type != "cpu":
            t = t.cpu()
        if t.dtype == torch.bfloat16:
            return t.view(torch.int16).numpy().view(np.uint16)
        if t.dtype in (torch.float8_e4m3fn, torch.float8_e5m2):
            return t.view(torch.uint8).numpy()
        return t.numpy()

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a.astype(dtype) if dtype is not None else a

    def item(self, *args):
        if args:
            return self._t[args].item() if len(args) > 1 else self._t.flatten()[args[0]].item()
        return self._t.item()

    def tolist(self):
        return self._t.tolist()

    def cpu(self):
        return Tensor._wrap(self._t.cpu())

    def cuda(self, device_id=None, blocking=True):
        dev = torch.device("cuda", device_id) if device_id is not None else torch.device("cuda", torch.cuda.current_device())
        return Tensor._wrap(self._t.to(dev, non_blocking=not blocking))

    def pin_memory(self):
        return Tensor._wrap(self._t.pin_memory())

    def to(self, *args, **kwargs):
        device = kwargs.pop("device", None)
        dtype = kwargs.pop("dtype", None)
        blocking = kwargs.pop("blocking", None)
        for a in args:
            if isinstance(a, (str, Place, torch.device)):
                s = str(a)
                try:
                    dtype = _dt.convert_dtype(a) if isinstance(a, str) and not _looks_like_device(s) else dtype
                    if dtype is not None and isinstance(a, str) and not _looks_like_device(s):
                        continue
                except TypeError:
                    pass
                device = a
            elif isinstance(a, torch.dtype):
                dtype = a
            elif isinstance(a, bool):
                blocking = a
        t = self._t
        if device is not None:
            from .place import _parse_device

            t = t.to(_parse_device(device), non_blocking=blocking is False)
        if dtype is not None:
            t = t.to(_dt.convert_dtype(dtype))
        return Tensor._wrap(t)

    # ------------------------------------------------------------------ dtype
    def astype(self, dtype):
        return Tensor._wrap(self._t.to(_dt.convert_dtype(dtype)))

    cast = astype

    def is_floating_point(self):
        return self._t.is_floating_point()

    def is_complex(self):
        return self._t.is_complex()

    def is_integer(self):
        return not (self._t.is_floating_point() or self._t.is_complex() or self._t.dtype == torch.bool)

    # --------------------------------------------------------------- autograd
    def backward(self, grad_tensor=None, retain_graph=False):
        g = None if grad_tensor is None else _unwrap(grad_tensor)
        if g is None and self._t.numel() != 1:
            g = torch.ones_like(self._t)
        self._t.backward(g, retain_graph=retain_graph)

    def clear_gradient(self, set_to_zero=True):
        g = self._t.grad
        if g is None:
            return
        if set_to_zero:
            g.zero_()
        else:
            self._t.grad = None

    def clear_grad(self, set_to_zero=True):
        self.clear_gradient(set_to_zero)

    def _clear_gradient(self):
        self._t.grad = None

    def detach(self):
        return Tensor._wrap(self._t.detach())

    def detach_(self):
        self._t = self._t.detach()
        return self

    def clone(self):
        return Tensor._wrap(self._t.clone())

    def register_hook(self, hook):
        def _h(g):
            r = hook(Tensor._wrap(g))
            return None if r is None else _unwrap(r)

        return self._t.register_hook(_h)

    def _register_backward_hook(self, hook):
        return self.register_hook(hook)

    # ------------------------------------------------------------- mutation
    def set_value(self, value):
        v = value._t if isinstance(value, Tensor) else torch.as_tensor(np.asarray(value))
        with torch.no_grad():
            if list(v.shape) != list(self._t.shape):
                raise ValueError(f"set_value shape mismatch {list(v.shape)} vs {self.shape}")
            self._t.copy_(v.to(self._t.dtype))
        return self

    def copy_(self, other, blocking=True):
        with torch.no_grad():
            self._t.copy_(_unwrap(other))
        return self

    def zero_(self):
        with torch.no_grad():
            self._t.zero_()
        return self

    def fill_(self, value):
        with torch.no_grad():
            self._t.fill_(value)
        return self

    def _share_buffer_to(self, other):
        other._t = self._t
        return other

    def _copy_to(self, place, blocking=True):
        return self.to(place)

    def share_memory_(self):
        self._t.share_memory_()
        return self

    # ------------------------------------------------------------- indexing
    def __getitem__(self, idx):
        return Tensor._wrap(self._t[_unwrap_index(idx)])

    def __setitem__(self, idx, value):
        v = _unwrap(value)
        if isinstance(v, torch.Tensor) and v.dtype != self._t.dtype:
            v = v.to(self._t.dtype)
        if self._t.requires_grad and self._t.is_leaf:
            with torch.no_grad():
                self._t[_unwrap_index(idx)] = v
        else:
            self._t[_unwrap_index(idx)] = v

    def __len__(self):
        return len(self._t)

    def __iter__(self):
        for i in range(len(self._t)):
            yield Tensor._wrap(self._t[i])

    def __contains__(self, item):
        return bool((self._t == _unwrap(item)).any())

    # --------------------------------------------------------------- python
    def __repr__(self):
        sg = self.stop_gradient
        return (f"Tensor(shape={self.shape}, dtype={_dt._DT2STR.get(self.dtype, self.dtype)}, "
                f"place={self.place}, stop_gradient={sg},\n       {self._t.detach().cpu().__repr__()[7:-1]})")

    __str__ = __repr__

    def __bool__(self):
        return bool(self._t)

    def __int__(self):
        return int(self._t)

    def __float__(self):
        return float(self._t.detach())

    def __index__(self):
        return int(self._t)

    def __complex__(self):
        return complex(self._t)

    def __hash__(self):
        return id(self)

    def __format__(self, spec):
        if self._t.dim() == 0:
            return format(self._t.item(), spec)
        return object.__format__(self, spec)

    def __deepcopy__(self, memo):
        o = Tensor._wrap(self._t.detach().clone().requires_grad_(self._t.requires_grad))
        o.__dict__.update({k: v for k, v in self.__dict__.items() if k != "_t"})
        memo[id(self)] = o
        return o

    def __reduce_ex__(self, proto):
        # plain pickling (paddle.save handles state dicts separately)
        return (_rebuild_tensor, (self.numpy(), _dt.dtype_name(self.dtype), self.stop_gradient, self.name))

    # dunder arithmetic is installed by paddle2_amd.tensor (see _patch_tensor_methods)


def _rebuild_tensor(arr, dtype, stop_gradient, name):
    t = Tensor(arr, dtype=dtype, place=CPUPlace())
    t.stop_gradient = stop_gradient
    t.name = name
    return t


def _looks_like_device(s: str) -> bool:
    s = s.lower()
    return s.startswith(("cpu", "gpu", "cuda", "hip", "place"))


def _unwrap(x):
    """Tensor -> torch.Tensor; leave python scalars alone; convert numpy/lists to torch."""
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x))
    return x


def _unwrap_index(idx):
    if isinstance(idx, Tensor):
        return idx._t
    if isinstance(idx, tuple):
        return tuple(_unwrap_index(i) for i in idx)
    if isinstance(idx, list):
        if any(isinstance(i, Tensor) for i in idx):
            return [_unwrap_index(i) for i in idx]
        return idx
    return idx


def _to_torch(value, dtype=None, place=None) -> torch.Tensor:
    """Build a torch tensor from Paddle-style input (to_tensor semantics)."""
    from .place import _parse_device

    dev = _parse_device(place) if place is not None else current_torch_device()
    tdt = _dt.convert_dtype(dtype) if dtype is not None else None
    if isinstance(value, Tensor):
        t = value._t.detach()
        if tdt is not None:
            t = t.to(tdt)
        return t.to(dev).clone()
    if isinstance(value, torch.Tensor):
        t = value.detach()
        if tdt is not None:
            t = t.to(tdt)
        return t.to(dev).clone()
    if isinstance(value, np.ndarray):
        arr = value
        if arr.dtype == np.float64 and tdt is None:
            tdt = torch.float64
        if arr.dtype == np.uint16 and tdt is None:  # paddle's numpy spelling of bfloat16
            tdt = torch.bfloat16
        t = torch.from_numpy(np.ascontiguousarray(arr))
        if arr.dtype == np.uint16 and tdt == torch.bfloat16:
            t = t.view(torch.bfloat16)
        elif tdt is not None:
            t = t.to(tdt)
        return t.to(dev)
    if isinstance(value, (bool, np.bool_)):
        t = torch.tensor(bool(value), dtype=tdt or torch.bool)
        return t.to(dev)
    if isinstance(value, numbers.Integral):
        return torch.tensor(int(value), dtype=tdt or torch.int64, device=dev)
    if isinstance(value, numbers.Real):
        return torch.tensor(float(value), dtype=tdt or _dt.default_float_dtype(), device=dev)
    if isinstance(value, numbers.Complex):
        return torch.tensor(complex(value), dtype=tdt or torch.complex64, device=dev)
    if isinstance(value, (list, tuple)):
        if len(value) > 0 and any(isinstance(v, Tensor) for v in value):
            ts = [(_to_torch(v, place=dev) if not isinstance(v, Tensor) else v._t.detach().to(dev)) for v in value]
            t = torch.stack(ts)
            return t.to(tdt) if tdt is not None else t
        arr = np.array(value)
        if arr.dtype == np.float64:
            arr = arr.astype(_dt.to_numpy_dtype(tdt) if tdt is not None and tdt != torch.bfloat16 else np.float32)
            if tdt is None:
                tdt = _dt.default_float_dtype()
        elif arr.dtype.kind in "iu" and tdt is None:
            arr = arr.astype(np.int64)
        t = torch.from_numpy(np.ascontiguousarray(arr))
        if tdt is not None:
            t = t.to(tdt)
        return t.to(dev)
    raise TypeError(f"cannot convert {type(value)} to Tensor")


def to_tensor(data, dtype=None, place=None, stop_gradient=True):
    """paddle.to_tensor (python/paddle/tensor/creation.py)."""
    t = Tensor.__new__(Tensor)
    t._t = _to_torch(data, dtype=dtype, place=place)
    if not stop_gradient:
        t.stop_gradient = False
    return t


def wrap(t):
    """Wrap torch output(s) into Tensor(s)."""
    if isinstance(t, torch.Tensor):
        return Tensor._wrap(t)
    if isinstance(t, list):
        return [wrap(x) for x in t]
    if isinstance(t, tuple):
        return tuple(wrap(x) for x in t)
    return t


unwrap = _unwrap


def is_tensor(x) -> bool:
    return isinstance(x, Tensor)
