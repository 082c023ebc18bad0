"""Shape / layout / indexing ops (reference: python/paddle/tensor/manipulation.py)."""
from __future__ import annotations

import numpy as np
import torch

from ..framework import dtype as _dt
from ..framework.tensor import Tensor
from ._helpers import axis_arg, shape_arg, u, ut, w

_wrap = Tensor._wrap


def _reshape_shape(t, shape):
    from ..framework import errors as E

    shp = shape_arg(shape)
    # paddle: 0 means "copy this dim from input"
    out = []
    for i, s in enumerate(shp):
        out.append(t.shape[i] if s == 0 and i < t.dim() else s)
    E.enforce(sum(1 for s in out if s == -1) <= 1, E.InvalidArgumentError,
              f"Only one dimension value of 'shape' in ReshapeOp can be -1, but received shape {list(shp)}.")
    known = 1
    for s in out:
        E.enforce(s >= -1, E.InvalidArgumentError, f"Each dimension value of 'shape' must be >= -1, got {s}.")
        known *= s if s > 0 else 1
    n = t.numel()
    if -1 in out:
        E.enforce(known > 0 and n % known == 0, E.InvalidArgumentError,
                  f"The 'shape' attribute in ReshapeOp is invalid: input numel {n} is not divisible by the known "
                  f"dims product {known} (shape {list(shp)}).")
    elif 0 not in out:
        E.enforce(known == n, E.InvalidArgumentError,
                  f"The 'shape' in ReshapeOp is invalid: the input tensor X's size is {n}, but the target shape "
                  f"{list(shp)} has {known} elements.",
                  hint=f"input shape {list(t.shape)}")
    return out


def reshape(x, shape, name=None):
    t = x._t
    return _wrap(t.reshape(_reshape_shape(t, shape)))


def reshape_(x, shape, name=None):
    x._t = x._t.reshape(_reshape_shape(x._t, shape))
    return x


def view(x, shape_or_dtype, name=None):
    if isinstance(shape_or_dtype, (list, tuple, Tensor)):
        return _wrap(x._t.view(_reshape_shape(x._t, shape_or_dtype)))
    return _wrap(x._t.view(_dt.convert_dtype(shape_or_dtype)))


def view_as(x, other, name=None):
    return _wrap(x._t.view_as(other._t))


def flatten(x, start_axis=0, stop_axis=-1, name=None):
    t = x._t
    if t.dim() == 0:
        return _wrap(t.reshape(1))
    return _wrap(torch.flatten(t, start_axis, stop_axis))


def flatten_(x, start_axis=0, stop_axis=-1, name=None):
    x._t = torch.flatten(x._t, start_axis, stop_axis)
    return x


def squeeze(x, axis=None, name=None):
    t = x._t
    ax = axis_arg(axis)
    if ax is None:
        return _wrap(t.squeeze())
    if isinstance(ax, int):
        ax = (ax,)
    ax = tuple(a for a in ax if t.dim() > 0 and t.shape[a] == 1)
    return _wrap(t.squeeze(ax) if ax else t)


def squeeze_(x, axis=None, name=None):
    x._t = squeeze(x, axis)._t
    return x


def unsqueeze(x, axis, name=None):
    t = x._t
    ax = axis_arg(axis)
    if isinstance(ax, int):
        return _wrap(t.unsqueeze(ax))
    for a in ax:
        a = a if a >= 0 else a + t.dim() + 1
        t = t.unsqueeze(a)
    return _wrap(t)


def unsqueeze_(x, axis, name=None):
    x._t = unsqueeze(x, axis)._t
    return x


def transpose(x, perm, name=None):
    return _wrap(x._t.permute(*[int(p) for p in perm]))


def transpose_(x, perm, name=None):
    x._t = x._t.permute(*perm)
    return x


def permute(x, *perm):
    if len(perm) == 1 and isinstance(perm[0], (list, tuple)):
        perm = perm[0]
    return _wrap(x._t.permute(*perm))


def t(input, name=None):
    tt = input._t
    return _wrap(tt if tt.dim() < 2 else tt.t())


def moveaxis(x, source, destination, name=None):
    return _wrap(torch.movedim(x._t, source, destination))


def swapaxes(x, axis0, axis1, name=None):
    return _wrap(torch.swapaxes(x._t, axis0, axis1))


swapdims = swapaxes


def concat(x, axis=0, name=None):
    ax = int(axis.item()) if isinstance(axis, Tensor) else int(axis)
    return _wrap(torch.cat([ut(i) for i in x], dim=ax))


def stack(x, axis=0, name=None):
    return _wrap(torch.stack([ut(i) for i in x], dim=int(axis)))


def hstack(x, name=None):
    return _wrap(torch.hstack([i._t for i in x]))


def vstack(x, name=None):
    return _wrap(torch.vstack([i._t for i in x]))


def dstack(x, name=None):
    return _wrap(torch.dstack([i._t for i in x]))


def column_stack(x, name=None):
    return _wrap(torch.column_stack([i._t for i in x]))


row_stack = vstack


def split(x, num_or_sections, axis=0, name=None):
    t = x._t
    ax = int(axis.item()) if isinstance(axis, Tensor) else int(axis)
    if ax < 0:
        ax += t.dim()
    if isinstance(num_or_sections, int):
        n = num_or_sections
        if t.shape[ax] % n != 0:
            raise ValueError(f"dim {t.shape[ax]} not divisible by {n}")
        return [_wrap(s) for s in torch.split(t, t.shape[ax] // n, dim=ax)]
    secs = [int(s.item()) if isinstance(s, Tensor) else int(s) for s in num_or_sections]
    if -1 in secs:
        known = sum(s for s in secs if s != -1)
        secs = [t.shape[ax] - known if s == -1 else s for s in secs]
    return [_wrap(s) for s in torch.split(t, secs, dim=ax)]


def tensor_split(x, num_or_indices, axis=0, name=None):
    return [_wrap(s) for s in torch.tensor_split(x._t, num_or_indices, dim=axis)]


def hsplit(x, num_or_indices, name=None):
    return [_wrap(s) for s in torch.hsplit(x._t, num_or_indices)]


def vsplit(x, num_or_indices, name=None):
    return [_wrap(s) for s in torch.vsplit(x._t, num_or_indices)]


def chunk(x, chunks, axis=0, name=None):
    return split(x, chunks, axis)


def unbind(input, axis=0):
    return [_wrap(s) for s in torch.unbind(input._t, dim=axis)]


def unstack(x, axis=0, num=None):
    return unbind(x, axis)


def gather(x, index, axis=None, name=None):
    t = x._t
    idx = index._t.long()
    ax = 0 if axis is None else int(axis.item() if isinstance(axis, Tensor) else axis)
    if idx.dim() == 0:
        return _wrap(torch.index_select(t, ax, idx.reshape(1)).squeeze(ax))
    return _wrap(torch.index_select(t, ax, idx.flatten()))


def gather_nd(x, index, name=None):
    t = x._t
    idx = index._t.long()
    k = idx.shape[-1]
    flat_idx = idx.reshape(-1, k)
    out = t[tuple(flat_idx[:, i] for i in range(k))]
    return _wrap(out.reshape(list(idx.shape[:-1]) + list(t.shape[k:])))


def scatter(x, index, updates, overwrite=True, name=None):
    t = x._t.clone()
    idx = index._t.long().flatten()
    upd = updates._t
    if overwrite:
        t[idx] = upd.to(t.dtype)
    else:
        t.index_fill_(0, idx, 0)
        t.index_add_(0, idx, upd.to(t.dtype))
    return _wrap(t)


def scatter_(x, index, updates, overwrite=True, name=None):
    r = scatter(x, index, updates, overwrite)
    with torch.no_grad():
        x._t.copy_(r._t)
    return x


def scatter_nd_add(x, index, updates, name=None):
    t = x._t.clone()
    idx = index._t.long()
    k = idx.shape[-1]
    flat = idx.reshape(-1, k)
    upd = updates._t.reshape([flat.shape[0]] + list(t.shape[k:]))
    t.index_put_(tuple(flat[:, i] for i in range(k)), upd.to(t.dtype), accumulate=True)
    return _wrap(t)


def scatter_nd(index, updates, shape, name=None):
    z = torch.zeros(shape_arg(shape), dtype=updates._t.dtype, device=updates._t.device)
    return scatter_nd_add(_wrap(z), index, updates)


def index_select(x, index, axis=0, name=None):
    return _wrap(torch.index_select(x._t, int(axis), index._t.long()))


def index_add(x, index, axis, value, name=None):
    return _wrap(torch.index_add(x._t, axis, index._t.long(), value._t))


def index_add_(x, index, axis, value, name=None):
    x._t.index_add_(axis, index._t.long(), value._t)
    return x


def index_put(x, indices, value, accumulate=False, name=None):
    return _wrap(torch.index_put(x._t, tuple(i._t for i in indices), ut(value, x._t), accumulate))


def index_put_(x, indices, value, accumulate=False, name=None):
    x._t.index_put_(tuple(i._t for i in indices), ut(value, x._t), accumulate)
    return x


def index_fill(x, index, axis, value, name=None):
    return _wrap(torch.index_fill(x._t, axis, index._t.long(), value))


def take_along_axis(arr, indices, axis, broadcast=True):
    t = arr._t
    idx = indices._t.long()
    if broadcast:
        shp = list(t.shape)
        shp[axis] = idx.shape[axis]
        idx = idx.expand(shp) if list(idx.shape) != shp else idx
    return _wrap(torch.gather(t, axis, idx))


def put_along_axis(arr, indices, values, axis, reduce="assign", include_self=True, broadcast=True):
    t = arr._t
    idx = indices._t.long()
    v = ut(values, t)
    if v.dim() == 0:
        v = v.expand(idx.shape)
    v = v.to(t.dtype)
    if reduce == "assign":
        return _wrap(torch.scatter(t, axis, idx, v))
    red = {"add": "sum", "mul": "prod", "multiply": "prod", "mean": "mean", "amax": "amax", "amin": "amin"}[reduce]
    return _wrap(torch.scatter_reduce(t, axis, idx, v, red, include_self=include_self))


def put_along_axis_(arr, indices, values, axis, reduce="assign"):
    r = put_along_axis(arr, indices, values, axis, reduce)
    with torch.no_grad():
        arr._t.copy_(r._t)
    return arr


def tile(x, repeat_times, name=None):
    return _wrap(x._t.repeat(*shape_arg(repeat_times)) if len(shape_arg(repeat_times)) >= x._t.dim()
                 else torch.tile(x._t, tuple(shape_arg(repeat_times))))


def expand(x, shape, name=None):
    shp = shape_arg(shape)
    return _wrap(x._t.expand(*shp))


def expand_as(x, y, name=None):
    return _wrap(x._t.expand_as(y._t))


def broadcast_to(x, shape, name=None):
    return _wrap(torch.broadcast_to(x._t, shape_arg(shape)))


def broadcast_tensors(input, name=None):
    return [_wrap(t) for t in torch.broadcast_tensors(*[i._t for i in input])]


def broadcast_shape(x_shape, y_shape):
    return list(torch.broadcast_shapes(tuple(x_shape), tuple(y_shape)))


def flip(x, axis, name=None):
    ax = axis_arg(axis)
    if isinstance(ax, int):
        ax = (ax,)
    return _wrap(torch.flip(x._t, ax))


def rot90(x, k=1, axes=[0, 1], name=None):
    return _wrap(torch.rot90(x._t, k, axes))


def roll(x, shifts, axis=None, name=None):
    return _wrap(torch.roll(x._t, shifts, axis))


def slice(input, axes, starts, ends):
    t = input._t
    idx = [builtins_slice(None)] * t.dim()
    for a, s, e in zip(axes, starts, ends):
        s = int(s.item()) if isinstance(s, Tensor) else int(s)
        e = int(e.item()) if isinstance(e, Tensor) else int(e)
        idx[a] = builtins_slice(s, e)
    return _wrap(t[tuple(idx)])


def strided_slice(x, axes, starts, ends, strides, name=None):
    t = x._t
    idx = [builtins_slice(None)] * t.dim()
    for a, s, e, st in zip(axes, starts, ends, strides):
        if st < 0:
            # negative strides: flip then slice
            n = t.shape[a]
            s = n + s if s < 0 else s
            e = n + e if e < 0 else e
            sel = torch.arange(min(s, n - 1), e, st, device=t.device)
            t = t.index_select(a, sel)
            continue
        idx[a] = builtins_slice(s, e, st)
    return _wrap(t[tuple(idx)])


import builtins  # noqa: E402

builtins_slice = builtins.slice


def crop(x, shape=None, offsets=None, name=None):
    t = x._t
    shp = shape_arg(shape) if shape is not None else list(t.shape)
    offs = shape_arg(offsets) if offsets is not None else [0] * t.dim()
    idx = tuple(builtins_slice(o, o + (s if s != -1 else t.shape[i] - o)) for i, (o, s) in enumerate(zip(offs, shp)))
    return _wrap(t[idx])


def unique(x, return_index=False, return_inverse=False, return_counts=False, axis=None, dtype="int64", name=None):
    t = x._t
    res = torch.unique(t, sorted=True, return_inverse=True, return_counts=True, dim=axis)
    out, inv, cnt = res
    outs = [_wrap(out)]
    idt = _dt.convert_dtype(dtype)
    if return_index:
        flat = t.flatten() if axis is None else t
        n = inv.numel()
        perm = torch.arange(n, device=t.device)
        first = torch.full((out.shape[0] if axis is not None else out.numel(),), n, dtype=torch.long, device=t.device)
        first = first.scatter_reduce(0, inv.flatten(), perm, "amin")
        outs.append(_wrap(first.to(idt)))
        del flat
    if return_inverse:
        outs.append(_wrap(inv.to(idt)))
    if return_counts:
        outs.append(_wrap(cnt.to(idt)))
    return outs[0] if len(outs) == 1 else tuple(outs)


def unique_consecutive(x, return_inverse=False, return_counts=False, axis=None, dtype="int64", name=None):
    out, inv, cnt = torch.unique_consecutive(x._t, return_inverse=True, return_counts=True, dim=axis)
    outs = [_wrap(out)]
    if return_inverse:
        outs.append(_wrap(inv.to(_dt.convert_dtype(dtype))))
    if return_counts:
        outs.append(_wrap(cnt.to(_dt.convert_dtype(dtype))))
    return outs[0] if len(outs) == 1 else tuple(outs)


def repeat_interleave(x, repeats, axis=None, name=None):
    r = repeats._t if isinstance(repeats, Tensor) else repeats
    return _wrap(torch.repeat_interleave(x._t, r, dim=axis))


def masked_fill(x, mask, value, name=None):
    v = value._t if isinstance(value, Tensor) else value
    return _wrap(x._t.masked_fill(mask._t, v))


def masked_fill_(x, mask, value, name=None):
    x._t.masked_fill_(mask._t, value._t if isinstance(value, Tensor) else value)
    return x


def masked_scatter(x, mask, value, name=None):
    return _wrap(x._t.masked_scatter(mask._t, value._t))


def as_complex(x, name=None):
    return _wrap(torch.view_as_complex(x._t.contiguous()))


def as_real(x, name=None):
    return _wrap(torch.view_as_real(x._t))


def as_strided(x, shape, stride, offset=0, name=None):
    return _wrap(torch.as_strided(x._t, shape, stride, offset))


def atleast_1d(*inputs, name=None):
    r = [_wrap(torch.atleast_1d(i._t)) for i in inputs]
    return r[0] if len(r) == 1 else r


def atleast_2d(*inputs, name=None):
    r = [_wrap(torch.atleast_2d(i._t)) for i in inputs]
    return r[0] if len(r) == 1 else r


def atleast_3d(*inputs, name=None):
    r = [_wrap(torch.atleast_3d(i._t)) for i in inputs]
    return r[0] if len(r) == 1 else r


def shard_index(input, index_num, nshards, shard_id, ignore_value=-1):
    t = input._t
    size = (index_num + nshards - 1) // nshards
    lo = shard_id * size
    in_shard = (t >= lo) & (t < lo + size)
    return _wrap(torch.where(in_shard, t - lo, torch.full_like(t, ignore_value)))


def tolist(x):
    return x._t.tolist()


def fill_diagonal_(x, value, offset=0, wrap=False, name=None):
    with torch.no_grad():
        x._t.fill_diagonal_(value, wrap=wrap)
    return x


def diagonal_scatter(x, y, offset=0, axis1=0, axis2=1, name=None):
    return _wrap(torch.diagonal_scatter(x._t, y._t, offset, axis1, axis2))


def select_scatter(x, values, axis, index, name=None):
    return _wrap(torch.select_scatter(x._t, values._t, axis, index))


def slice_scatter(x, value, axes, starts, ends, strides, name=None):
    t = x._t.clone()
    idx = [builtins_slice(None)] * t.dim()
    for a, s, e, st in zip(axes, starts, ends, strides):
        idx[a] = builtins_slice(s, e, st)
    t[tuple(idx)] = value._t
    return _wrap(t)


def unflatten(x, axis, shape, name=None):
    return _wrap(torch.unflatten(x._t, axis, shape_arg(shape)))


def unfold(x, axis, size, step, name=None):
    return _wrap(x._t.unfold(axis, size, step))


def _np(x):
    return np.asarray(x)


def cast(x, dtype):
    return _wrap(x._t.to(_dt.convert_dtype(dtype)))


def cast_(x, dtype):
    x._t = x._t.to(_dt.convert_dtype(dtype))
    return x


def numel(x, name=None):
    return _wrap(torch.tensor(x._t.numel(), dtype=torch.int64, device=x._t.device))


def shape(input):
    return _wrap(torch.tensor(list(input._t.shape), dtype=torch.int32))


def rank(input):
    return _wrap(torch.tensor(input._t.dim(), dtype=torch.int32))


def is_empty(x, name=None):
    return _wrap(torch.tensor(x._t.numel() == 0))


def u_(x):
    return u(x)


def _wrap_list(ts):
    return w(ts)


__all__ = [_n for _n, _v in list(globals().items())
           if not _n.startswith("_") and callable(_v) and getattr(_v, "__module__", None) == __name__]
