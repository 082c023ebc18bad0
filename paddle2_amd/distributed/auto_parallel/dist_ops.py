"""SPMD dispatch at op entry for DistTensors (reference: the generated dist branch of every phi API —
paddle/phi/api/lib/api_gen (dist_api_gen.py): InferSpmd -> reshard inputs -> local kernel -> set output dist
attrs; rules in paddle/phi/infermeta/spmd_rules/).

The framework's hot ops (rms_norm / layer_norm, linear, rope, flash attention, swiglu, embedding) check for
DistTensor arguments at entry (``ops/torch_ops.py``, ``nn/functional``) and come here:

  1. build a ``DistTensorSpec`` (global shape, dims_mapping, partial dims) per input;
  2. ask the op's rule (``spmd_rules.get_spmd_rule``) for the input and output distributions;
  3. reshard every input to its required placements with the framework's own engine (``reshard.py``:
     all-gather / all-reduce / reduce-scatter / all-to-all over the mesh dim's group);
  4. run the op's LOCAL implementation — the same native HIP kernels as the single-device path — on the local
     shards (``to_local`` with the gradient placements the op's backward produces: a contraction over a mesh-
     sharded letter makes that input's gradient PARTIAL);
  5. wrap the local outputs as DistTensors with the rule's output placements.

Ops without a hook go through DistTensor's aten-level SPMD dispatch (dist_tensor.py).
"""
from __future__ import annotations

import torch

from . import spmd_rules as R
from .dist_tensor import DistTensor
from .placement import Partial as _TPartial
from .placement import Replicate as _TReplicate
from .placement import Shard as _TShard
from .reshard import reshard

DTensor = DistTensor
TRACE = []   # (op, [input dims_mapping], [output dims_mapping]) of every dispatched op (tests inspect it)


class _MeshInfo:
    def __init__(self, dm):
        self.shape = list(dm.shape)
        self.device_mesh = dm


def is_dist(*ts):
    return any(isinstance(t, DTensor) for t in ts)


def _mesh_of(*ts):
    for t in ts:
        if isinstance(t, DTensor):
            return t.device_mesh
    return None


def _spec(t, dm):
    if t is None:
        return None
    nd = t.dim()
    mapping = [-1] * nd
    partial = set()
    if isinstance(t, DTensor):
        for m, p in enumerate(t.placements):
            if isinstance(p, _TShard):
                a = p.dim % nd
                if mapping[a] != -1:
                    raise NotImplementedError("one tensor axis sharded over two mesh dims")
                mapping[a] = m
            elif isinstance(p, _TPartial):
                partial.add(m)
    return R.DistTensorSpec(list(t.shape), R.TensorDistAttr(mapping, _MeshInfo(dm), partial))


def _placements(attr, ndim_mesh, partial_extra=()):
    out = [_TReplicate() for _ in range(ndim_mesh)]
    for axis, m in enumerate(attr.dims_mapping):
        if m != -1:
            out[m] = _TShard(axis)
    for m in set(attr._partial_dims()) | set(partial_extra):
        if isinstance(out[m], _TReplicate):
            out[m] = _TPartial()
    return tuple(out)


def _as_dist(t, dm):
    """plain tensors join the computation replicated over the mesh"""
    if t is None or isinstance(t, DTensor):
        return t
    return DistTensor.from_local(t, dm, [_TReplicate()] * dm.ndim)


def _local(t, dm, attr, grad_partial=()):
    """reshard ``t`` to ``attr`` and return the local shard; its gradient is declared PARTIAL on
    ``grad_partial`` mesh dims (the op's backward sums over letters sharded there)."""
    if t is None:
        return None
    t = _as_dist(t, dm)
    pl = _placements(attr, dm.ndim)
    t = reshard(t, pl)
    gpl = _placements(attr, dm.ndim, grad_partial)
    return t.to_local(grad_placements=gpl)


def _wrap(local, dm, attr, shape=None):
    return DistTensor.from_local(local, dm, _placements(attr, dm.ndim), shape=None if shape is None else tuple(shape))


def _sharded_dims(dms):
    return {m for dm in dms for m in dm if m != -1}


# ------------------------------------------------------------------------------------------------ ops
def rms_norm(x, w, eps, residual=None, layer=False, b=None):
    from ...ops import torch_ops as T

    dm = _mesh_of(x, w, residual)
    xs, ws = _spec(x, dm), _spec(_as_dist(w, dm), dm)
    if layer:
        ins, outs = R.layer_norm_forward(xs, ws, _spec(_as_dist(b, dm), dm) if b is not None else None,
                                         eps, x.dim() - 1)
    else:
        ins, outs = R.rms_norm_forward(xs, ws, eps)
    xa = ins[0]
    lead = _sharded_dims([xa.dims_mapping[:-1]])
    xl = _local(x, dm, xa)
    wl = _local(w, dm, R.TensorDistAttr([-1], None), lead)   # d_scale sums over the sharded rows
    bl = _local(b, dm, R.TensorDistAttr([-1], None), lead) if b is not None else None
    rl = _local(residual, dm, xa) if residual is not None else None
    TRACE.append(("layer_norm" if layer else "rms_norm", [xa.dims_mapping], [outs[0].dims_mapping]))
    if layer:
        r = T.layer_norm(xl, wl, bl, eps, rl)
    else:
        r = T.rms_norm(xl, wl, eps, rl)
    if residual is None:
        return _wrap(r, dm, outs[0], x.shape)
    y, h = r
    return _wrap(y, dm, outs[0], x.shape), _wrap(h, dm, outs[0], x.shape)


def linear(x, w, b=None):
    """y = x @ w (+ b), w [K, N]: matmul rule; a sharded K makes y PARTIAL (row-parallel), a sharded N makes
    d_x PARTIAL (column-parallel), sharded rows of x make d_w PARTIAL (data-parallel)."""
    from ...ops import torch_ops as T

    dm = _mesh_of(x, w, b)
    xs, ws = _spec(_as_dist(x, dm), dm), _spec(_as_dist(w, dm), dm)
    ins, outs = R.matmul_forward(xs, ws)
    xa, wa, oa = ins[0], ins[1], outs[0]
    n_dim = wa.dims_mapping[-1]
    x_lead = _sharded_dims([xa.dims_mapping[:-1]])
    xl = _local(x, dm, xa, {n_dim} - {-1} - set(xa.dims_mapping))
    wl = _local(w, dm, wa, x_lead - set(wa.dims_mapping))
    TRACE.append(("matmul", [xa.dims_mapping, wa.dims_mapping], [oa.dims_mapping, sorted(oa._partial_dims())]))
    y = T.linear(xl, wl) if (xl.is_cuda and xl.dtype in (torch.bfloat16, torch.float16)) else torch.matmul(xl, wl)
    shape = list(x.shape[:-1]) + [w.shape[-1]]
    out = _wrap(y, dm, oa, shape)
    if b is not None:
        out = add(out, b)
    return out


def add(x, y):
    """elementwise add through the elementwise rule (a PARTIAL operand is reduced first: adding a replicated
    value to a partial sum would count it once per rank)."""
    dm = _mesh_of(x, y)
    xs, ys = _spec(_as_dist(x, dm), dm), _spec(_as_dist(y, dm), dm)
    clean = [R.DistTensorSpec(s.shape, R.TensorDistAttr(s.dims_mapping, s.dist_attr.process_mesh)) for s in (xs, ys)]
    ins, outs = R.elementwise_forward(*clean)
    notas, on = R._bcast_notations([xs.shape, ys.shape])
    amap = dict(zip(on, outs[0].dims_mapping))
    gp = [{amap[a] for a in on if a not in n and amap.get(a, -1) != -1} for n in notas]
    xl = _local(x, dm, ins[0], gp[0])
    yl = _local(y, dm, ins[1], gp[1])
    TRACE.append(("add", [ins[0].dims_mapping, ins[1].dims_mapping], [outs[0].dims_mapping]))
    shape = list(torch.broadcast_shapes(tuple(x.shape), tuple(y.shape)))
    return _wrap(xl + yl, dm, outs[0], shape)


def swiglu(x, y=None):
    from ...ops import torch_ops as T

    dm = _mesh_of(x, y)
    xs = _spec(x, dm)
    ys = _spec(_as_dist(y, dm), dm) if y is not None else None
    ins, outs = R.swiglu_forward(xs, ys)
    xl = _local(x, dm, ins[0])
    yl = _local(y, dm, ins[1]) if y is not None else None
    TRACE.append(("swiglu", [ins[0].dims_mapping], [outs[0].dims_mapping]))
    r = T.swiglu(xl, yl)
    shape = list(x.shape) if y is not None else list(x.shape[:-1]) + [x.shape[-1] // 2]
    return _wrap(r, dm, outs[0], shape)


def rope(x, cos, sin, pos=None, style=0, time_major=False):
    """x [b, s, h, d]: rotary tables are indexed by absolute position, so the sequence axis is replicated
    (fused_rope rule without sin/cos specs); batch and heads keep their sharding."""
    from ...ops import torch_ops as T

    dm = _mesh_of(x)
    ins, outs = R.fused_rope_forward(_spec(x, dm), time_major=time_major)
    xl = _local(x, dm, ins[0])
    TRACE.append(("rope", [ins[0].dims_mapping], [outs[0].dims_mapping]))
    pl = pos.to_local() if isinstance(pos, DTensor) else pos
    return _wrap(T.rope(xl, cos, sin, pl, style=style, time_major=time_major), dm, outs[0], x.shape)


def flash_attention(q, k, v, causal=False, scale=None):
    from ...ops import torch_ops as T

    dm = _mesh_of(q, k, v)
    qs, ks, vs = (_spec(_as_dist(t, dm), dm) for t in (q, k, v))
    ins, outs = R.flash_attention_forward(qs, ks, vs, causal)
    ql, kl, vl = (_local(t, dm, a) for t, a in zip((q, k, v), ins))
    TRACE.append(("flash_attention", [a.dims_mapping for a in ins], [outs[0].dims_mapping]))
    o, lse = T.flash_attention(ql, kl, vl, causal, scale)
    return _wrap(o, dm, outs[0], q.shape), _wrap(lse, dm, outs[1], [q.shape[0], q.shape[2], q.shape[1]])


def embedding(ids, w, padding_idx=None, start=0):
    """Vocab-sharded weight -> c_embedding (this shard's vocab range, output PARTIAL); otherwise the embedding
    rule.  d_weight is PARTIAL on the mesh dims that shard the ids."""
    from ...ops import torch_ops as T

    dm = _mesh_of(ids, w)
    ws, xs = _spec(_as_dist(w, dm), dm), _spec(_as_dist(ids, dm), dm)
    ins, outs = R.c_embedding_forward(ws, xs, start)
    wa, xa, oa = ins[0], ins[1], outs[0]
    lead = _sharded_dims([xa.dims_mapping])
    wl = _local(w, dm, wa, lead - set(wa.dims_mapping))
    il = _local(ids, dm, xa)
    vd = wa.dims_mapping[0]
    st = start
    if vd != -1:
        st = start + dm.get_local_rank(vd) * wl.shape[0]
    TRACE.append(("c_embedding", [wa.dims_mapping, xa.dims_mapping], [oa.dims_mapping, sorted(oa._partial_dims())]))
    out = T.embedding(il, wl, padding_idx, st)
    return _wrap(out, dm, oa, list(ids.shape) + [w.shape[-1]])
