"""Reshard engine for DistTensors on the framework's own collective calls (reference:
paddle/phi/core/distributed/auto_parallel/reshard/ — s_to_r_reshard_function.cc:45 (all-gather),
p_to_r :66 (all-reduce), p_to_s :70 (reduce-scatter), s_to_s :101 (all-to-all), r_to_s (local slice),
r_to_p (keep on one rank), nd_mesh_reshard_function.cc (one mesh dim at a time)).

A DistTensor (dist_tensor.py: local shard + MeshGroups + placements) moves between two placements here, per mesh
dimension, with collectives on that dimension's process group (``MeshGroups.get_group(dim)`` — the framework's
ProcessGroupRCCL over xGMI on the GPU, gloo on the CPU).  Order per mesh dim follows the reference's nd-mesh function: partial dims are
resolved first (p->r / p->s), then shard moves (s->s / s->r), then new shards (r->s) — so a reduction is never
applied to data that was already replicated by a gather.

``reshard(dt, placements)`` is differentiable: the backward reshards the gradient from the target placements
back to the source placements with the same engine; a replicated gradient flowing back into a partial source
stays replicated (converting it to partial would only force a later reduction — torch's ``is_backward`` rule).

Shards must divide evenly (the LLM shapes do); an uneven shard raises instead of silently padding.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .placement import Partial as _TPartial
from .placement import Replicate as _TReplicate
from .placement import Shard as _TShard

_RED = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.AVG, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN}
COMM_LOG = []   # (kind, mesh_dim) of every collective issued (tests assert the expected plan)


def _group(mesh, dim):
    return mesh.get_group(dim)


def _coord(mesh, dim):
    return mesh.get_local_rank(dim)


def _all_gather(x, axis, mesh, dim):
    g = _group(mesh, dim)
    n = dist.get_world_size(g)
    xm = x.movedim(axis, 0).contiguous()
    out = torch.empty((n * xm.shape[0],) + tuple(xm.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, xm, group=g)
    COMM_LOG.append(("all_gather", dim))
    return out.movedim(0, axis).contiguous()


def _all_reduce(x, op, mesh, dim):
    g = _group(mesh, dim)
    y = x.contiguous().clone()
    if op == "avg" and dist.get_backend(g) == "gloo":
        dist.all_reduce(y, op=dist.ReduceOp.SUM, group=g)
        y.div_(dist.get_world_size(g))
    else:
        dist.all_reduce(y, op=_RED[op], group=g)
    COMM_LOG.append(("all_reduce", dim))
    return y


def _reduce_scatter(x, axis, op, mesh, dim):
    g = _group(mesh, dim)
    n = dist.get_world_size(g)
    xm = x.movedim(axis, 0).contiguous()
    if xm.shape[0] % n:
        raise ValueError(f"reshard p->s: axis {axis} of size {xm.shape[0]} does not split over {n} ranks")
    out = torch.empty((xm.shape[0] // n,) + tuple(xm.shape[1:]), dtype=x.dtype, device=x.device)
    avg_gloo = op == "avg" and dist.get_backend(g) == "gloo"
    dist.reduce_scatter_tensor(out, xm, op=dist.ReduceOp.SUM if avg_gloo else _RED[op], group=g)
    if avg_gloo:
        out.div_(n)
    COMM_LOG.append(("reduce_scatter", dim))
    return out.movedim(0, axis).contiguous()


def _all_to_all(x, src_axis, dst_axis, mesh, dim):
    """Shard(src_axis) -> Shard(dst_axis) over one mesh dim: split dst_axis into n blocks, exchange, concatenate
    the received blocks along src_axis."""
    g = _group(mesh, dim)
    n = dist.get_world_size(g)
    if x.shape[dst_axis] % n:
        raise ValueError(f"reshard s->s: axis {dst_axis} of size {x.shape[dst_axis]} does not split over {n}")
    blocks = [b.contiguous() for b in x.chunk(n, dim=dst_axis)]
    inp = torch.stack(blocks)                       # [n, ...block]
    out = torch.empty_like(inp)
    dist.all_to_all_single(out, inp, group=g)
    COMM_LOG.append(("all_to_all", dim))
    return torch.cat(list(out.unbind(0)), dim=src_axis)


def _slice(x, axis, mesh, dim):
    n = mesh.size(dim)
    if x.shape[axis] % n:
        raise ValueError(f"reshard r->s: axis {axis} of size {x.shape[axis]} does not split over {n} ranks")
    return x.chunk(n, dim=axis)[_coord(mesh, dim)].contiguous()


def _to_partial(x, mesh, dim):
    """r -> p(sum): the value lives on coordinate 0 of the mesh dim, zeros elsewhere."""
    return x.clone() if _coord(mesh, dim) == 0 else torch.zeros_like(x)


def _red_name(p):
    return p.reduce_op


def reshard_local(local, mesh, src, dst, backward=False):
    """Move ``local`` (this rank's piece under placements ``src``) to placements ``dst`` (tuples of torch
    placements, one per mesh dim)."""
    cur = list(src)
    x = local
    nd = mesh.ndim
    # 1. partial dims: reduce (to replicate or straight into a shard)
    for d in range(nd):
        s, t = cur[d], dst[d]
        if isinstance(s, _TPartial) and not isinstance(t, _TPartial):
            if isinstance(t, _TShard) and not any(isinstance(c, _TShard) and c.dim == t.dim for c in cur):
                x = _reduce_scatter(x, t.dim, _red_name(s), mesh, d)
                cur[d] = t
            else:
                x = _all_reduce(x, _red_name(s), mesh, d)
                cur[d] = _TReplicate()
    # 2. shard moves: s->s (all-to-all) when the target axis is free, else s->r (all-gather).  Innermost mesh dim
    #    first (reference nd_mesh_reshard_function.cc:149): a tensor axis sharded over several mesh dims was split
    #    outer dim first, so it must be gathered inner dim first or the pieces come back interleaved.
    for d in reversed(range(nd)):
        s, t = cur[d], dst[d]
        if isinstance(s, _TShard) and s != t:
            if isinstance(t, _TShard) and not any(isinstance(c, _TShard) and c.dim == t.dim
                                                  for i, c in enumerate(cur) if i != d):
                x = _all_to_all(x, s.dim, t.dim, mesh, d)
                cur[d] = t
            else:
                x = _all_gather(x, s.dim, mesh, d)
                cur[d] = _TReplicate()
    # 3. new shards / partials from replicated data (no communication)
    for d in range(nd):
        s, t = cur[d], dst[d]
        if isinstance(s, _TReplicate) and isinstance(t, _TShard):
            x = _slice(x, t.dim, mesh, d)
            cur[d] = t
        elif isinstance(s, _TReplicate) and isinstance(t, _TPartial):
            if not backward:   # backward: keep a replicated gradient replicated (see module doc)
                x = _to_partial(x, mesh, d)
            cur[d] = t
    return x


class _Reshard(torch.autograd.Function):
    @staticmethod
    def forward(ctx, dt, mesh, src, dst):
        from .dist_tensor import DistTensor

        ctx.mesh, ctx.src, ctx.dst = mesh, src, dst
        local = reshard_local(dt._local_tensor, mesh, src, dst)
        return DistTensor(local, mesh, dst, dt.shape)

    @staticmethod
    def backward(ctx, g):
        from .dist_tensor import DistTensor

        if not isinstance(g, DistTensor):
            return None, None, None, None
        gsrc = tuple(g.placements)
        tgt = tuple(_TReplicate() if isinstance(p, _TPartial) and isinstance(q, _TReplicate) else p
                    for p, q in zip(ctx.src, gsrc))
        local = reshard_local(g._local_tensor, ctx.mesh, gsrc, tgt, backward=True)
        return DistTensor(local, ctx.mesh, tgt, g.shape), None, None, None


def reshard(dt, placements):
    """Differentiable reshard of a DistTensor to ``placements`` (one per mesh dim)."""
    dst = tuple(placements)
    src = tuple(dt.placements)
    if src == dst:
        return dt
    return _Reshard.apply(dt, dt.device_mesh, src, dst)


# ------------------------------------------------------------------------------------------- cross-mesh
def _local_shape(shape, mesh_shape, placements):
    out = list(shape)
    for d, p in enumerate(placements):
        if isinstance(p, _TShard):
            if out[p.dim] % mesh_shape[d]:
                raise ValueError(f"cross-mesh reshard: axis {p.dim} of size {out[p.dim]} does not split over "
                                 f"{mesh_shape[d]} ranks")
            out[p.dim] //= mesh_shape[d]
    return out


def reshard_cross_mesh(dt, dst_mesh, dst_placements):
    """DistTensor on one process mesh -> DistTensor on another (reference reshard/same_status_reshard_function.cc and
    the cross-mesh path of nd_mesh_reshard_function.cc).

    * same status (meshes of one shape, identical placements): every source coordinate sends its local shard to
      the destination rank at the same coordinate (point-to-point, no collective);
    * otherwise: the source mesh first resolves its placements to Replicate with the same-mesh engine
      (all-reduce / all-gather), source rank k % |src| sends the full tensor to destination rank k, and each
      destination rank slices (or makes partial) its piece.

    Every rank of both meshes must call it.  Ranks outside the destination mesh get a DistTensor without local
    data.  Forward only (a
    pipeline-stage hand-off differentiates through its own send / recv pair)."""
    src_dm = dt.device_mesh
    src_ranks = src_dm.mesh.flatten().tolist()
    dst_ranks = dst_mesh.mesh.flatten().tolist()
    me = dist.get_rank()
    shape, dtype = tuple(dt.shape), dt.dtype
    dst_placements = tuple(dst_placements)
    dev = dt._local_tensor.device if me in src_ranks else (
        torch.device("cuda", torch.cuda.current_device()) if dst_mesh.device_type == "cuda" else torch.device("cpu"))
    same = tuple(src_dm.mesh.shape) == tuple(dst_mesh.mesh.shape) and tuple(dt.placements) == dst_placements
    local = None
    if same:
        if me in src_ranks:
            peer = dst_ranks[src_ranks.index(me)]
            if peer == me:
                local = dt._local_tensor
            else:
                dist.send(dt._local_tensor.contiguous(), peer)
                COMM_LOG.append(("send", -1))
        if me in dst_ranks and local is None:
            peer = src_ranks[dst_ranks.index(me)]
            local = torch.empty(_local_shape(shape, list(dst_mesh.mesh.shape), dst_placements), dtype=dtype,
                                device=dev)
            dist.recv(local, peer)
            COMM_LOG.append(("recv", -1))
    else:
        full = None
        if me in src_ranks:
            full = reshard_local(dt._local_tensor, src_dm, tuple(dt.placements),
                                 tuple(_TReplicate() for _ in range(src_dm.ndim))).contiguous()
        for j, d in enumerate(dst_ranks):
            s = src_ranks[j % len(src_ranks)]
            if s == d:
                continue
            if me == s:
                dist.send(full, d)
                COMM_LOG.append(("send", -1))
            elif me == d:
                full = torch.empty(shape, dtype=dtype, device=dev)
                dist.recv(full, s)
                COMM_LOG.append(("recv", -1))
        if me in dst_ranks:
            local = reshard_local(full, dst_mesh, tuple(_TReplicate() for _ in range(dst_mesh.ndim)), dst_placements)
    if me not in dst_ranks:  # a non-member holds the DistTensor's metadata with no local data
        local = torch.empty(0, dtype=dtype, device=dev)
    from .dist_tensor import DistTensor

    return DistTensor(local, dst_mesh, dst_placements, shape)
