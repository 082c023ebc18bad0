"""Placements and the device mesh of a DistTensor (reference: python/paddle/distributed/auto_parallel/
placement_type.py, paddle/phi/core/distributed/auto_parallel/placement_types.h, process_mesh.h).

``MeshGroups`` is the runtime side of a ProcessMesh: one communicator (process group) per 1-D slice of the rank
grid along every mesh dimension — the groups the reshard engine's collectives run on (RCCL over xGMI on the GPU,
gloo on the CPU).  Creating them is collective: every rank of the job builds every slice's group in the same order
(``torch.distributed.new_group`` semantics), so a mesh is materialised on all ranks the first time any of them
uses it.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist


class Placement:
    def is_shard(self, dim=None):
        return False

    def is_replicated(self):
        return False

    def is_partial(self):
        return False


class Shard(Placement):
    def __init__(self, dim, **kw):
        self.dim = int(dim)

    def get_dim(self):
        return self.dim

    def is_shard(self, dim=None):
        return dim is None or dim == self.dim

    def __eq__(self, o):
        return isinstance(o, Shard) and o.dim == self.dim

    def __hash__(self):
        return hash(("S", self.dim))

    def __repr__(self):
        return f"Shard(dim={self.dim})"


class Replicate(Placement):
    def is_replicated(self):
        return True

    def __eq__(self, o):
        return isinstance(o, Replicate)

    def __hash__(self):
        return hash("R")

    def __repr__(self):
        return "Replicate()"


_RED_NAMES = {"sum", "avg", "max", "min"}


class Partial(Placement):
    """Each rank holds a term of the value; ``reduce_type`` combines them (a ReduceOp or its name)."""

    def __init__(self, reduce_type=None):
        self.reduce_type = "sum" if reduce_type is None else reduce_type

    @property
    def reduce_op(self):
        """The reduction's name: sum | avg | max | min."""
        r = self.reduce_type
        if isinstance(r, str):
            return r
        try:
            from ..collective import ReduceOp

            return {ReduceOp.SUM: "sum", ReduceOp.AVG: "avg", ReduceOp.MAX: "max", ReduceOp.MIN: "min"}[r]
        except (ImportError, KeyError):
            return "sum"

    def is_partial(self):
        return True

    def __eq__(self, o):
        return isinstance(o, Partial) and o.reduce_op == self.reduce_op

    def __hash__(self):
        return hash(("P", self.reduce_op))

    def __repr__(self):
        return f"Partial(reduce_type={self.reduce_op})"


# ----------------------------------------------------------------------------------------------- mesh groups
_GROUPS: dict = {}


class MeshGroups:
    """A ProcessMesh's rank grid with its per-dimension communicators."""

    def __init__(self, ranks, dim_names=None, device_type="cpu"):
        self.mesh = torch.as_tensor(np.asarray(ranks, dtype=np.int64))
        self.shape = tuple(self.mesh.shape)
        self.ndim = self.mesh.dim()
        self.mesh_dim_names = tuple(dim_names) if dim_names is not None else tuple(f"d{i}" for i in range(self.ndim))
        self.device_type = device_type
        self._rank = dist.get_rank() if dist.is_initialized() else 0
        hit = (self.mesh == self._rank).nonzero()
        self._coord = [int(c) for c in hit[0]] if len(hit) else None
        self._groups = [self._build(d) for d in range(self.ndim)]

    def _build(self, d):
        """The group of the slice along mesh dim ``d`` through this rank (every slice is created on every rank)."""
        if not dist.is_initialized():
            return None
        moved = self.mesh.movedim(d, -1).reshape(-1, self.shape[d])
        mine = None
        for row in moved.tolist():
            key = tuple(row)
            g = _GROUPS.get(key)
            if g is None:
                g = dist.group.WORLD if len(row) == dist.get_world_size() and row == sorted(row) and \
                    row == list(range(len(row))) else dist.new_group(row)
                _GROUPS[key] = g
            if self._rank in row:
                mine = g
        return mine

    def size(self, dim=None):
        return int(self.mesh.numel()) if dim is None else self.shape[dim]

    def get_group(self, dim=0):
        return self._groups[dim]

    def get_local_rank(self, dim=0):
        return self._coord[dim] if self._coord is not None else 0

    def get_coordinate(self):
        return list(self._coord) if self._coord is not None else None

    def contains_me(self):
        return self._coord is not None

    def __deepcopy__(self, memo):
        return self   # communicators are shared, never copied

    def __eq__(self, o):
        return isinstance(o, MeshGroups) and torch.equal(o.mesh, self.mesh)

    def __hash__(self):
        return hash((tuple(self.mesh.reshape(-1).tolist()), self.shape))

    def __repr__(self):
        return f"MeshGroups(shape={list(self.shape)}, ranks={self.mesh.reshape(-1).tolist()})"


def local_shape_and_offset(shape, mesh, placements):
    """This rank's shard shape and its offset in the global tensor (even splits; nested shards of one axis split
    outer mesh dim first)."""
    shape = list(shape)
    local, off = list(shape), [0] * len(shape)
    for d, p in enumerate(placements):
        if isinstance(p, Shard):
            n = mesh.size(d)
            a = p.dim % len(shape)
            if local[a] % n:
                raise ValueError(f"axis {a} of size {local[a]} does not split evenly over {n} ranks")
            local[a] //= n
            off[a] += mesh.get_local_rank(d) * local[a]
    return local, off
