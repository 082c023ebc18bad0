"""N-D rank topology and hybrid communicate groups (reference: fleet/base/topology.py:70 CommunicateTopology,
:189 HybridCommunicateGroup, ParallelMode :300-336).

Axis order defaults to Paddle's ``[data, pipe, sharding, sep, model]``: ``model`` (TP) is the
fastest-varying axis, so a TP group is always a block of consecutive ranks — on an 8-GPU MI355X
node every TP pair/quad sits on directly-linked xGMI peers, and PP/DP/sharding groups stride across.
"""
from __future__ import annotations

import itertools

import numpy as np

from .. import base  # noqa: F401
from ... import collective as C


class ParallelMode:
    DATA_PARALLEL = 0
    TENSOR_PARALLEL = 1
    PIPELINE_PARALLEL = 2
    SHARDING_PARALLEL = 3
    SEGMENT_PARALLEL = 4


class CommunicateTopology:
    def __init__(self, hybrid_group_names=("data", "pipe", "sharding", "sep", "model"), dims=(1, 1, 1, 1, 1)):
        self._parallel_names = list(hybrid_group_names)
        self._dims = [int(d) for d in dims]
        self._world_size = int(np.prod(self._dims))
        self._coords = list(itertools.product(*[range(d) for d in self._dims]))
        self._coord2rank = {c: i for i, c in enumerate(self._coords)}

    def get_hybrid_group_names(self):
        return self._parallel_names

    def get_dim(self, axis_name):
        return self._dims[self._parallel_names.index(axis_name)]

    get_dim_size = get_dim

    def world_size(self):
        return self._world_size

    def get_rank(self, **kw):
        c = tuple(kw[n] for n in self._parallel_names)
        return self._coord2rank[c]

    def get_coord(self, rank):
        return dict(zip(self._parallel_names, self._coords[rank]))

    def get_axis_list(self, axis_name, index):
        ax = self._parallel_names.index(axis_name)
        return [r for r, c in enumerate(self._coords) if c[ax] == index]

    def get_comm_list(self, axis_name):
        """All rank lists that form one group along ``axis_name`` (other coords fixed)."""
        ax = self._parallel_names.index(axis_name)
        others = [range(d) for i, d in enumerate(self._dims) if i != ax]
        out = []
        for oc in itertools.product(*others):
            ranks = []
            for k in range(self._dims[ax]):
                c = list(oc)
                c.insert(ax, k)
                ranks.append(self._coord2rank[tuple(c)])
            out.append(ranks)
        return out

    def get_fused_ranks(self, fused_axis):
        """Rank lists for groups spanning several axes (e.g. dp x sep, pp x mp)."""
        axes = [self._parallel_names.index(a) for a in fused_axis]
        others = [i for i in range(len(self._dims)) if i not in axes]
        out = []
        for oc in itertools.product(*[range(self._dims[i]) for i in others]):
            ranks = []
            for fc in itertools.product(*[range(self._dims[i]) for i in axes]):
                c = [0] * len(self._dims)
                for i, v in zip(others, oc):
                    c[i] = v
                for i, v in zip(axes, fc):
                    c[i] = v
                ranks.append(self._coord2rank[tuple(c)])
            out.append(sorted(ranks))
        return out

    def get_rank_from_stage(self, global_rank, **kw):
        coord = self.get_coord(global_rank)
        coord.update(kw)
        return self.get_rank(**coord)


class HybridCommunicateGroup:
    def __init__(self, topology: CommunicateTopology):
        self._topo = topology
        self.global_rank = C.get_rank()
        self.nranks = topology.world_size()
        names = topology.get_hybrid_group_names()
        self._dp_degree = topology.get_dim("data") if "data" in names else 1
        self._mp_degree = topology.get_dim("model") if "model" in names else 1
        self._pp_degree = topology.get_dim("pipe") if "pipe" in names else 1
        self._sharding_degree = topology.get_dim("sharding") if "sharding" in names else 1
        self._sep_degree = topology.get_dim("sep") if "sep" in names else 1
        self._groups = {}
        for axis in names:
            self._groups[axis] = self._make(topology.get_comm_list(axis))
        self._groups["dp_sep"] = self._make(topology.get_fused_ranks(["data", "sep"])) if "sep" in names else \
            self._groups["data"]
        self._groups["pp_mp"] = self._make(topology.get_fused_ranks(["pipe", "model"]))
        # check group: ranks that hold the same model shard along non-replicated axes
        self._groups["check"] = self._make(topology.get_fused_ranks(
            [a for a in names if a in ("model", "pipe", "sharding")] or ["model"]))
        coord = topology.get_coord(self.global_rank)
        self.stage_id = coord.get("pipe", 0)
        # warm-up allreduce on the pipe group (topology.py:218)
        if self._pp_degree > 1:
            import torch

            dev = "cuda" if torch.cuda.is_available() else "cpu"
            t = torch.zeros(1, dtype=torch.int32, device=dev if dev == "cpu" else torch.device("cuda", torch.cuda.current_device()))
            C._all_reduce_torch(t, group=self._groups["pipe"])
        # p2p neighbours in the pipeline
        pipe_ranks = self._groups["pipe"].ranks
        i = pipe_ranks.index(self.global_rank)
        self._prev_rank = pipe_ranks[(i - 1) % len(pipe_ranks)]
        self._next_rank = pipe_ranks[(i + 1) % len(pipe_ranks)]

    def _make(self, lists):
        mine = None
        for ranks in lists:
            if len(ranks) == self.nranks and C.get_world_size() == self.nranks:
                g = C._get_default_group() if self.nranks == 1 else C.new_group(ranks)
            else:
                g = C.new_group(ranks)
            if self.global_rank in ranks:
                mine = g
        return mine

    # -------------------------------------------------------------- mode
    def get_parallel_mode(self):
        if self._mp_degree == 1 and self._pp_degree == 1 and self._sharding_degree == 1 and self._sep_degree == 1:
            return ParallelMode.DATA_PARALLEL
        if self._pp_degree > 1:
            return ParallelMode.PIPELINE_PARALLEL
        if self._sep_degree > 1:
            return ParallelMode.SEGMENT_PARALLEL
        if self._mp_degree > 1:
            return ParallelMode.TENSOR_PARALLEL
        return ParallelMode.SHARDING_PARALLEL

    def topology(self):
        return self._topo

    def get_global_rank(self):
        return self.global_rank

    # -------------------------------------------------------------- per-axis accessors
    def _rank_in(self, axis):
        g = self._groups[axis]
        return g.rank if g is not None else 0

    def get_data_parallel_rank(self):
        return self._rank_in("data")

    def get_data_parallel_world_size(self):
        return self._dp_degree

    def get_data_parallel_group(self):
        return self._groups["data"]

    def get_data_parallel_group_src_rank(self):
        return self._groups["data"].ranks[0]

    def get_model_parallel_rank(self):
        return self._rank_in("model")

    def get_model_parallel_world_size(self):
        return self._mp_degree

    def get_model_parallel_group(self):
        return self._groups["model"]

    def get_model_parallel_group_src_rank(self):
        return self._groups["model"].ranks[0]

    def get_stage_id(self):
        return self.stage_id

    def get_pipe_parallel_world_size(self):
        return self._pp_degree

    def get_pipe_parallel_group(self):
        return self._groups["pipe"]

    def is_first_stage(self):
        return self.stage_id == 0

    def is_last_stage(self):
        return self.stage_id == self._pp_degree - 1

    def get_sharding_parallel_rank(self):
        return self._rank_in("sharding")

    def get_sharding_parallel_world_size(self):
        return self._sharding_degree

    def get_sharding_parallel_group(self):
        return self._groups["sharding"]

    def get_sharding_parallel_group_src_rank(self):
        return self._groups["sharding"].ranks[0]

    def get_sep_parallel_rank(self):
        return self._rank_in("sep") if "sep" in self._groups else 0

    def get_sep_parallel_world_size(self):
        return self._sep_degree

    def get_sep_parallel_group(self):
        return self._groups.get("sep")

    def get_data_sep_parallel_group(self):
        return self._groups["dp_sep"]

    def get_pp_mp_parallel_group(self):
        return self._groups["pp_mp"]

    def get_check_parallel_group(self, sharding=False):
        return self._groups["check"]

    def get_p2p_groups(self):
        return self._prev_rank, self._next_rank

    @property
    def prev_rank(self):
        return self._prev_rank

    @property
    def next_rank(self):
        return self._next_rank

    def get_rank_from_stage(self, stage_id, **kw):
        return self._topo.get_rank_from_stage(self.global_rank, pipe=stage_id, **kw)
