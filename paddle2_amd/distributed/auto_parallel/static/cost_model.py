"""Static auto-parallel: cost model + planner (reference python/paddle/distributed/auto_parallel/static/cost/ —
``CostEstimator``, comp_op_cost.py / comm_op_cost.py; tuner/rule_based_tuner.py) for MI355X nodes.

Costs are priced for the hardware this framework targets, not copied from the reference's GPU tables:

* compute: matmul-class ops at ``peak_bf16 * mfma_eff`` (2.5 PF/s dense bf16, 0.6 achieved by the framework's
  GEMMs at LLM shapes), everything else as HBM traffic (inputs + outputs) at ``hbm_bw * hbm_eff`` (8 TB/s);
* communication: RCCL ring collectives over point-to-point xGMI — a GPU has 7 links of ~153 GB/s, and a ring
  over n ranks of a fully connected node can run on min(7, n - 1) links in parallel, so
  all-reduce = 2 (n-1)/n * bytes / bw, all-gather / reduce-scatter / all-to-all = (n-1)/n * bytes / bw, plus a
  per-collective launch latency;
* memory: parameter bytes per rank (local shards) checked against the per-GPU HBM budget (288 GB).

``estimate(ctx)`` walks a completed Program exactly as the partitioner would execute it (same reshard decisions,
local shapes) and returns compute / communication / total seconds with a per-op breakdown.  ``Planner`` searches
parameter placements (exhaustively for small spaces, coordinate descent otherwise) for the lowest estimate under
the memory budget.
"""
from __future__ import annotations

import itertools
import math

import torch
import torch.utils._pytree as pytree

from .completion import Completer, DistAttr, tensor_key

MATMUL_OPS = {"addmm", "mm", "matmul", "bmm", "linear"}


class ClusterSpec:
    def __init__(self, peak_bf16=2.5e15, mfma_eff=0.6, hbm_bw=8e12, hbm_eff=0.8, link_bw=153e9, links=7,
                 coll_eff=0.7, coll_latency=12e-6, hbm_bytes=288e9, dtype_bytes=2):
        self.peak_bf16, self.mfma_eff = peak_bf16, mfma_eff
        self.hbm_bw, self.hbm_eff = hbm_bw, hbm_eff
        self.link_bw, self.links, self.coll_eff, self.coll_latency = link_bw, links, coll_eff, coll_latency
        self.hbm_bytes, self.dtype_bytes = hbm_bytes, dtype_bytes


def _local_shape(shape, attr, mesh_shape):
    return [s // mesh_shape[d] if d != -1 else s for s, d in zip(shape, attr.dims_mapping)]


def reshard_steps(src, dst, nd):
    """The collectives reshard_local would issue for src -> dst (DistAttr): [(kind, mesh_dim)]."""
    steps = []
    cur_dm = list(src.dims_mapping)
    cur_p = set(src.partial)
    for d in range(nd):
        if d in cur_p and d not in dst.partial:
            if d in dst.dims_mapping and d not in cur_dm:
                steps.append(("reduce_scatter", d))
                cur_dm[dst.dims_mapping.index(d)] = d
            else:
                steps.append(("all_reduce", d))
            cur_p.discard(d)
    for d in range(nd):
        if d in cur_dm and cur_dm.index(d) != (dst.dims_mapping.index(d) if d in dst.dims_mapping else -2):
            a = cur_dm.index(d)
            if d in dst.dims_mapping and cur_dm[dst.dims_mapping.index(d)] == -1:
                steps.append(("all_to_all", d))
                cur_dm[a] = -1
                cur_dm[dst.dims_mapping.index(d)] = d
            else:
                steps.append(("all_gather", d))
                cur_dm[a] = -1
    return steps


class CostModel:
    def __init__(self, cluster=None):
        self.c = cluster or ClusterSpec()

    def collective_time(self, kind, nbytes, n):
        if n <= 1 or nbytes <= 0:
            return 0.0
        bw = self.c.link_bw * min(self.c.links, n - 1) * self.c.coll_eff
        factor = 2.0 * (n - 1) / n if kind in ("all_reduce", "grad_all_reduce") else (n - 1) / n
        # all_gather moves the GATHERED size; the others are priced on their input size
        return factor * nbytes / bw + self.c.coll_latency

    def op_time(self, key, in_shapes, out_shapes):
        b = self.c.dtype_bytes
        if key in MATMUL_OPS and len(in_shapes) >= 2 and out_shapes:
            x, w = (in_shapes[1], in_shapes[2]) if key == "addmm" and len(in_shapes) == 3 else in_shapes[:2]
            kdim = w[-1] if key == "linear" else (w[0] if len(w) == 2 else w[-2])
            flops = 2.0 * math.prod(out_shapes[0]) * kdim
            return flops / (self.c.peak_bf16 * self.c.mfma_eff)
        nbytes = b * (sum(math.prod(s) for s in in_shapes) + sum(math.prod(s) for s in out_shapes))
        return nbytes / (self.c.hbm_bw * self.c.hbm_eff)

    def estimate(self, ctx, training=True):
        """-> {"compute_s", "comm_s", "total_s", "param_bytes_per_rank", "ops": [...]}.  training=True adds the
        backward as 2x the forward compute plus each forward collective's conjugate."""
        from ....static.graph import VarRef

        prog, mesh = ctx.program, ctx.mesh
        mshape = mesh.shape
        nd = mesh.ndim
        cur = {}
        comp = comm = 0.0
        ops = []
        params = {}
        feeds = {v._vid for v in prog.feeds.values()}
        for op, plan in zip(prog.ops, ctx.plans):
            if plan is None:
                continue
            leaves = [x for x in pytree.tree_leaves((op.args, op.kwargs))
                      if isinstance(x, VarRef) or (isinstance(x, torch.Tensor) and x.dim() > 0)]
            ins, op_comm = [], 0.0
            for x, req in zip(leaves, plan.in_attrs):
                key = tensor_key(x)
                shape = list(prog.vars[x.vid].shape) if isinstance(x, VarRef) else list(x.shape)
                if not isinstance(x, VarRef) and getattr(x, "_pd_param", None) is not None:
                    a = ctx.attrs.get(key) or DistAttr([-1] * len(shape))
                    params[key] = math.prod(_local_shape(shape, a, mshape)) * self.c.dtype_bytes
                src = cur.get(key) or ctx.attrs.get(key) or DistAttr([-1] * len(shape))
                for kind, d in reshard_steps(src, req, nd):
                    local = _local_shape(shape, src, mshape)
                    nbytes = math.prod(local) * self.c.dtype_bytes
                    if kind == "all_gather":
                        nbytes *= mshape[d]
                    t = self.collective_time(kind, nbytes, mshape[d])
                    op_comm += t * (2.0 if training else 1.0)
                ins.append(_local_shape(shape, req, mshape))
                gd = [d for d in plan.split_dims if d not in req.dims_mapping and d not in req.partial]
                if isinstance(x, VarRef) and x.vid in feeds:
                    gd = []  # data needs no gradient
                if training and gd:  # the replicated input's gradient is summed over the op's split dims
                    nbytes = math.prod(_local_shape(shape, req, mshape)) * self.c.dtype_bytes
                    op_comm += sum(self.collective_time("grad_all_reduce", nbytes, mshape[d]) for d in gd)
            outs = []
            for i, v in enumerate(op.outs):
                if v is None:
                    continue
                a = plan.out_attrs[i]
                cur[("v", v)] = a
                outs.append(_local_shape(list(prog.vars[v].shape), a, mshape))
            t = self.op_time(plan.key, ins, outs) * (3.0 if training else 1.0)
            comp += t
            comm += op_comm
            ops.append({"op": plan.key, "compute_s": t, "comm_s": op_comm})
        pbytes = sum(params.values())
        return {"compute_s": comp, "comm_s": comm, "total_s": comp + comm, "param_bytes_per_rank": pbytes,
                "fits_memory": pbytes * 8 <= self.c.hbm_bytes, "ops": ops}


class Planner:
    """Search parameter placements for the lowest estimated step time (reference rule_based_tuner.py)."""

    def __init__(self, program, mesh, cost_model=None, training=True):
        self.program, self.mesh = program, mesh
        self.cm = cost_model or CostModel()
        self.training = training

    def _cost(self, annotations):
        ctx = Completer(self.mesh).complete(self.program, annotations)
        est = self.cm.estimate(ctx, self.training)
        # equal time: prefer fewer resident parameter bytes (1 GiB ~ 1 us, far below any collective's cost)
        return (est["total_s"] + 1e-15 * est["param_bytes_per_rank"] if est["fits_memory"] else float("inf")), est

    def search(self, fixed, candidates, max_exhaustive=4096):
        """fixed: annotations kept as given; candidates: {param: [placements, ...]} -> (best annotations, est)."""
        keys = list(candidates)
        space = [candidates[k] for k in keys]
        total = math.prod(len(s) for s in space) if space else 1
        best, best_est, best_cost = None, None, float("inf")
        if total <= max_exhaustive:
            for combo in itertools.product(*space):
                ann = dict(fixed)
                ann.update(zip(keys, combo))
                cost, est = self._cost(ann)
                if cost < best_cost:
                    best, best_est, best_cost = ann, est, cost
            return best, best_est
        choice = {k: candidates[k][0] for k in keys}
        improved = True
        while improved:
            improved = False
            for k in keys:
                for opt in candidates[k]:
                    trial = dict(choice)
                    trial[k] = opt
                    cost, est = self._cost({**fixed, **trial})
                    if cost < best_cost - 1e-12:
                        best_cost, best_est, choice, improved = cost, est, trial, True
        return {**fixed, **choice}, best_est
