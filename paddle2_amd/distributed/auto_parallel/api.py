"""Semi-automatic parallelism: ProcessMesh, placements and DistTensor (reference:
python/paddle/distributed/auto_parallel/api.py — ``shard_tensor`` :206, ``dtensor_from_fn`` :665,
``reshard`` :705, ``shard_layer`` :806, ``shard_optimizer`` :1261-1641 (ShardingStage1/2/3),
``shard_dataloader`` :3208, ``to_static``/``DistModel`` :2110/:2693, ``unshard_dtensor`` :2854;
process_mesh.py; placement_type.py).

MI355X design: a Paddle DistTensor is our Tensor whose storage is the framework's own ``DistTensor``
(dist_tensor.py: local shard + the ProcessMesh's communicators + placements).  The framework's hot ops (norms,
linear, RoPE, flash attention, SwiGLU, embedding) dispatch DistTensor arguments at op entry through the SPMD rules
of ``spmd_rules.py`` and the reshard engine (``dist_ops.py`` / ``reshard.py``), running the native kernels on the
local shards; every other op goes through DistTensor's aten-level SPMD dispatch; ``reshard`` below uses the same
engine.
"""
from __future__ import annotations

import copy

import numpy as np
import torch

from ...framework.tensor import Tensor
from ...framework.place import current_torch_device

_wrap = Tensor._wrap


# ----------------------------------------------------------------------------- placements
from .placement import MeshGroups, Partial, Placement, Replicate, Shard  # noqa: E402,F401
from .dist_tensor import DistTensor, distribute_tensor  # noqa: E402


# ----------------------------------------------------------------------------- ProcessMesh
_MESH_CACHE: dict = {}


class ProcessMesh:
    def __init__(self, mesh=None, dim_names=None, shape=None, process_ids=None):
        if mesh is None:
            mesh = np.array(process_ids).reshape(shape)
        self._mesh = np.array(mesh, dtype=np.int64)
        if dim_names is None:
            dim_names = [f"d{i}" for i in range(self._mesh.ndim)]
        assert len(dim_names) == self._mesh.ndim
        self._dim_names = list(dim_names)

    @property
    def mesh(self):
        return self._mesh

    @property
    def shape(self):
        return list(self._mesh.shape)

    @property
    def ndim(self):
        return self._mesh.ndim

    @property
    def dim_names(self):
        return self._dim_names

    @property
    def process_ids(self):
        return self._mesh.reshape(-1).tolist()

    def get_dim_size(self, dim):
        if isinstance(dim, str):
            dim = self._dim_names.index(dim)
        return self._mesh.shape[dim]

    def get_mesh_with_dim(self, dim_name, index=None):
        ax = self._dim_names.index(dim_name)
        order = [ax] + [i for i in range(self.ndim) if i != ax]
        m = np.transpose(self._mesh, order)
        names = [self._dim_names[i] for i in order]
        if index is None:
            return ProcessMesh(m, names)
        return ProcessMesh(m[index], names[1:])

    def __getitem__(self, idx):
        sub = self._mesh[idx]
        if np.ndim(sub) == 0:
            return ProcessMesh(np.array([int(sub)]), [self._dim_names[-1]])
        kept = [n for n, s in zip(self._dim_names, (idx if isinstance(idx, tuple) else (idx,)))
                if isinstance(s, slice)]
        kept += self._dim_names[len(idx) if isinstance(idx, tuple) else 1:]
        return ProcessMesh(sub, kept[:np.ndim(sub)])

    def contains(self, rank):
        return rank in self.process_ids

    def __eq__(self, o):
        return isinstance(o, ProcessMesh) and np.array_equal(o._mesh, self._mesh) and o._dim_names == self._dim_names

    def __hash__(self):
        return hash((self._mesh.tobytes(), tuple(self._mesh.shape), tuple(self._dim_names)))

    def __repr__(self):
        return f"ProcessMesh(shape={self.shape}, process_ids={self.process_ids}, dim_names={self._dim_names})"

    def _device_mesh(self):
        """The mesh's communicators (placement.MeshGroups; collective: every rank builds them in the same order)."""
        key = hash(self)
        dm = _MESH_CACHE.get(key)
        if dm is None:
            from .. import collective as C

            C.init_parallel_env()
            dm = MeshGroups(self._mesh, self._dim_names, current_torch_device().type)
            _MESH_CACHE[key] = dm
        return dm


_global_mesh = None


def set_mesh(mesh):
    global _global_mesh
    _global_mesh = mesh


def get_mesh():
    return _global_mesh


# ----------------------------------------------------------------------------- DistTensor API
def _placements(mesh, placements):
    out = list(placements)
    while len(out) < mesh.ndim:
        out.append(Replicate())
    return tuple(out)


def is_dist_tensor(t):
    return isinstance(getattr(t, "_t", None), DistTensor)


def _attach(w, mesh):
    w.process_mesh = mesh
    return w


def shard_tensor(data, mesh, placements, dtype=None, place=None, stop_gradient=None):
    """Distribute a (replicated, identical on every rank) global tensor by ``placements``."""
    from ...framework.tensor import to_tensor
    from .reshard import reshard as _own

    t = data if isinstance(data, Tensor) else to_tensor(data, dtype=dtype)
    src = t._t
    if dtype is not None:
        from ...framework.dtype import convert_dtype

        src = src.to(convert_dtype(dtype))
    dm = mesh._device_mesh()
    if isinstance(src, DistTensor):
        out = _own(src, _placements(mesh, placements))
    else:
        src = src.to("cpu" if dm.device_type == "cpu" else current_torch_device())
        out = distribute_tensor(src.detach(), dm, _placements(mesh, placements))
    sg = t.stop_gradient if stop_gradient is None else stop_gradient
    if isinstance(t, Tensor) and hasattr(t, "trainable") and type(t).__name__ in ("Parameter", "EagerParamBase"):
        from ...framework.param import Parameter

        p = Parameter(out.detach(), name=getattr(t, "name", None))
        p.stop_gradient = sg
        return _attach(p, mesh)
    out = out.detach().requires_grad_(not sg) if not sg else out.detach()
    return _attach(_wrap(out), mesh)


def dtensor_from_local(local_tensor, mesh, placements):
    lt = local_tensor._t if isinstance(local_tensor, Tensor) else local_tensor
    out = DistTensor.from_local(lt, mesh._device_mesh(), _placements(mesh, placements))
    return _attach(_wrap(out), mesh)


def dtensor_from_fn(fn, mesh, placements, *args, **kwargs):
    return shard_tensor(fn(*args, **kwargs), mesh, placements)


def reshard(dist_tensor, mesh, placements):
    """Same mesh: the framework's reshard engine (reshard.py: s->r all-gather, p->r all-reduce, p->s
    reduce-scatter, s->s all-to-all, r->s slice; differentiable).  A different mesh: the cross-mesh path
    (reshard.reshard_cross_mesh: p2p for same-status meshes, else replicate -> send -> slice); ranks outside the
    destination mesh hold no local data."""
    t = dist_tensor._t
    assert isinstance(t, DistTensor), "reshard expects a DistTensor"
    dm = mesh._device_mesh()
    if dm == t.device_mesh:
        from .reshard import reshard as _own

        return _attach(_wrap(_own(t, _placements(mesh, placements))), mesh)
    from .reshard import reshard_cross_mesh

    return _attach(_wrap(reshard_cross_mesh(t, dm, _placements(mesh, placements))), mesh)


def unshard_dtensor(dist_tensor):
    t = dist_tensor._t
    if isinstance(t, DistTensor):
        return _wrap(t.full_tensor())
    return dist_tensor


def local_tensor(dist_tensor):
    t = dist_tensor._t
    return _wrap(t.to_local()) if isinstance(t, DistTensor) else dist_tensor


def placements_of(dist_tensor):
    t = dist_tensor._t
    return list(t.placements) if isinstance(t, DistTensor) else None


def shard_layer(layer, process_mesh, shard_fn=None, input_fn=None, output_fn=None):
    """Convert every parameter of ``layer`` to a DistTensor: ``shard_fn(name, sublayer, mesh)`` may
    shard some of them itself; the rest are replicated over the mesh."""
    from ...framework.param import Parameter

    if shard_fn is not None:
        for name, sub in layer.named_sublayers(include_self=True):
            shard_fn(name, sub, process_mesh)
    for name, sub in layer.named_sublayers(include_self=True):
        for pname, p in list(sub._parameters.items()):
            if p is None or is_dist_tensor(p):
                continue
            d = distribute_tensor(p._t.detach(), process_mesh._device_mesh(), _placements(process_mesh, []))
            np_ = Parameter(d, name=p.name)
            np_.stop_gradient = p.stop_gradient
            np_.process_mesh = process_mesh
            sub._parameters[pname] = np_
    if input_fn is not None:
        layer.register_forward_pre_hook(lambda l, inp: input_fn(inp, process_mesh))
    if output_fn is not None:
        layer.register_forward_post_hook(lambda l, inp, out: output_fn(out, process_mesh))
    return layer


class _ShardingStageBase:
    def __init__(self, mesh_dim=None, mesh=None, sharding_mesh_dim=None):
        self._mesh = mesh or get_mesh()
        self._dim = mesh_dim if mesh_dim is not None else sharding_mesh_dim
        if self._dim is None:
            self._dim = 0

    def _placements_for(self, param):
        """Optimizer-state placements: param's own placements with the sharding dim set to Shard(0)."""
        t = param._t
        mesh = getattr(param, "process_mesh", self._mesh)
        if isinstance(t, DistTensor):
            pl = list(t.placements)
        else:
            pl = [Replicate()] * mesh.ndim
        ax = mesh.dim_names.index(self._dim) if isinstance(self._dim, str) else int(self._dim)
        if isinstance(pl[ax], Replicate) and t.shape[0] % mesh.shape[ax] == 0:
            pl[ax] = Shard(0)
        return mesh, pl


class ShardingStage1(_ShardingStageBase):
    stage = 1


class ShardingStage2(_ShardingStageBase):
    stage = 2


class ShardingStage3(_ShardingStageBase):
    stage = 3


class _ShardOptimizer:
    """Optimizer whose accumulators (and, for stage 3, parameters) are sharded over a mesh dim."""

    def __init__(self, optimizer, shard_fn=None, gradient_accumulation_steps=1):
        self._inner_opt = optimizer
        self._shard_fn = shard_fn
        self._gas = gradient_accumulation_steps
        if shard_fn is not None:
            orig_acc = optimizer._acc

            def sharded_acc(name, p, like=None, dtype=torch.float32, fill=0.0, _orig=orig_acc):
                d = optimizer._accumulators[name]
                t = d.get(p.name)
                if t is None and isinstance(p._t, DistTensor):
                    mesh, pl = shard_fn._placements_for(p)
                    full = torch.full(tuple(p._t.shape), fill, dtype=dtype, device=p._t._local_tensor.device)
                    t = distribute_tensor(full, mesh._device_mesh(), pl)
                    d[p.name] = t
                    return t
                return _orig(name, p, like, dtype, fill)

            optimizer._acc = sharded_acc

    def step(self):
        self._inner_opt.step()

    def clear_grad(self, set_to_zero=True):
        self._inner_opt.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def state_dict(self):
        return self._inner_opt.state_dict()

    def set_state_dict(self, sd):
        return self._inner_opt.set_state_dict(sd)

    def __getattr__(self, name):
        return getattr(self._inner_opt, name)


def shard_optimizer(optimizer, shard_fn=None, gradient_accumulation_steps=1):
    return _ShardOptimizer(optimizer, shard_fn, gradient_accumulation_steps)


def shard_scaler(scaler):
    return scaler


class ShardDataloader:
    """Yields batches as DistTensors sharded on the batch dim over ``shard_dims`` of the mesh."""

    def __init__(self, dataloader, meshes, input_keys=None, shard_dims=None, is_dataset_splitted=False):
        self._dl = dataloader
        self._mesh = meshes[0] if isinstance(meshes, (list, tuple)) else meshes
        self._dims = shard_dims
        self._split = is_dataset_splitted

    def _convert(self, x):
        if isinstance(x, Tensor):
            mesh = self._mesh
            pl = [Replicate()] * mesh.ndim
            if self._dims is not None:
                ax = mesh.dim_names.index(self._dims) if isinstance(self._dims, str) else int(self._dims)
                pl[ax] = Shard(0)
            if self._split:
                return dtensor_from_local(x, mesh, pl)
            return shard_tensor(x, mesh, pl)
        if isinstance(x, (list, tuple)):
            return type(x)(self._convert(e) for e in x)
        if isinstance(x, dict):
            return {k: self._convert(v) for k, v in x.items()}
        return x

    def __iter__(self):
        for batch in self._dl:
            yield self._convert(batch)

    def __len__(self):
        return len(self._dl)


def shard_dataloader(dataloader, meshes, input_keys=None, shard_dims=None, is_dataset_splitted=False):
    return ShardDataloader(dataloader, meshes, input_keys, shard_dims, is_dataset_splitted)


class Strategy:
    """auto_parallel Strategy (config namespaces only; the dygraph engine reads sharding/amp/gradient merge)."""

    class _NS(dict):
        def __getattr__(self, k):
            return self.get(k)

        def __setattr__(self, k, v):
            self[k] = v

    def __init__(self, config=None):
        config = config or {}
        for ns in ("sharding", "amp", "recompute", "pipeline", "gradient_merge", "fused_passes"):
            setattr(self, ns, Strategy._NS(config.get(ns, {"enable": False})))


class DistModel:
    """Static-graph training engine behind ``dist.to_static`` (reference: auto_parallel/api.py DistModel +
    static/engine.py).  The first call records the train step (forward, loss, backward, optimizer) into a
    Program for the micro-batch shape; the strategy's pipeline / gradient-merge settings become a job plan
    (distributed/passes: FThenB, 1F1B, Eager1F1B, VPP, ZBH1) that ``PlanExecutor`` runs over the micro-batches,
    averaging gradients over data-parallel ranks once per step.  ``strategy.amp`` records the step under
    auto_cast.  eval() records forward + loss, predict() forward only."""

    def __init__(self, layer, loader=None, loss=None, optimizer=None, strategy=None, metrics=None, input_spec=None):
        self._layer = layer
        self._loss = loss
        self._opt = optimizer
        self._strategy = strategy or Strategy()
        self._mode = "train" if optimizer is not None else ("eval" if loss is not None else "predict")
        self.dist_loader = loader
        pp = self._strategy.pipeline
        gm = self._strategy.gradient_merge
        self._micro = int(pp.get("accumulate_steps") or 0) if pp.get("enable") else 0
        if not self._micro and gm.get("enable"):
            self._micro = int(gm.get("k_steps") or 1)
        self._micro = max(self._micro, 1)
        self._schedule = pp.get("schedule_mode") or "1F1B"
        self._cache = {}

    def train(self):
        self._mode = "train"
        self._layer.train()

    def eval(self):
        self._mode = "eval"
        self._layer.eval()

    def predict(self):
        self._mode = "predict"
        self._layer.eval()

    # ---------------------------------------------------------------- recording
    def _record(self, mode, inputs, labels):
        from ... import static
        from ...amp import auto_cast
        from ...static import graph as g

        prog = static.Program()
        was = g._state.static
        g._state.static = True
        amp = self._strategy.amp
        try:
            with static.program_guard(prog, static.Program()):
                xs = [static.data(f"input_{i}", list(t.shape), t.dtype) for i, t in enumerate(inputs)]
                ys = [static.data(f"label_{i}", list(t.shape), t.dtype) for i, t in enumerate(labels)]
                ctx = auto_cast(True, level=amp.get("level", "O1").upper(), dtype=amp.get("dtype", "bfloat16")) \
                    if amp.get("enable") else _null()
                with ctx:
                    out = self._layer(*xs)
                    loss = self._loss(out, *ys) if (mode != "predict" and self._loss is not None) else None
                if mode == "train":
                    self._opt.minimize(loss)
        finally:
            g._state.static = was
        feeds = [f"input_{i}" for i in range(len(inputs))] + [f"label_{i}" for i in range(len(labels))]
        return prog, feeds, out, loss

    def _split(self, tensors):
        n = self._micro
        outs = []
        for t in tensors:
            if t.shape[0] % n:
                raise ValueError(f"batch {t.shape[0]} is not divisible into {n} micro-batches")
            outs.append(t.split(n) if isinstance(t, Tensor) else None)   # n equal sections
        return outs

    # ---------------------------------------------------------------- step
    def __call__(self, *args):
        from ..passes import PlanExecutor, create_job_list, split_program
        from ..passes.pipeline_scheduler_pass import FORWARD, Job, Plan

        args = [a if isinstance(a, Tensor) else Tensor._wrap(torch.as_tensor(a)) for a in args]
        if self._mode == "predict":
            inputs, labels = args, []
        else:
            inputs, labels = args[:-1], args[-1:]
        n = self._micro if self._mode == "train" else 1
        parts = self._split(list(inputs) + list(labels)) if n > 1 else [[a] for a in list(inputs) + list(labels)]
        micro = [[p[i] for p in parts] for i in range(n)]
        key = (self._mode, tuple((tuple(t.shape), str(t.dtype)) for t in micro[0]))
        if key not in self._cache:
            self._cache[key] = self._record(self._mode, micro[0][:len(inputs)], micro[0][len(inputs):])
        prog, feeds, out, loss = self._cache[key]
        micro_feeds = [dict(zip(feeds, m)) for m in micro]
        if self._mode == "train":
            pp = self._strategy.pipeline
            plan = Plan(create_job_list(self._schedule, n, int(pp.get("pp_stage") or 0),
                                        int(pp.get("pp_degree") or 1), int(pp.get("vpp_degree") or 1)),
                        split_program(prog))
            res = PlanExecutor().run(prog, plan, micro_feeds, [loss])
            return Tensor._wrap(torch.stack([r[0].detach() for r in res]).mean())
        plan = Plan([Job(FORWARD, 0)], split_program(prog))
        res = PlanExecutor().run(prog, plan, micro_feeds, [loss] if self._mode == "eval" else [out])
        return Tensor._wrap(res[0][0].detach())

    def state_dict(self, mode="all"):
        sd = dict(self._layer.state_dict())
        if mode in ("all", "opt") and self._opt is not None:
            sd.update(self._opt.state_dict())
        return sd

    def set_state_dict(self, sd):
        self._layer.set_state_dict(sd)


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def to_static(layer, loader=None, loss=None, optimizer=None, strategy=None, input_spec=None):
    return DistModel(layer, loader, loss, optimizer, strategy, input_spec=input_spec)
