"""paddle.distributed.fleet (reference: fleet/fleet.py:218 init, :674 _init_hybrid_parallel_env,
fleet/model.py:32 distributed_model, fleet/optimizer.py:39 distributed_optimizer)."""
from __future__ import annotations

from ... import distributed as _dist  # noqa: F401
from .. import collective as C
from .base.distributed_strategy import DistributedStrategy, validate_hybrid_configs  # noqa: F401
from .base.topology import CommunicateTopology, HybridCommunicateGroup, ParallelMode  # noqa: F401

_state = {"strategy": None, "hcg": None, "initialized": False, "is_collective": True}


class UserDefinedRoleMaker:
    def __init__(self, is_collective=True, **kw):
        self.is_collective = is_collective


class PaddleCloudRoleMaker(UserDefinedRoleMaker):
    pass


def init(role_maker=None, is_collective=True, strategy=None, log_level="INFO"):
    strategy = strategy or DistributedStrategy()
    if not isinstance(strategy, DistributedStrategy):
        raise TypeError("fleet.init: strategy must be a fleet.DistributedStrategy")
    _state["strategy"] = strategy
    validate_hybrid_configs(strategy)
    C.init_parallel_env()
    world = C.get_world_size()
    hc = strategy.hybrid_configs
    dp = strategy.validate_world(world)  # degrees multiply to the world size, order is a permutation
    mp, pp = hc["mp_degree"], hc["pp_degree"]
    sh, sep = hc["sharding_degree"], hc["sep_degree"]
    hc["dp_degree"] = dp
    order = list(hc["order"])
    name_map = {"dp": "data", "pp": "pipe", "sharding": "sharding", "sep": "sep", "mp": "model"}
    deg = {"dp": dp, "pp": pp, "sharding": sh, "sep": sep, "mp": mp}
    topo = CommunicateTopology([name_map[o] for o in order], [deg[o] for o in order])
    _state["hcg"] = HybridCommunicateGroup(topo)
    _state["initialized"] = True
    if mp > 1:
        from .layers.mpu.random import model_parallel_random_seed

        model_parallel_random_seed()
    return None


def get_hybrid_communicate_group():
    return _state["hcg"]


def _hcg():
    if _state["hcg"] is None:
        init()
    return _state["hcg"]


def worker_index():
    return C.get_rank()


def worker_num():
    return C.get_world_size()


def is_first_worker():
    return C.get_rank() == 0


def is_worker():
    return True


def is_server():
    return False


def barrier_worker():
    C.barrier()


def _apply_model_strategy(model, strategy):
    """strategy.recompute (recompute_configs.checkpoints) and strategy.amp (amp_configs) on the model."""
    if strategy.recompute:
        ckpts = list(strategy.recompute_configs["checkpoints"])
        cfg = getattr(model, "config", None)
        if not ckpts and cfg is not None and hasattr(cfg, "recompute"):
            cfg.recompute = True  # model-native per-layer recompute (e.g. Llama / GPT decoder layers)
        else:
            from .recompute import recompute

            named = dict(model.named_sublayers())
            missing = [c for c in ckpts if c not in named]
            if missing:
                raise ValueError(f"recompute_configs.checkpoints: no sublayer named {missing}")
            for name in ckpts:
                layer = named[name]
                fwd = layer.forward

                def wrapped(*a, _fwd=fwd, **k):
                    return recompute(_fwd, *a, **k)

                layer.forward = wrapped
    if strategy.amp:
        model = _AmpModel(model, strategy.amp_configs)
    return model


class _AmpModel:
    """Runs the wrapped layer's forward under auto_cast with the strategy's amp_configs."""

    def __init__(self, layer, cfg):
        self._layer = layer
        self._cfg = cfg

    def __call__(self, *a, **k):
        from ...amp import auto_cast

        c = self._cfg
        pure = c["use_pure_fp16"] or c["use_pure_bf16"]
        with auto_cast(enable=True, custom_white_list=set(c["custom_white_list"]) or None,
                       custom_black_list=set(c["custom_black_list"]) or None, level="O2" if pure else "O1",
                       dtype="bfloat16" if c["use_pure_bf16"] else "float16"):
            return self._layer(*a, **k)

    forward = __call__

    def __getattr__(self, name):
        return getattr(self._layer, name)


def distributed_model(model):
    """Wrap by parallel mode (reference fleet/model.py:32-179), after applying the strategy's recompute /
    amp settings."""
    hcg = _hcg()
    mode = hcg.get_parallel_mode()
    strategy = _state["strategy"]
    model = _apply_model_strategy(model, strategy)
    if mode == ParallelMode.DATA_PARALLEL:
        from ..parallel import DataParallel

        if hcg.get_data_parallel_world_size() > 1:
            return DataParallel(model, group=hcg.get_data_parallel_group(),
                                find_unused_parameters=strategy.find_unused_parameters)
        return model
    if mode == ParallelMode.PIPELINE_PARALLEL:
        from .meta_parallel import pipeline_parallel as PPm

        mode_s = str(strategy.pipeline_configs.get("schedule_mode", "1F1B"))
        if getattr(model, "_num_virtual_pipeline_stages", 1) > 1:
            if mode_s == "FThenB":
                return PPm.PipelineParallelWithInterleaveFthenB(model, hcg, strategy)
            return PPm.PipelineParallelWithInterleave(model, hcg, strategy)
        cls = {"FThenB": PPm.PipelineParallelFThenB, "ZBH1": PPm.PipelineParallelZeroBubble,
               "ZB": PPm.PipelineParallelZeroBubble}.get(mode_s, PPm.PipelineParallel)
        return cls(model, hcg, strategy)
    if mode == ParallelMode.TENSOR_PARALLEL:
        from .meta_parallel.tensor_parallel import TensorParallel

        return TensorParallel(model, hcg, strategy)
    if mode == ParallelMode.SEGMENT_PARALLEL:
        from .meta_parallel.segment_parallel import SegmentParallel

        return SegmentParallel(model, hcg, strategy)
    from .meta_parallel.sharding_parallel import ShardingParallel

    return ShardingParallel(model, hcg, strategy)


def distributed_optimizer(optimizer, strategy=None):
    hcg = _hcg()
    if hcg.get_parallel_mode() == ParallelMode.DATA_PARALLEL and hcg.nranks == 1:
        return optimizer
    from .meta_optimizers import HybridParallelOptimizer

    return HybridParallelOptimizer(optimizer, hcg, strategy or _state["strategy"])


def distributed_scaler(scaler):
    return scaler


def _device_for_group(group):
    import torch

    if group is not None and group.backend == "nccl" and torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def collective_perf(comm_type, round=50, size_and_time=None):
    """Time collectives over the hybrid groups (reference fleet.py:621); see fleet/collective_perf.py."""
    from .collective_perf import collective_perf as _cp

    return _cp(comm_type, round, size_and_time)


def get_log_level_code():
    return 20


def set_log_level(level):
    pass


class _FleetUtil:
    @staticmethod
    def get_file_shard(files):
        r, n = C.get_rank(), C.get_world_size()
        return files[r::n]


util = _FleetUtil()


def __getattr__(name):
    import importlib

    if name in ("meta_parallel", "layers", "utils", "recompute", "meta_optimizers", "base", "launch", "elastic"):
        return importlib.import_module(f".{name}", __name__)
    raise AttributeError(name)
