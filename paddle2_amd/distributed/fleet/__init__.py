"""paddle.distributed.fleet (reference: fleet/fleet.py:218 init, :674 _init_hybrid_parallel_env,
fleet/model.py:32 distributed_model, fleet/optimizer.py:39 distributed_optimizer)."""
from __future__ import annotations

from ... import distributed as _dist  # noqa: F401
from .. import collective as C
from .base.distributed_strategy import DistributedStrategy  # noqa: F401
from .base.topology import CommunicateTopology, HybridCommunicateGroup, ParallelMode  # noqa: F401

_state = {"strategy": None, "hcg": None, "initialized": False, "is_collective": True}


class UserDefinedRoleMaker:
    def __init__(self, is_collective=True, **kw):
        self.is_collective = is_collective


class PaddleCloudRoleMaker(UserDefinedRoleMaker):
    pass


def init(role_maker=None, is_collective=True, strategy=None, log_level="INFO"):
    strategy = strategy or DistributedStrategy()
    _state["strategy"] = strategy
    C.init_parallel_env()
    world = C.get_world_size()
    hc = strategy.hybrid_configs
    mp, pp = int(hc.get("mp_degree", 1)), int(hc.get("pp_degree", 1))
    sh, sep = int(hc.get("sharding_degree", 1)), int(hc.get("sep_degree", 1))
    dp = int(hc.get("dp_degree", -1))
    if dp in (-1, 0):
        dp = max(1, world // (mp * pp * sh * sep))
    assert dp * mp * pp * sh * sep == world, f"degrees dp{dp}*mp{mp}*pp{pp}*sharding{sh}*sep{sep} != world {world}"
    hc["dp_degree"] = dp
    order = hc.get("order", ["dp", "pp", "sharding", "sep", "mp"])
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


def distributed_model(model):
    """Wrap by parallel mode (reference fleet/model.py:32-179)."""
    hcg = _hcg()
    mode = hcg.get_parallel_mode()
    strategy = _state["strategy"]
    if mode == ParallelMode.DATA_PARALLEL:
        from ..parallel import DataParallel

        if hcg.get_data_parallel_world_size() > 1:
            return DataParallel(model, group=hcg.get_data_parallel_group(),
                                find_unused_parameters=strategy.find_unused_parameters)
        return model
    if mode == ParallelMode.PIPELINE_PARALLEL:
        from .meta_parallel.pipeline_parallel import PipelineParallel, PipelineParallelWithInterleave

        acc = strategy.pipeline_configs.get("accumulate_steps", 1)
        if getattr(model, "_num_virtual_pipeline_stages", 1) > 1:
            return PipelineParallelWithInterleave(model, hcg, strategy)
        return PipelineParallel(model, hcg, strategy)
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
    from .meta_optimizers.hybrid_parallel_optimizer import HybridParallelOptimizer

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
