"""paddle.distributed (reference: python/paddle/distributed/__init__.py, 65 public names)."""
from . import collective, watchdog  # noqa: F401
from .process_group import ProcessGroup, ProcessGroupGloo, ProcessGroupMPI, ProcessGroupNCCL  # noqa: F401
from .comm_context import CommContextManager, GlooCommContext, NCCLCommContext  # noqa: F401
from .collective import (Group, P2POp, ParallelEnv, ReduceOp, all_gather, all_gather_into_tensor,  # noqa: F401
                         all_gather_object, all_reduce, alltoall, alltoall_single, barrier, batch_isend_irecv,
                         broadcast, broadcast_object_list, destroy_process_group, gather, get_backend, get_group,
                         get_rank, get_world_size, init_parallel_env, irecv, is_available, is_initialized, isend,
                         new_group, partial_allgather, partial_recv, partial_send, recv, reduce, reduce_scatter,
                         scatter, scatter_object_list, send, stream, wait)
from .parallel import DataParallel, sync_params_buffers  # noqa: F401


def __getattr__(name):
    # heavy sub-packages load lazily
    import importlib

    if name in ("fleet", "launch", "checkpoint", "auto_parallel", "sharding", "spawn", "rpc", "utils", "elastic",
                "auto_tuner", "passes", "communication", "models"):
        mod = importlib.import_module(f".{name}", __name__)
        if name == "spawn":
            return mod.spawn
        return mod
    if name in ("shard_tensor", "reshard", "dtensor_from_fn", "shard_layer", "shard_optimizer", "ProcessMesh",
                "Shard", "Replicate", "Partial", "to_static", "unshard_dtensor", "shard_dataloader", "DistModel",
                "Strategy", "ShardingStage1", "ShardingStage2", "ShardingStage3", "dtensor_from_local",
                "shard_scaler", "set_mesh", "get_mesh", "Placement", "is_dist_tensor"):
        mod = importlib.import_module(".auto_parallel", __name__)
        return getattr(mod, name)
    if name in ("save_state_dict", "load_state_dict"):
        mod = importlib.import_module(".checkpoint", __name__)
        return getattr(mod, name)
    if name in ("group_sharded_parallel", "save_group_sharded_model"):
        mod = importlib.import_module(".sharding", __name__)
        return getattr(mod, name)
    raise AttributeError(name)
