"""paddle.distributed.auto_parallel (semi-automatic parallelism on DistTensors)."""
# load the reshard ENGINE module first: importing a submodule later would rebind the package attribute
# ``reshard`` (the API function below) to the module object
from . import reshard as _reshard_engine  # noqa: F401,E402
from .api import (DistModel, Partial, Placement, ProcessMesh, Replicate, Shard, ShardDataloader,  # noqa
                  ShardingStage1, ShardingStage2, ShardingStage3, Strategy, dtensor_from_fn, dtensor_from_local,
                  get_mesh, is_dist_tensor, local_tensor, placements_of, reshard, set_mesh, shard_dataloader,
                  shard_layer, shard_optimizer, shard_scaler, shard_tensor, to_static, unshard_dtensor)
from .spmd_rules import DistTensorSpec, TensorDistAttr, get_phi_spmd_rule, get_spmd_rule  # noqa: F401,E402
