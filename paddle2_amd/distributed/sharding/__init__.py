"""paddle.distributed.sharding."""
from .group_sharded import (GroupShardedModel, GroupShardedOptimizer, group_sharded_parallel,  # noqa: F401
                            save_group_sharded_model)
