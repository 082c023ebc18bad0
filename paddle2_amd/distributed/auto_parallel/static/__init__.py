"""Static-graph auto-parallel engine: completion (SPMD-rule propagation over a recorded Program), partitioner
with reshard insertion (per-rank SPMD execution on the framework's reshard engine), MI355X cost model and a
placement planner (reference python/paddle/distributed/auto_parallel/static/)."""
from .completion import Completer, DistAttr, DistContext, attr_from_placements  # noqa: F401
from .cost_model import ClusterSpec, CostModel, Planner, reshard_steps  # noqa: F401
from .partitioner import DistributedProgram, parallelize_program  # noqa: F401
from .engine import Engine  # noqa: F401
from .resharder import DistMainProgram, Resharder, build_dist_main_program, comm_kinds  # noqa: F401,E402
from .passes import (allreduce_matmul_grad_overlap_pass, amp_pass, fuse_allreduce_pass, gradient_merge_pass,  # noqa: F401,E402
                     recompute_pass, sequence_parallel_optimization_pass, sharding_pass)
