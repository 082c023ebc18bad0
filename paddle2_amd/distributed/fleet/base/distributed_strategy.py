"""DistributedStrategy (reference: fleet/base/distributed_strategy.py:284, distributed_strategy.proto).

Protobuf-free: a plain attribute bag with the proto's field names and defaults
(``hybrid_configs`` with dp/mp/pp/sharding/sep degrees, ``MpConfig``/``PpConfig``/
``DygraphShardingConfig`` sub-dicts, amp/recompute/sharding/pipeline switches).
"""
from __future__ import annotations

import copy


_HYBRID_DEFAULT = {
    "dp_degree": -1, "mp_degree": 1, "pp_degree": 1, "sharding_degree": 1, "sep_degree": 1,
    "order": ["dp", "pp", "sharding", "sep", "mp"],
    "mp_configs": {"sync_param": False, "sync_grad": False, "sync_moment": False, "mp_async_allreduce": False,
                   "mp_skip_c_identity": False, "mp_fused_linear_param_grad_add": False,
                   "recompute_allgather": False, "sync_mode": "broadcast"},
    "pp_configs": {"dp_comm_overlap": False, "sharding_comm_overlap": False, "enable_timer": False,
                   "delay_scale_loss": False, "enable_dynamic_shape": False, "use_batch_p2p_comm": True,
                   "clear_every_step_cache": False, "use_dualpipev": False},
    "sharding_configs": {"tensor_fusion": False, "comm_overlap": False, "split_param": False,
                         "accumulate_steps": 1, "comm_buffer_size_MB": 256, "release_gradients": False},
}


class DistributedStrategy:
    def __init__(self):
        self._hybrid = copy.deepcopy(_HYBRID_DEFAULT)
        self.amp = False
        self.amp_configs = {"init_loss_scaling": 32768.0, "incr_every_n_steps": 1000, "decr_every_n_nan_or_inf": 2,
                            "incr_ratio": 2.0, "decr_ratio": 0.5, "use_dynamic_loss_scaling": True,
                            "custom_white_list": [], "custom_black_list": [], "use_pure_fp16": False,
                            "use_fp16_guard": True, "use_bf16": True}
        self.recompute = False
        self.recompute_configs = {"checkpoints": [], "enable_offload": False}
        self.pipeline = False
        self.pipeline_configs = {"micro_batch_size": 1, "accumulate_steps": 1, "schedule_mode": "1F1B"}
        self.tensor_parallel = False
        self.tensor_parallel_configs = {"tensor_parallel_degree": 1}
        self.sharding = False
        self.sharding_configs = {"sharding_degree": 8, "stage": 1, "segment_broadcast_MB": 32.0}
        self.gradient_merge = False
        self.gradient_merge_configs = {"k_steps": 1, "avg": True}
        self.lamb = False
        self.lars = False
        self.dgc = False
        self.localsgd = False
        self.fuse_all_reduce_ops = True
        self.fuse_grad_size_in_MB = 32
        self.find_unused_parameters = False
        self.without_graph_optimization = True
        self.heter_ccl_mode = False
        self.a_sync = False
        self.sync_nccl_allreduce = True
        self.nccl_comm_num = 1
        self.fuse_grad_merge = False

    @property
    def hybrid_configs(self):
        return self._hybrid

    @hybrid_configs.setter
    def hybrid_configs(self, cfg):
        for k, v in cfg.items():
            if isinstance(v, dict) and isinstance(self._hybrid.get(k), dict):
                self._hybrid[k].update(v)
            else:
                self._hybrid[k] = v

    def __repr__(self):
        return f"DistributedStrategy(hybrid_configs={self._hybrid})"
