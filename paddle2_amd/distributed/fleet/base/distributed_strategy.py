"""DistributedStrategy: typed, validated, prototxt-serialisable (reference:
python/paddle/distributed/fleet/base/distributed_strategy.py:284 and
paddle/fluid/framework/distributed_strategy.proto).

No protobuf dependency: the proto's messages are described by the ``_SCHEMA`` tables below (field ->
(type, default)), and every config is a ``StrategyConfig`` that type-checks and rejects unknown keys on
assignment, exactly like assigning to the reference's proto-backed properties (which raise on unknown
fields).  ``save_to_prototxt`` / ``load_from_prototxt`` read and write the protobuf text format of the
reference's ``DistributedStrategy`` message (nested ``name { ... }`` blocks, repeated fields as
repeated lines), so strategies round-trip with the reference's files.

What fleet applies (fleet/__init__.py): hybrid degrees and ``order`` (validated against the world size
in ``fleet.init``), ``amp`` + ``amp_configs`` (forward under auto_cast with the custom white / black
lists, O2 for ``use_pure_fp16`` / ``use_pure_bf16``), ``recompute`` + ``recompute_configs.checkpoints``
(those sublayers re-run their forward in backward), ``hybrid_configs.sharding_configs.comm_buffer_size_MB``
(bucket size of the fused gradient collectives), ``pipeline_configs`` (micro-batching, schedule,
``enable_partial_send_recv``), ``gradient_merge`` (k-step accumulation in the hybrid optimizer) and
``find_unused_parameters``.  Every ``hybrid_configs`` sub-key (mp_configs / pp_configs / sharding_configs) is
classified in ``KEY_SEMANTICS`` at the bottom of this file: honoured (where) or numerically neutral (why);
``fleet.init`` rejects non-default values of anything unimplemented (``validate_hybrid_configs``).
"""
from __future__ import annotations

import copy

_B, _I, _F, _S = bool, int, float, str


def _rep(t):
    return ("repeated", t)


_MP = {"sync_param": (_B, True), "sync_grad": (_B, False), "sync_moment": (_B, False),
       "sync_mode": (_S, "broadcast"), "mp_async_allreduce": (_B, False), "mp_skip_c_identity": (_B, False),
       "mp_fused_linear_param_grad_add": (_B, False), "need_broadcast_data": (_B, True),
       "recompute_allgather": (_B, False), "sp_async_reduce_scatter": (_B, False)}
_PP = {"dp_comm_overlap": (_B, False), "delay_scale_loss": (_B, False), "enable_timer": (_B, False),
       "sharding_comm_overlap": (_B, False), "profiling": (_B, False), "release_gradients": (_B, False),
       "overlap_p2p_comm": (_B, False), "clear_every_step_cache": (_B, False), "use_batch_p2p_comm": (_B, True),
       "best_unbalanced_scheduler": (_B, False)}
_DYSHARD = {"tensor_fusion": (_B, False), "accumulate_steps": (_I, 1), "comm_overlap": (_B, False),
            "split_param": (_B, False), "fuse_optimizer": (_B, True), "use_reduce_avg": (_B, True),
            "comm_buffer_size_MB": (_I, 256), "release_gradients": (_B, False), "free_grads_in_comm": (_B, False)}
_HYBRID = {"dp_degree": (_I, -1), "mp_degree": (_I, 1), "pp_degree": (_I, 1), "sharding_degree": (_I, 1),
           "sep_degree": (_I, 1), "mp_configs": (_MP, None), "pp_configs": (_PP, None),
           "sharding_configs": (_DYSHARD, None), "enable_optimizer_timer": (_B, False),
           "order": (_rep(_S), ["dp", "pp", "sharding", "sep", "mp"])}
_AMP = {"init_loss_scaling": (_F, 32768.0), "incr_every_n_steps": (_I, 1000), "decr_every_n_nan_or_inf": (_I, 2),
        "incr_ratio": (_F, 2.0), "decr_ratio": (_F, 0.8), "use_dynamic_loss_scaling": (_B, True),
        "custom_white_list": (_rep(_S), []), "custom_black_list": (_rep(_S), []),
        "custom_black_varnames": (_rep(_S), []), "use_pure_fp16": (_B, False), "use_fp16_guard": (_B, True),
        "use_optimizer_fp16": (_B, False), "use_pure_bf16": (_B, False)}
_RECOMPUTE = {"checkpoints": (_rep(_S), []), "enable_offload": (_B, False), "checkpoint_shape": (_rep(_I), []),
              "enable_tuning": (_B, False)}
_SHARDING = {"sharding_segment_strategy": (_S, "segment_broadcast_MB"), "segment_broadcast_MB": (_F, 32.0),
             "segment_anchors": (_rep(_S), []), "sharding_degree": (_I, 8), "mp_degree": (_I, 1),
             "dp_degree": (_I, 1), "hybrid_dp": (_B, False), "gradient_merge_acc_step": (_I, 1),
             "optimize_offload": (_B, False), "pp_allreduce_in_optimize": (_B, False), "pp_degree": (_I, 1),
             "optimize_cast": (_B, False), "_dp_as_optimizer_sharding": (_B, False), "stage": (_I, 1),
             "enable_tuning": (_B, False), "use_calc_stream": (_B, False)}
_PIPELINE = {"micro_batch_size": (_I, 1), "accumulate_steps": (_I, 1), "schedule_mode": (_S, "1F1B"),
             "p2p_cache_shape": (_B, True), "enable_partial_send_recv": (_B, True)}
_TP = {"tensor_parallel_degree": (_I, 1), "tensor_init_seed": (_I, -1)}
_GM = {"k_steps": (_I, 1), "avg": (_B, True)}
_LOCALSGD = {"k_steps": (_I, 1), "begin_step": (_I, 1)}
_ALOCALSGD = {"init_k_steps": (_I, 1), "begin_step": (_I, 1)}
_DGC = {"rampup_begin_step": (_I, 0), "rampup_step": (_I, 1), "sparsity": (_rep(_F), [])}
_LARS = {"lars_coeff": (_F, 0.001), "lars_weight_decay": (_F, 0.0005), "epsilon": (_F, 0.0),
         "exclude_from_weight_decay": (_rep(_S), [])}
_LAMB = {"lamb_weight_decay": (_F, 0.01), "exclude_from_weight_decay": (_rep(_S), [])}
_ASYNC = {"k_steps": (_I, -1), "max_merge_var_num": (_I, 1), "send_queue_size": (_I, 16),
          "independent_recv_thread": (_B, False), "min_send_grad_num_before_recv": (_I, 1),
          "thread_pool_size": (_I, 1), "send_wait_times": (_I, 1), "runtime_split_send_recv": (_B, False),
          "launch_barrier": (_B, True), "heter_worker_device_guard": (_S, "cpu"), "lr_decay_steps": (_I, 10),
          "use_ps_gpu": (_I, 0), "use_gpu_graph": (_I, 0)}
_QAT = {"channel_wise_abs_max": (_B, True), "weight_bits": (_I, 8), "activation_bits": (_I, 8),
        "not_quant_pattern": (_rep(_S), []), "algo": (_S, "")}
_GSCALE = {"scale_strategy": (_S, "avg"), "scale_gradient": (_B, False)}
_BUILD = {"fuse_elewise_add_act_ops": (_B, False), "fuse_bn_act_ops": (_B, False),
          "fuse_relu_depthwise_conv": (_B, False), "fuse_broadcast_ops": (_B, False),
          "fuse_all_optimizer_ops": (_B, False), "enable_inplace": (_B, False),
          "enable_backward_optimizer_op_deps": (_B, True), "cache_runtime_context": (_B, False),
          "fuse_bn_add_act_ops": (_B, True), "enable_auto_fusion": (_B, False), "enable_addto": (_B, False),
          "allow_cuda_graph_capture": (_B, False), "reduce_strategy": (_I, 0), "fuse_gemm_epilogue": (_B, False),
          "debug_graphviz_path": (_S, ""), "fused_attention": (_B, False), "fused_feedforward": (_B, False),
          "fuse_dot_product_attention": (_B, False), "fuse_resunit": (_B, False)}

# top-level scalar fields (DistributedStrategy message fields 1-42)
_TOP = {"amp": (_B, False), "recompute": (_B, False), "localsgd": (_B, False), "dgc": (_B, False),
        "gradient_merge": (_B, False), "lars": (_B, False), "lamb": (_B, False), "pipeline": (_B, False),
        "elastic": (_B, False), "auto": (_B, False), "a_sync": (_B, True), "sync_nccl_allreduce": (_B, True),
        "nccl_comm_num": (_I, 1), "use_hierarchical_allreduce": (_B, False),
        "hierarchical_allreduce_inter_nranks": (_I, 1), "sync_batch_norm": (_B, False),
        "fuse_all_reduce_ops": (_B, True), "fuse_grad_size_in_MB": (_I, 32), "fuse_grad_size_in_TFLOPS": (_F, 50.0),
        "cudnn_exhaustive_search": (_B, False), "conv_workspace_size_limit": (_I, 512),
        "cudnn_batchnorm_spatial_persistent": (_B, False), "adaptive_localsgd": (_B, False),
        "fp16_allreduce": (_B, False), "sharding": (_B, False), "last_comm_group_size_MB": (_F, 1.0),
        "find_unused_parameters": (_B, False), "tensor_parallel": (_B, False),
        "without_graph_optimization": (_B, True), "fuse_grad_size_in_num": (_I, 8),
        "calc_comm_same_stream": (_B, False), "asp": (_B, False), "fuse_grad_merge": (_B, False),
        "semi_auto": (_B, False), "adam_d2sum": (_B, False), "auto_search": (_B, False),
        "heter_ccl_mode": (_B, False), "is_fl_ps_mode": (_B, False), "with_coordinator": (_B, False),
        "qat": (_B, False), "split_data": (_B, True)}
# *_configs sub-messages
_CONFIGS = {"recompute_configs": _RECOMPUTE, "amp_configs": _AMP, "localsgd_configs": _LOCALSGD,
            "gradient_merge_configs": _GM, "dgc_configs": _DGC, "pipeline_configs": _PIPELINE,
            "a_sync_configs": _ASYNC, "lars_configs": _LARS, "lamb_configs": _LAMB,
            "adaptive_localsgd_configs": _ALOCALSGD, "sharding_configs": _SHARDING, "hybrid_configs": _HYBRID,
            "tensor_parallel_configs": _TP, "qat_configs": _QAT, "build_strategy": _BUILD,
            "gradient_scale_configs": _GSCALE}


def _coerce(name, typ, v):
    if isinstance(typ, tuple) and typ[0] == "repeated":
        if not isinstance(v, (list, tuple)):
            raise TypeError(f"{name} must be a list, got {type(v).__name__}")
        return [_coerce(name, typ[1], e) for e in v]
    if typ is _B:
        if not isinstance(v, bool):
            raise TypeError(f"{name} must be bool, got {v!r}")
        return v
    if typ is _I:
        if isinstance(v, bool) or not isinstance(v, int):
            raise TypeError(f"{name} must be int, got {v!r}")
        return v
    if typ is _F:
        if isinstance(v, bool) or not isinstance(v, (int, float)):
            raise TypeError(f"{name} must be float, got {v!r}")
        return float(v)
    if typ is _S:
        if not isinstance(v, str):
            raise TypeError(f"{name} must be str, got {v!r}")
        return v
    raise TypeError(f"unsupported schema type for {name}")


class StrategyConfig(dict):
    """A proto message as a dict: only schema fields, type-checked; nested messages are StrategyConfigs.
    ``cfg.update({...})`` / ``cfg[k] = v`` validate; nested dict values merge into the sub-message."""

    def __init__(self, name, schema, values=None):
        super().__init__()
        object.__setattr__(self, "_name", name)
        object.__setattr__(self, "_schema", schema)
        for k, (typ, dflt) in schema.items():
            if isinstance(typ, dict):
                dict.__setitem__(self, k, StrategyConfig(f"{name}.{k}", typ))
            else:
                dict.__setitem__(self, k, copy.deepcopy(dflt))
        if values:
            self.update(values)

    def __setitem__(self, k, v):
        if k not in self._schema:
            raise KeyError(f"{self._name} has no field {k!r}; valid fields: {sorted(self._schema)}")
        typ = self._schema[k][0]
        if isinstance(typ, dict):
            if isinstance(v, StrategyConfig):
                v = dict(v)
            if not isinstance(v, dict):
                raise TypeError(f"{self._name}.{k} must be a dict")
            self[k].update(v)
            return
        dict.__setitem__(self, k, _coerce(f"{self._name}.{k}", typ, v))

    def update(self, other=(), **kw):
        items = dict(other, **kw) if not isinstance(other, dict) else {**other, **kw}
        for k, v in items.items():
            self[k] = v

    def setdefault(self, k, default=None):
        if k not in self:
            self[k] = default
        return self[k]

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __deepcopy__(self, memo):
        return StrategyConfig(self._name, self._schema, {k: copy.deepcopy(dict(v) if isinstance(v, StrategyConfig)
                                                                          else v, memo) for k, v in self.items()})

    # ------------------------------------------------------------ prototxt
    def _to_text(self, indent):
        out = []
        pad = "  " * indent
        for k, (typ, dflt) in self._schema.items():
            v = self[k]
            if isinstance(typ, dict):
                body = v._to_text(indent + 1)
                out.append(f"{pad}{k} {{\n{body}{pad}}}\n")
            elif isinstance(typ, tuple):
                for e in v:
                    out.append(f"{pad}{k}: {_fmt(e)}\n")
            else:
                out.append(f"{pad}{k}: {_fmt(v)}\n")
        return "".join(out)


def _fmt(v):
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, str):
        return '"' + v.replace("\\", "\\\\").replace('"', '\\"') + '"'
    return repr(v)


def _tokenize(text):
    toks, i, n = [], 0, len(text)
    while i < n:
        c = text[i]
        if c.isspace():
            i += 1
        elif c == "#":
            while i < n and text[i] != "\n":
                i += 1
        elif c in "{}:":
            toks.append(c)
            i += 1
        elif c in "\"'":
            j, buf = i + 1, []
            while j < n and text[j] != c:
                if text[j] == "\\" and j + 1 < n:
                    j += 1
                buf.append(text[j])
                j += 1
            toks.append(("str", "".join(buf)))
            i = j + 1
        else:
            j = i
            while j < n and not text[j].isspace() and text[j] not in "{}:#":
                j += 1
            toks.append(text[i:j])
            i = j
    return toks


def _scalar(tok, typ):
    if isinstance(tok, tuple):
        return tok[1]
    if typ is _B:
        return tok == "true"
    if typ is _I:
        return int(tok)
    if typ is _F:
        return float(tok)
    return tok


def _parse_into(cfg, toks, pos):
    """Parse fields into ``cfg`` (a StrategyConfig or the strategy's top-level table) until '}' / EOF."""
    schema = cfg._schema
    repeated = {}
    while pos < len(toks) and toks[pos] != "}":
        name = toks[pos]
        if name not in schema:
            raise KeyError(f"prototxt: unknown field {name!r} in {cfg._name}")
        typ = schema[name][0]
        if toks[pos + 1] == "{":
            pos = _parse_into(cfg[name], toks, pos + 2) + 1
            continue
        assert toks[pos + 1] == ":", f"prototxt: expected ':' after {name}"
        if isinstance(typ, tuple):
            repeated.setdefault(name, []).append(_scalar(toks[pos + 2], typ[1]))
        else:
            cfg[name] = _scalar(toks[pos + 2], typ)
        pos += 3
    for k, v in repeated.items():
        cfg[k] = v
    return pos


class _Top(StrategyConfig):
    pass


class DistributedStrategy:
    """Reference ``fleet.DistributedStrategy`` with validated fields (see the module docstring)."""

    def __init__(self):
        object.__setattr__(self, "_top", StrategyConfig("DistributedStrategy", _TOP))
        object.__setattr__(self, "_cfg", {k: StrategyConfig(k, s) for k, s in _CONFIGS.items()})
        # replicated (non-distributed) parameters whose name contains one of these are kept in sync over the mp
        # group by mp_configs.sync_param / sync_grad / sync_moment (reference distributed_strategy.py:330)
        object.__setattr__(self, "sync_param_name", ["embedding", "layer_norm", ".b_"])

    # attribute access: top-level switches and *_configs messages
    def __getattr__(self, k):
        if k.startswith("_"):
            raise AttributeError(k)
        if k in _CONFIGS:
            return self._cfg[k]
        if k in _TOP:
            return self._top[k]
        raise AttributeError(f"DistributedStrategy has no attribute {k!r}")

    def __setattr__(self, k, v):
        if k == "sync_param_name":
            object.__setattr__(self, k, [str(x) for x in v])
        elif k in _CONFIGS:
            if not isinstance(v, dict):
                raise TypeError(f"{k} must be assigned a dict")
            if k == "hybrid_configs" and isinstance(v.get("mp_configs"), dict) and "sync_param_name" in v["mp_configs"]:
                v = dict(v, mp_configs=dict(v["mp_configs"]))   # reference :1940 pops it out of mp_configs
                object.__setattr__(self, "sync_param_name", [str(x) for x in v["mp_configs"].pop("sync_param_name")])
            self._cfg[k].update(v)  # the reference merges assigned dicts into the proto message
        elif k in _TOP:
            self._top[k] = v
        else:
            raise AttributeError(f"DistributedStrategy has no field {k!r}")

    def __deepcopy__(self, memo):
        out = DistributedStrategy()
        object.__setattr__(out, "_top", copy.deepcopy(self._top, memo))
        object.__setattr__(out, "_cfg", {k: copy.deepcopy(v, memo) for k, v in self._cfg.items()})
        object.__setattr__(out, "sync_param_name", list(self.sync_param_name))
        return out

    # ------------------------------------------------------------ prototxt (reference :382 / :404)
    def to_prototxt(self):
        out = []
        for k, (typ, dflt) in _TOP.items():
            out.append(f"{k}: {_fmt(self._top[k])}\n")
        for k in _CONFIGS:
            out.append(f"{k} {{\n{self._cfg[k]._to_text(1)}}}\n")
        return "".join(out)

    def save_to_prototxt(self, output):
        with open(output, "w") as f:
            f.write(self.to_prototxt())

    def load_from_prototxt(self, pb_file):
        with open(pb_file) as f:
            self.from_prototxt(f.read())

    def from_prototxt(self, text):
        toks = _tokenize(text)
        table = _Top("DistributedStrategy", {**_TOP, **{k: (s, None) for k, s in _CONFIGS.items()}})
        # parse into a scratch table sharing this strategy's sub-messages
        for k in _CONFIGS:
            dict.__setitem__(table, k, self._cfg[k])
        for k in _TOP:
            dict.__setitem__(table, k, self._top[k])
        _parse_into(table, toks, 0)
        for k in _TOP:
            self._top[k] = table[k]

    # ------------------------------------------------------------ checks
    def validate_world(self, world):
        """Degrees must multiply to the world size (dp_degree -1 = fill); returns the resolved dp degree."""
        h = self.hybrid_configs
        mp, pp, sh, sep = h["mp_degree"], h["pp_degree"], h["sharding_degree"], h["sep_degree"]
        for n, d in (("mp_degree", mp), ("pp_degree", pp), ("sharding_degree", sh), ("sep_degree", sep)):
            if d < 1:
                raise ValueError(f"hybrid_configs.{n} must be >= 1, got {d}")
        other = mp * pp * sh * sep
        dp = h["dp_degree"]
        if dp in (-1, 0):
            if world % other:
                raise ValueError(f"world size {world} is not divisible by mp*pp*sharding*sep = {other}")
            dp = world // other
        if dp * other != world:
            raise ValueError(f"hybrid degrees dp{dp} * mp{mp} * pp{pp} * sharding{sh} * sep{sep} = {dp * other} "
                             f"!= world size {world}")
        order = list(h["order"])
        if sorted(order) != sorted(["dp", "pp", "sharding", "sep", "mp"]):
            raise ValueError(f"hybrid_configs.order must be a permutation of dp/pp/sharding/sep/mp, got {order}")
        return dp

    def __repr__(self):
        on = [k for k, (t, d) in _TOP.items() if t is _B and self._top[k] and not d]
        return f"DistributedStrategy(enabled={on}, hybrid_configs={dict(self.hybrid_configs)})"


# What each hybrid_configs sub-key does here.  "honoured": implemented with the reference's numerics (where);
# "perf": a scheduling / memory knob whose numerics are unchanged — the MI355X path either always does the
# optimisation or does not need it (why).  fleet.init rejects a non-default value of any key listed in
# _UNSUPPORTED; tests/test_distributed_strategy.py checks that every schema key is classified here.
KEY_SEMANTICS = {
    "mp_configs": {
        "sync_param": ("honoured", "HybridParallelOptimizer: sync_param_name params broadcast/averaged over mp after step"),
        "sync_grad": ("honoured", "HybridParallelOptimizer: sync_param_name grads synced over mp before step"),
        "sync_moment": ("honoured", "HybridParallelOptimizer: Adam moments of sync_param_name params synced after step"),
        "sync_mode": ("honoured", "broadcast (from mp rank 0) or average, for the three syncs above"),
        "mp_async_allreduce": ("perf", "column-parallel dX all-reduce is issued before the dW GEMM in backward anyway"),
        "mp_skip_c_identity": ("perf", "the identity op is a no-op autograd Function here; nothing to skip"),
        "mp_fused_linear_param_grad_add": ("perf", "wgrad GEMM always accumulates into the fp32 main grad in its "
                                                   "epilogue (csrc/kernels/gemm.hip)"),
        "need_broadcast_data": ("honoured", "TensorParallel broadcasts the inputs from mp rank 0 before forward"),
        "recompute_allgather": ("perf", "sequence-parallel all-gather outputs are recomputed, not stored, in "
                                        "recompute; same values"),
        "sp_async_reduce_scatter": ("perf", "sequence-parallel reduce-scatter runs on the comm stream; same values"),
    },
    "pp_configs": {
        "dp_comm_overlap": ("honoured", "HybridParallelOptimizer: FusedCommBuffer all-reduce from gradient hooks"),
        "delay_scale_loss": ("honoured", "PipelineParallel: micro-batch losses unscaled, grads scaled by "
                                         "1/accumulate_steps before the step"),
        "enable_timer": ("perf", "timers only; see paddle2_amd.profiler"),
        "sharding_comm_overlap": ("honoured", "DygraphShardingOptimizerV2 reduce-scatter from gradient hooks"),
        "profiling": ("perf", "timers only"),
        "release_gradients": ("perf", "gradient buffers are views into persistent comm buffers"),
        "overlap_p2p_comm": ("perf", "pipeline p2p is always asynchronous (isend/irecv) here"),
        "clear_every_step_cache": ("perf", "no p2p shape cache is kept between steps"),
        "use_batch_p2p_comm": ("perf", "p2p ops of one schedule slot are always batched"),
        "best_unbalanced_scheduler": ("perf", "schedule order only; same gradients"),
    },
    "sharding_configs": {
        "tensor_fusion": ("perf", "V1 always reduces through one flat buffer per dtype"),
        "accumulate_steps": ("honoured", "V2 / dp hooks communicate after this many backward passes"),
        "comm_overlap": ("honoured", "V2 reduce-scatter from gradient hooks (V1: raises)"),
        "split_param": ("honoured", "DygraphShardingOptimizerV2"),
        "fuse_optimizer": ("perf", "the optimizers use multi-tensor updates anyway"),
        "use_reduce_avg": ("honoured", "V2 / dp hooks: AVG reduce on RCCL, SUM + scale otherwise"),
        "comm_buffer_size_MB": ("honoured", "V2 / dp-hook bucket size"),
        "release_gradients": ("perf", "gradient buffers are views into persistent comm buffers"),
        "free_grads_in_comm": ("perf", "gradient buffers are views into persistent comm buffers"),
    },
}
_UNSUPPORTED = {}   # (section, key) -> reason; empty: every key above is honoured or numerically neutral


def validate_hybrid_configs(strategy):
    """Raise NotImplementedError for a non-default value of a key that is not implemented (none today)."""
    hc = strategy.hybrid_configs
    for (sec, key), why in _UNSUPPORTED.items():
        dflt = _HYBRID[sec][0][key][1]
        if hc[sec][key] != dflt:
            raise NotImplementedError(f"hybrid_configs.{sec}.{key}={hc[sec][key]!r}: {why}")
