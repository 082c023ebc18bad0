"""Op schema over the reference's op inventory (reference: paddle/phi/ops/yaml/ops.yaml, fused_ops.yaml,
sparse_ops.yaml — the 600 op names the generated ``_C_ops`` exposes; phi/infermeta/ for InferMeta).

``reference_op_names.txt`` lists those names.  ``resolve(name)`` maps each to the implementation in this
framework — the same-named public function, or an entry of ``ALIASES`` for ops whose public API has a different
name (``bilinear_interp`` -> ``nn.functional.interpolate(mode="bilinear")``, ``p_norm`` -> ``norm``, the
``c_*`` collectives -> ``distributed``, detection ops -> ``vision.ops``, ...).  ``populate()`` registers every
resolvable op in the op table (ops/registry.py), so ``_C_ops.<name>``, ``kernel_info`` and ``op_schema``
answer for the whole inventory, and ``infer_meta(name, *args)`` gives output shapes / dtypes of any op outside
static capture by running it on meta tensors.
"""
from __future__ import annotations

import functools
import importlib
import inspect
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))

# reference op name -> (dotted path under paddle2_amd, fixed kwargs)
ALIASES = {
    # interpolation / pooling / conv variants
    "bilinear_interp": ("nn.functional.interpolate", {"mode": "bilinear"}),
    "bicubic_interp": ("nn.functional.interpolate", {"mode": "bicubic"}),
    "nearest_interp": ("nn.functional.interpolate", {"mode": "nearest"}),
    "linear_interp": ("nn.functional.interpolate", {"mode": "linear"}),
    "trilinear_interp": ("nn.functional.interpolate", {"mode": "trilinear"}),
    "pool2d": ("ops.op_schema._pool2d", {}),
    "pool3d": ("ops.op_schema._pool3d", {}),
    "max_pool2d_with_index": ("nn.functional.max_pool2d", {"return_mask": True}),
    "max_pool3d_with_index": ("nn.functional.max_pool3d", {"return_mask": True}),
    "depthwise_conv2d": ("nn.functional.conv2d", {}),
    "depthwise_conv2d_transpose": ("nn.functional.conv2d_transpose", {}),
    "conv2d_transpose_bias": ("nn.functional.conv2d_transpose", {}),
    "unpool": ("nn.functional.max_unpool2d", {}),
    "unpool3d": ("nn.functional.max_unpool3d", {}),
    "pad3d": ("nn.functional.pad", {}),
    "shuffle_channel": ("nn.functional.channel_shuffle", {}),
    "deformable_conv": ("vision.ops.deform_conv2d", {}),
    # norms / reductions
    "p_norm": ("linalg.norm", {}),
    "frobenius_norm": ("linalg.norm", {"p": "fro"}),
    "l1_norm": ("ops.op_schema._l1_norm", {}),
    "squared_l2_norm": ("ops.op_schema._squared_l2_norm", {}),
    "clip_by_norm": ("ops.op_schema._clip_by_norm", {}),
    "mean_all": ("mean", {}),
    "reduce_as": ("ops.op_schema._reduce_as", {}),
    # activations / losses
    "logsigmoid": ("nn.functional.log_sigmoid", {}),
    "tanh_shrink": ("nn.functional.tanhshrink", {}),
    "kldiv_loss": ("nn.functional.kl_div", {}),
    "bce_loss": ("nn.functional.binary_cross_entropy", {}),
    "sigmoid_cross_entropy_with_logits": ("nn.functional.binary_cross_entropy_with_logits", {"reduction": "none"}),
    "cross_entropy_with_softmax": ("nn.functional.softmax_with_cross_entropy", {}),
    "hinge_loss": ("ops.op_schema._hinge_loss", {}),
    "warpctc": ("nn.functional.ctc_loss", {}),
    "warprnnt": ("nn.functional.rnnt_loss", {}),
    "identity_loss": ("ops.op_schema._identity_loss", {}),
    # fft
    "fft_c2c": ("fft.fftn", {}),
    "fft_r2c": ("fft.rfftn", {}),
    "fft_c2r": ("fft.irfftn", {}),
    # attention / fusions
    "flash_attn": ("nn.functional.flash_attention", {}),
    "memory_efficient_attention": ("incubate.nn.memory_efficient_attention_op", {}),
    "fused_softmax_mask": ("incubate.softmax_mask_fuse", {}),
    "fused_softmax_mask_upper_triangle": ("incubate.softmax_mask_fuse_upper_triangle", {}),
    "fused_batch_norm_act": ("nn.functional.batch_norm", {}),
    "fused_bn_add_activation": ("nn.functional.batch_norm", {}),
    "sync_batch_norm_": ("nn.functional.batch_norm", {}),
    # creation / manipulation spellings
    "full_batch_size_like": ("ops.op_schema._full_batch_size_like", {}),
    "full_int_array": ("ops.op_schema._full_int_array", {}),
    "full_with_tensor": ("full", {}),
    "fill": ("full_like", {}),
    "reverse": ("flip", {}),
    "split_with_num": ("split", {}),
    "repeat_interleave_with_tensor_index": ("repeat_interleave", {}),
    "index_select_strided": ("index_select", {}),
    "view_shape": ("reshape", {}),
    "view_dtype": ("ops.op_schema._view_dtype", {}),
    "tensor_unfold": ("ops.op_schema._tensor_unfold", {}),
    "copy_to": ("ops.op_schema._copy_to", {}),
    "memcpy_d2h": ("ops.op_schema._memcpy_d2h", {}),
    "memcpy_h2d": ("ops.op_schema._memcpy_h2d", {}),
    "share_data": ("assign", {}),
    "depend": ("ops.op_schema._depend", {}),
    "data": ("static.data", {}),
    "uniform_inplace": ("ops.op_schema._uniform_inplace", {}),
    "gaussian_inplace": ("ops.op_schema._gaussian_inplace", {}),
    "exponential_": ("ops.op_schema._exponential_", {}),
    "truncated_gaussian_random": ("ops.op_schema._truncated_gaussian_random", {}),
    "uniform_random_batch_size_like": ("ops.op_schema._uniform_batch_size_like", {}),
    "affine_channel": ("ops.op_schema._affine_channel", {}),
    "segment_pool": ("ops.op_schema._segment_pool", {}),
    # collectives (static-graph op names of the communication API)
    "c_allreduce_sum": ("ops.op_schema._c_allreduce_sum", {}),
    "c_allreduce_max": ("ops.op_schema._c_allreduce_max", {}),
    "c_allreduce_min": ("ops.op_schema._c_allreduce_min", {}),
    "c_allreduce_prod": ("ops.op_schema._c_allreduce_prod", {}),
    "c_broadcast": ("distributed.broadcast", {}),
    "c_allgather": ("distributed.all_gather", {}),
    "c_reduce_sum": ("distributed.reduce", {}),
    "c_scatter": ("distributed.scatter", {}),
    "c_concat": ("distributed.fleet.layers.mpu.mp_ops._c_concat", {}),
    "c_identity": ("distributed.fleet.layers.mpu.mp_ops._c_identity", {}),
    "all_gather": ("distributed.all_gather", {}),
    "all_to_all": ("distributed.alltoall", {}),
    "broadcast": ("distributed.broadcast", {}),
    "reduce": ("distributed.reduce", {}),
    "reduce_scatter": ("distributed.reduce_scatter", {}),
    "c_sync_calc_stream": ("ops.op_schema._c_sync_calc_stream", {}),
    "c_sync_comm_stream": ("ops.op_schema._c_sync_comm_stream", {}),
    "sync_calc_stream": ("ops.op_schema._c_sync_calc_stream", {}),
    # detection / vision
    "yolo_box": ("vision.ops.yolo_box", {}),
    "yolo_loss": ("vision.ops.yolo_loss", {}),
    "prior_box": ("vision.ops.prior_box", {}),
    "box_coder": ("vision.ops.box_coder", {}),
    "roi_align": ("vision.ops.roi_align", {}),
    "roi_pool": ("vision.ops.roi_pool", {}),
    "psroi_pool": ("vision.ops.psroi_pool", {}),
    "nms": ("vision.ops.nms", {}),
    "matrix_nms": ("vision.ops.matrix_nms", {}),
    "generate_proposals": ("vision.ops.generate_proposals", {}),
    "distribute_fpn_proposals": ("vision.ops.distribute_fpn_proposals", {}),
    "read_file": ("vision.ops.read_file", {}),
    "decode_jpeg": ("vision.ops.decode_jpeg", {}),
    # quantization / weight-only
    "weight_only_linear": ("nn.quant.weight_only_linear", {}),
    "weight_quantize": ("nn.quant.weight_quantize", {}),
    "weight_dequantize": ("nn.quant.weight_dequantize", {}),
    "llm_int8_linear": ("nn.quant.llm_int8_linear", {}),
    # training-state ops
    "check_finite_and_unscale_": ("_C_ops.check_finite_and_unscale_", {}),
    "update_loss_scaling_": ("_C_ops.update_loss_scaling_", {}),
    "adamw_": ("_C_ops.adamw_", {}),
    "accuracy": ("metric.accuracy", {}),
    "viterbi_decode": ("text.viterbi_decode", {}),
    "merge_selected_rows": ("ops.op_schema._merge_selected_rows", {}),
    "check_numerics": ("ops.op_schema._check_numerics", {}),
    "enable_check_model_nan_inf": ("ops.op_schema._enable_nan_inf", {}),
    "disable_check_model_nan_inf": ("ops.op_schema._disable_nan_inf", {}),
    "sparse_attention": ("ops.op_schema._sparse_attention", {}),
    # optimizer update ops with the reference's argument order (functional, in place)
    "sgd_": ("ops.op_schema.sgd_", {}),
    "momentum_": ("ops.op_schema.momentum_", {}),
    "adam_": ("ops.op_schema.adam_", {}),
    "adamax_": ("ops.op_schema.adamax_", {}),
    "adagrad_": ("ops.op_schema.adagrad_", {}),
    "rmsprop_": ("ops.op_schema.rmsprop_", {}),
    "lamb_": ("ops.op_schema.lamb_", {}),
    # remaining spellings
    "fill_diagonal": ("ops.op_schema._fill_diagonal", {}),
    "fill_diagonal_tensor": ("ops.op_schema._fill_diagonal_tensor", {}),
    "matrix_rank_tol": ("linalg.matrix_rank", {}),
    "matrix_rank_atol_rtol": ("linalg.matrix_rank", {}),
    "spectral_norm": ("ops.op_schema._spectral_norm", {}),
    "set_value_with_tensor": ("ops.op_schema._set_value_with_tensor", {}),
    "assign_value_": ("ops.op_schema._assign_value_", {}),
    "assign_out_": ("ops.op_schema._assign_out_", {}),
    "gammaincc": ("ops.op_schema._gammaincc", {}),
    "dirichlet": ("ops.op_schema._dirichlet", {}),
    "npu_identity": ("ops.op_schema._depend", {}),
    "trans_layout": ("transpose", {}),
    "edit_distance": ("ops.op_schema._edit_distance", {}),
    "box_clip": ("ops.op_schema._box_clip", {}),
    "max_pool2d_v2": ("nn.functional.max_pool2d", {}),
    "fc": ("ops.op_schema._fc", {}),
    "gemm_epilogue": ("ops.op_schema._fc", {}),
    "skip_layernorm": ("ops.op_schema._skip_layernorm", {}),
    "fused_elementwise_add": ("add", {}),
    "fused_elementwise_sub": ("subtract", {}),
    "fused_elementwise_mul": ("multiply", {}),
    "fused_elementwise_div": ("divide", {}),
    "fused_bias_residual_layernorm": ("incubate.nn.functional.fused_layer_norm", {}),
    "fused_bias_dropout_residual_layer_norm": ("incubate.nn.functional.fused_bias_dropout_residual_layer_norm",
                                               {}),
    "fused_dot_product_attention": ("ops.op_schema._fused_dot_product_attention", {}),
    "sparse_values": ("ops.op_schema._sparse_values", {}),
    "sparse_indices": ("ops.op_schema._sparse_indices", {}),
    "sparse_to_sparse_coo": ("ops.op_schema._sparse_to_coo", {}),
    "sparse_to_sparse_csr": ("ops.op_schema._sparse_to_csr", {}),
    "sparse_scale": ("ops.op_schema._sparse_scale", {}),
    "sparse_divide_scalar": ("ops.op_schema._sparse_divide_scalar", {}),
    "sparse_maxpool": ("sparse.nn.functional.max_pool3d", {}),
    "fused_bias_dropout_residual_layer_norm": ("ops.op_schema._fused_bias_dropout_residual_layer_norm", {}),
    "adadelta_": ("ops.op_schema.adadelta_", {}),
    "merged_adam_": ("ops.op_schema.merged_adam_", {}),
    "merged_momentum_": ("ops.op_schema.merged_momentum_", {}),
    "fake_quantize_abs_max": ("ops.op_schema.fake_quantize_abs_max", {}),
    "fake_quantize_dequantize_abs_max": ("ops.op_schema.fake_quantize_dequantize_abs_max", {}),
    "fake_channel_wise_quantize_abs_max": ("ops.op_schema.fake_channel_wise_quantize_abs_max", {}),
    "fake_channel_wise_quantize_dequantize_abs_max": ("ops.op_schema.fake_channel_wise_quantize_dequantize_abs_max",
                                                      {}),
    "fake_dequantize_max_abs": ("ops.op_schema.fake_dequantize_max_abs", {}),
    "fake_channel_wise_dequantize_max_abs": ("ops.op_schema.fake_channel_wise_dequantize_max_abs", {}),
    "fake_quantize_moving_average_abs_max": ("ops.op_schema.fake_quantize_moving_average_abs_max", {}),
    "fake_quantize_dequantize_moving_average_abs_max": (
        "ops.op_schema.fake_quantize_dequantize_moving_average_abs_max", {}),
    "dequantize_abs_max": ("ops.op_schema.fake_dequantize_max_abs", {}),
    "dequantize_log": ("ops.op_schema.dequantize_log", {}),
    # dygraph / static-graph core spellings (inconsistent/*.yaml, legacy/static_ops.yaml)
    "all_reduce": ("distributed.all_reduce", {}),
    "barrier": ("distributed.barrier", {}),
    "c_allreduce_avg": ("ops.op_schema._c_allreduce_avg", {}),
    "c_reduce_avg": ("distributed.reduce", {}),
    "c_reduce_max": ("distributed.reduce", {}),
    "c_reduce_min": ("distributed.reduce", {}),
    "c_reduce_prod": ("distributed.reduce", {}),
    "c_softmax_with_cross_entropy": ("distributed.fleet.layers.mpu.mp_ops._c_softmax_with_cross_entropy", {}),
    "c_split": ("distributed.fleet.layers.mpu.mp_ops._c_split", {}),
    "p_send": ("distributed.send", {}),
    "p_recv": ("distributed.recv", {}),
    "send_v2": ("distributed.send", {}),
    "recv_v2": ("distributed.recv", {}),
    "global_gather": ("distributed.utils.global_gather", {}),
    "global_scatter": ("distributed.utils.global_scatter", {}),
    "lookup_table": ("nn.functional.embedding", {}),
    "elementwise_pow": ("pow", {}),
    "flatten2": ("flatten", {}),
    "cross_entropy2": ("nn.functional.cross_entropy", {}),
    "matmul_with_flatten": ("ops.op_schema._fc", {}),
    "legacy_matmul": ("matmul", {}),
    "legacy_reshape": ("reshape", {}),
    "legacy_expand": ("expand", {}),
    "legacy_crop": ("crop", {}),
    "legacy_bilinear_interp": ("nn.functional.interpolate", {"mode": "bilinear"}),
    "legacy_nearest_interp": ("nn.functional.interpolate", {"mode": "nearest"}),
    "legacy_generate_proposals": ("vision.ops.generate_proposals", {}),
    "topk_v1": ("topk", {}),
    "tril_triu": ("ops.op_schema._tril_triu", {}),
    "seed": ("seed", {}),
    "set_value": ("ops.op_schema._set_value_with_tensor", {}),
    "write_to_array": ("tensor.array_write", {}),
    "lod_array_length": ("tensor.array_length", {}),
    "lrn": ("nn.functional.local_response_norm", {}),
    "soft_relu": ("ops.op_schema._soft_relu", {}),
    "memcpy": ("ops.op_schema._copy_to", {}),
    "nop": ("ops.op_schema._depend", {}),
    "share_buffer": ("assign", {}),
    "share_data_": ("assign", {}),
    "quantize_linear": ("ops.op_schema.quantize_linear", {}),
    "dequantize_linear": ("ops.op_schema.dequantize_linear", {}),
    "fused_adam_": ("ops.op_schema.merged_adam_", {}),
    "fused_gemm_epilogue": ("ops.op_schema._fused_gemm_epilogue", {}),
    "get_tensor_from_selected_rows": ("ops.op_schema._selected_rows_value", {}),
    "save_combine": ("static.save", {}),
    "load_combine": ("static.load", {}),
    "print": ("static.Print", {}),
    "partial_send": ("distributed.partial_send", {}),
    "partial_recv": ("distributed.partial_recv", {}),
    "partial_allgather": ("distributed.partial_allgather", {}),
    "sync_comm_stream": ("device.synchronize", {}),
    "assign_value": ("assign", {}),
    "fused_attention": ("incubate.nn.functional.fused_multi_head_attention", {}),
}

# long-tail ops implemented in ops/extra_ops.py under their reference names
for _n in ("nadam_", "radam_", "asgd_", "rprop_", "decayed_adagrad", "ftrl", "dpsgd", "lars_momentum_",
           "average_accumulates_", "number_count", "assign_pos", "limit_by_capacity", "prune_gate_by_capacity",
           "random_routing", "partial_concat", "partial_sum", "shuffle_batch",
           "add_position_encoding", "cvm", "batch_fc", "accuracy_check", "coalesce_tensor", "coalesce_tensor_",
           "embedding_grad_dense", "straight_through_estimator_grad", "fused_elemwise_activation",
           "fused_elemwise_add_activation", "fused_fc_elementwise_layernorm", "fused_scale_bias_add_relu",
           "fused_embedding_eltwise_layernorm", "squeeze_excitation_block", "fp8_fp8_half_gemm_fused",
           "apply_per_channel_scale", "quant_linear", "fake_quantize_range_abs_max", "moving_average_abs_max_scale",
           "sparse_acos", "sparse_acosh", "sparse_full_like", "rnn", "lstm", "gru_unit", "beam_search",
           "beam_search_decode", "ctc_align", "crf_decoding", "chunk_eval", "auc", "bipartite_match",
           "anchor_generator", "multiclass_nms", "multiclass_nms3", "im2sequence", "correlation",
           "add_group_norm_silu", "fused_conv2d_add_act", "fusion_repeated_fc_relu", "fusion_squared_mat_sub",
           "fusion_transpose_flatten_concat", "multihead_matmul", "self_dp_attention", "fused_gate_attention",
           "cudnn_lstm", "resnet_basic_block", "resnet_unit", "blha_get_max_len", "calc_reduced_attn_scores",
           "sparse_batch_norm_", "sparse_sync_batch_norm_", "yolo_box_head", "dgc_clip_by_norm", "dgc_momentum",
           "dgc", "collect_fpn_proposals", "fusion_seqpool_concat", "fused_seqpool_cvm", "fusion_seqpool_cvm_concat",
           "dist_concat", "fused_token_prune", "graph_khop_sampler", "tdm_child", "lookup_table_dequant", "gru",
           "fusion_gru", "fusion_lstm", "rank_attention", "qkv_unpack_mha", "match_matrix_tensor",
           "fusion_seqconv_eltadd_relu", "fusion_seqexpand_concat_fc", "fused_embedding_fc_lstm", "attention_lstm",
           "yolo_box_post", "p_send_array", "p_recv_array", "fused_scale_bias_relu_conv_bn",
           "fused_multi_transformer_int8", "tdm_sampler", "detection_map", "faster_tokenizer", "fusion_group",
           "pyramid_hash", "distributed_fused_lamb_init", "fused_dconv_drelu_dbn"):
    ALIASES.setdefault(_n, ("ops.extra_ops." + _n, {}))
ALIASES.setdefault("nce", ("static.nn.nce", {}))
ALIASES.setdefault("row_conv", ("static.nn.row_conv", {}))
ALIASES.setdefault("graph_sample_neighbors", ("geometric.sample_neighbors", {}))
ALIASES["print"] = ("ops.extra_ops.print_op", {})
ALIASES.setdefault("hash", ("ops.extra_ops.hash_op", {}))
for _n in ("sequence_pool", "sequence_softmax", "sequence_expand", "sequence_conv", "lod_reset"):
    ALIASES.setdefault(_n, ("static.sequence." + _n, {}))
ALIASES.setdefault("sparse_conv3d_implicit_gemm", ("sparse.nn.functional.conv3d", {}))
ALIASES.setdefault("sparse_fused_attention", ("sparse.nn.functional.attention", {}))

# reference ops that only exist for other hardware (XPU fused kernels): outside this framework's scope
_PS_OPS = {"distributed_lookup_table", "distributed_push_sparse", "send_and_recv", "fetch_barrier",
           "sparse_momentum", "pull_box_sparse", "pull_gpups_sparse", "pull_sparse_v2", "push_dense", "push_sparse_v2",
           "onednn_to_paddle_layout", "transfer_layout", "shadow_feed", "shadow_feed_tensors", "shadow_output",
           "comm_init_all", "feed"}


def _out_of_scope(name):
    """XPU-only fused kernels, parameter-server / oneDNN plumbing (SURVEY [OUT])."""
    return name.endswith("_xpu") or name in _PS_OPS


# ------------------------------------------------------------------------------ small adapters
def _raw(x):
    return x._t if hasattr(x, "_t") else x


def _wrap(t):
    from ..framework.tensor import Tensor

    return Tensor._wrap(t)


def _pool2d(x, kernel_size, strides=None, paddings=0, ceil_mode=False, exclusive=True, data_format="NCHW",
            pooling_type="max", global_pooling=False, adaptive=False, padding_algorithm="EXPLICIT"):
    from ..nn import functional as F

    if global_pooling:
        return (F.adaptive_max_pool2d if pooling_type == "max" else F.adaptive_avg_pool2d)(x, 1)
    if adaptive:
        return (F.adaptive_max_pool2d if pooling_type == "max" else F.adaptive_avg_pool2d)(x, kernel_size)
    if pooling_type == "max":
        return F.max_pool2d(x, kernel_size, strides, paddings, ceil_mode=ceil_mode, data_format=data_format)
    return F.avg_pool2d(x, kernel_size, strides, paddings, ceil_mode=ceil_mode, exclusive=exclusive,
                        data_format=data_format)


def _pool3d(x, kernel_size, strides=None, paddings=0, ceil_mode=False, exclusive=True, data_format="NCDHW",
            pooling_type="max", global_pooling=False, adaptive=False, padding_algorithm="EXPLICIT"):
    from ..nn import functional as F

    if global_pooling:
        return (F.adaptive_max_pool3d if pooling_type == "max" else F.adaptive_avg_pool3d)(x, 1)
    if adaptive:
        return (F.adaptive_max_pool3d if pooling_type == "max" else F.adaptive_avg_pool3d)(x, kernel_size)
    if pooling_type == "max":
        return F.max_pool3d(x, kernel_size, strides, paddings, ceil_mode=ceil_mode, data_format=data_format)
    return F.avg_pool3d(x, kernel_size, strides, paddings, ceil_mode=ceil_mode, exclusive=exclusive,
                        data_format=data_format)


def _c_sync_calc_stream(x=None):
    """c_sync_calc_stream: the host waits for the CALCULATION stream of the tensor's device only (not the
    whole device: comm / copy streams keep running)."""
    import torch

    t = _raw(x) if x is not None else None
    if torch.cuda.is_available():
        dev = t.device if isinstance(t, torch.Tensor) and t.is_cuda else torch.cuda.current_device()
        torch.cuda.current_stream(dev).synchronize()
    return x


def _c_sync_comm_stream(x=None, ring_id=0):
    """c_sync_comm_stream: the host waits for the device's COMMUNICATION stream (GPUContext.comm_stream)."""
    import torch

    t = _raw(x) if x is not None else None
    if torch.cuda.is_available():
        from ..device.context import get_context

        dev = t.device.index if isinstance(t, torch.Tensor) and t.is_cuda else torch.cuda.current_device()
        get_context(dev).comm_stream().synchronize()
    return x


def _l1_norm(x):
    return _wrap(_raw(x).abs().sum())


def _squared_l2_norm(x):
    return _wrap(_raw(x).float().pow(2).sum().reshape([1]))


def _clip_by_norm(x, max_norm):
    t = _raw(x)
    n = t.float().norm()
    return _wrap(torch.where(n > max_norm, t * (max_norm / n), t))


def _reduce_as(x, target):
    t, ref = _raw(x), _raw(target)
    lead = t.dim() - ref.dim()
    dims = list(range(lead)) + [i + lead for i, s in enumerate(ref.shape) if s == 1 and t.shape[i + lead] != 1]
    out = t.sum(dims, keepdim=True) if dims else t
    return _wrap(out.reshape(ref.shape))


def _hinge_loss(logits, labels):
    lg, lb = _raw(logits), _raw(labels)
    return _wrap(torch.clamp(1 - lg * (2 * lb - 1), min=0))


def _identity_loss(x, reduction=1):
    t = _raw(x)
    return _wrap(t.sum() if reduction == 0 else (t.mean() if reduction == 1 else t))


def _full_batch_size_like(input, shape, dtype="float32", value=0.0, input_dim_idx=0, output_dim_idx=0):
    from .. import full

    shape = list(shape)
    shape[output_dim_idx] = _raw(input).shape[input_dim_idx]
    return full(shape, value, dtype)


def _uniform_batch_size_like(input, shape, dtype="float32", input_dim_idx=0, output_dim_idx=0, min=-1.0, max=1.0,
                             seed=0):
    from .. import uniform

    shape = list(shape)
    shape[output_dim_idx] = _raw(input).shape[input_dim_idx]
    return uniform(shape, dtype, min, max)


def _full_int_array(value, dtype="int64"):
    from .. import to_tensor

    return to_tensor(list(value), dtype=dtype)


def _view_dtype(x, dtype):
    from ..framework.dtype import to_torch_dtype

    return _wrap(_raw(x).view(to_torch_dtype(dtype)))


def _tensor_unfold(x, axis, size, step):
    return _wrap(_raw(x).unfold(axis, size, step))


def _copy_to(x, place, blocking=True):
    from ..framework.place import _parse_device

    return _wrap(_raw(x).to(_parse_device(place), non_blocking=not blocking))


def _memcpy_d2h(x, dst_place_type=0):
    return _wrap(_raw(x).cpu())


def _memcpy_h2d(x, dst_place_type=1):
    return _wrap(_raw(x).cuda() if torch.cuda.is_available() else _raw(x))


def _depend(x, dep=None):
    return x


def _uniform_inplace(x, min=-1.0, max=1.0, seed=0, diag_num=0, diag_step=0, diag_val=1.0):
    _raw(x).uniform_(min, max)
    return x


def _gaussian_inplace(x, mean=0.0, std=1.0, seed=0):
    _raw(x).normal_(mean, std)
    return x


def _exponential_(x, lam=1.0):
    _raw(x).exponential_(lam)
    return x


def _truncated_gaussian_random(shape, mean=0.0, std=1.0, seed=0, a=-2.0, b=2.0, dtype="float32"):
    from ..framework.dtype import to_torch_dtype

    t = torch.empty(list(shape), dtype=to_torch_dtype(dtype))
    torch.nn.init.trunc_normal_(t, mean, std, mean + a * std, mean + b * std)
    return _wrap(t)


def _affine_channel(x, scale, bias, data_layout="NCHW"):
    t = _raw(x)
    shape = [1, -1] + [1] * (t.dim() - 2) if data_layout == "NCHW" else [1] * (t.dim() - 1) + [-1]
    return _wrap(t * _raw(scale).view(shape) + _raw(bias).view(shape))


def _segment_pool(x, segment_ids, pooltype="SUM"):
    from .. import geometric

    fn = {"SUM": geometric.segment_sum, "MEAN": geometric.segment_mean, "MAX": geometric.segment_max,
          "MIN": geometric.segment_min}[pooltype.upper()]
    return fn(x, segment_ids)


def _c_allreduce(op):
    def f(x, ring_id=0, use_calc_stream=False, use_model_parallel=False):
        from .. import distributed as dist

        dist.all_reduce(x, op=op)
        return x

    return f


def _c_allreduce_sum(x, ring_id=0, use_calc_stream=False, use_model_parallel=False):
    from ..distributed import ReduceOp

    return _c_allreduce(ReduceOp.SUM)(x)


def _c_allreduce_max(x, ring_id=0, use_calc_stream=False, use_model_parallel=False):
    from ..distributed import ReduceOp

    return _c_allreduce(ReduceOp.MAX)(x)


def _c_allreduce_min(x, ring_id=0, use_calc_stream=False, use_model_parallel=False):
    from ..distributed import ReduceOp

    return _c_allreduce(ReduceOp.MIN)(x)


def _c_allreduce_prod(x, ring_id=0, use_calc_stream=False, use_model_parallel=False):
    from ..distributed import ReduceOp

    return _c_allreduce(ReduceOp.PROD)(x)


def _merge_selected_rows(x):
    from ..framework.tensor_types import SelectedRows

    return x.merge_add() if isinstance(x, SelectedRows) else x


def _check_numerics(tensor, op_type="", var_name="", check_nan_inf_level=0, stack_height_limit=-1,
                    output_dir=""):
    t = _raw(tensor)
    stats = torch.stack([torch.isnan(t).sum(), torch.isinf(t).sum(), (t == 0).sum()]).to(torch.int64)
    vals = torch.stack([t.float().amax(), t.float().amin(), t.float().mean()]) if t.numel() else torch.zeros(3)
    return _wrap(stats), _wrap(vals)


def _enable_nan_inf(flag=1):
    from ..framework import flags

    flags.set_flags({"FLAGS_check_nan_inf": True})


def _disable_nan_inf(flag=0):
    from ..framework import flags

    flags.set_flags({"FLAGS_check_nan_inf": False})


def _sparse_attention(q, k, v, offset, columns, key_padding_mask=None, attn_mask=None):
    """Block-sparse attention over a CSR pattern (offset [B, H, S+1], columns [B, H, nnz]) -> [B, H, S, D]."""
    qt, kt, vt = _raw(q), _raw(k), _raw(v)
    off, col = _raw(offset).long(), _raw(columns).long()
    B, H, S, D = qt.shape
    mask = torch.zeros(B, H, S, S, dtype=torch.bool, device=qt.device)
    rows = torch.repeat_interleave(torch.arange(S, device=qt.device).expand(B, H, S).reshape(-1),
                                   (off[..., 1:] - off[..., :-1]).reshape(-1))
    bh = torch.repeat_interleave(torch.arange(B * H, device=qt.device), (off[..., -1] - off[..., 0]).reshape(-1))
    cols = torch.cat([col[b, h, :off[b, h, -1]] for b in range(B) for h in range(H)])
    mask.view(B * H, S, S)[bh, rows, cols] = True
    s = qt @ kt.transpose(-1, -2) / D ** 0.5
    s = s.masked_fill(~mask, float("-inf"))
    if key_padding_mask is not None:
        s = s + _raw(key_padding_mask).view(B, 1, 1, S)
    if attn_mask is not None:
        s = s + _raw(attn_mask).view(1, 1, S, S)
    p = torch.softmax(s, -1).nan_to_num(0.0)
    return _wrap(p @ vt)


# ------------------------------------------------------------------------------ optimizer ops (reference args)
def _lr(v):
    t = _raw(v)
    return t.reshape(-1)[0] if isinstance(t, torch.Tensor) else float(t)


def _upd(dst, val):
    """Write ``val`` into the framework tensor / torch tensor ``dst`` in place; returns dst."""
    if dst is None:
        return None
    _raw(dst).copy_(val.to(_raw(dst).dtype))
    return dst


@torch.no_grad()
def sgd_(param, learning_rate, grad, master_param=None, multi_precision=False):
    tgt = _raw(master_param) if (multi_precision and master_param is not None) else _raw(param)
    new = tgt.float() - _lr(learning_rate) * _raw(grad).float()
    _upd(master_param if (multi_precision and master_param is not None) else param, new)
    if multi_precision and master_param is not None:
        _upd(param, new)
    return param, master_param


@torch.no_grad()
def momentum_(param, grad, velocity, learning_rate, master_param=None, mu=0.9, use_nesterov=False,
              regularization_method="", regularization_coeff=0.0, multi_precision=False, rescale_grad=1.0):
    p = _raw(master_param if (multi_precision and master_param is not None) else param).float()
    g = _raw(grad).float() * rescale_grad
    if regularization_method == "l2_decay":
        g = g + regularization_coeff * p
    v = _raw(velocity).float() * mu + g
    lr = _lr(learning_rate)
    new = p - lr * (g + mu * v) if use_nesterov else p - lr * v
    _upd(velocity, v)
    _upd(param, new)
    if master_param is not None and multi_precision:
        _upd(master_param, new)
    return param, velocity, master_param


@torch.no_grad()
def adam_(param, grad, learning_rate, moment1, moment2, beta1_pow, beta2_pow, master_param=None, skip_update=None,
          beta1=0.9, beta2=0.999, epsilon=1e-8, lazy_mode=False, min_row_size_to_use_multithread=1000,
          multi_precision=False, use_global_beta_pow=False):
    if skip_update is not None and bool(_raw(skip_update).reshape(-1)[0]):
        return param, moment1, moment2, beta1_pow, beta2_pow, master_param
    p = _raw(master_param if (multi_precision and master_param is not None) else param).float()
    g = _raw(grad).float()
    m1 = _raw(moment1).float() * beta1 + (1 - beta1) * g
    m2 = _raw(moment2).float() * beta2 + (1 - beta2) * g * g
    b1p, b2p = _raw(beta1_pow).float(), _raw(beta2_pow).float()
    lr = _lr(learning_rate) * torch.sqrt(1 - b2p) / (1 - b1p)
    new = p - lr * (m1 / (torch.sqrt(m2) + epsilon * torch.sqrt(1 - b2p)))
    _upd(moment1, m1)
    _upd(moment2, m2)
    _upd(param, new)
    if master_param is not None and multi_precision:
        _upd(master_param, new)
    if not use_global_beta_pow:
        _upd(beta1_pow, b1p * beta1)
        _upd(beta2_pow, b2p * beta2)
    return param, moment1, moment2, beta1_pow, beta2_pow, master_param


@torch.no_grad()
def adamax_(param, grad, learning_rate, moment, inf_norm, beta1_pow, master_param=None, beta1=0.9, beta2=0.999,
            epsilon=1e-8, multi_precision=False):
    p = _raw(master_param if (multi_precision and master_param is not None) else param).float()
    g = _raw(grad).float()
    m = _raw(moment).float() * beta1 + (1 - beta1) * g
    u = torch.maximum(_raw(inf_norm).float() * beta2 + epsilon, g.abs())
    lr = _lr(learning_rate) / (1 - _raw(beta1_pow).float())
    new = p - lr * m / u
    _upd(moment, m)
    _upd(inf_norm, u)
    _upd(param, new)
    if master_param is not None and multi_precision:
        _upd(master_param, new)
    return param, moment, inf_norm, master_param


@torch.no_grad()
def adagrad_(param, grad, moment, learning_rate, master_param=None, epsilon=1e-6, multi_precision=False):
    p = _raw(master_param if (multi_precision and master_param is not None) else param).float()
    g = _raw(grad).float()
    m = _raw(moment).float() + g * g
    new = p - _lr(learning_rate) * g / (torch.sqrt(m) + epsilon)
    _upd(moment, m)
    _upd(param, new)
    if master_param is not None and multi_precision:
        _upd(master_param, new)
    return param, moment, master_param


@torch.no_grad()
def rmsprop_(param, mean_square, grad, moment, learning_rate, mean_grad=None, master_param=None, epsilon=1e-10,
             decay=0.9, momentum=0.0, centered=False, multi_precision=False):
    p = _raw(master_param if (multi_precision and master_param is not None) else param).float()
    g = _raw(grad).float()
    ms = _raw(mean_square).float() * decay + (1 - decay) * g * g
    if centered:
        mg = _raw(mean_grad).float() * decay + (1 - decay) * g
        denom = ms - mg * mg + epsilon
        _upd(mean_grad, mg)
    else:
        denom = ms + epsilon
    mom = _raw(moment).float() * momentum + _lr(learning_rate) * g / torch.sqrt(denom)
    new = p - mom
    _upd(mean_square, ms)
    _upd(moment, mom)
    _upd(param, new)
    if master_param is not None and multi_precision:
        _upd(master_param, new)
    return param, moment, mean_square, mean_grad, master_param


@torch.no_grad()
def lamb_(param, grad, learning_rate, moment1, moment2, beta1_pow, beta2_pow, master_param=None, skip_update=None,
          weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6, always_adapt=False, multi_precision=False):
    if skip_update is not None and bool(_raw(skip_update).reshape(-1)[0]):
        return param, moment1, moment2, beta1_pow, beta2_pow, master_param
    p = _raw(master_param if (multi_precision and master_param is not None) else param).float()
    g = _raw(grad).float()
    m1 = _raw(moment1).float() * beta1 + (1 - beta1) * g
    m2 = _raw(moment2).float() * beta2 + (1 - beta2) * g * g
    b1p, b2p = _raw(beta1_pow).float() * beta1, _raw(beta2_pow).float() * beta2
    r = (m1 / (1 - b1p)) / (torch.sqrt(m2 / (1 - b2p)) + epsilon) + weight_decay * p
    pn, rn = p.norm(), r.norm()
    trust = torch.where((pn > 0) & (rn > 0), pn / rn, torch.ones_like(pn)) if (weight_decay > 0 or always_adapt) \
        else torch.ones_like(pn)
    new = p - _lr(learning_rate) * trust * r
    _upd(moment1, m1)
    _upd(moment2, m2)
    _upd(beta1_pow, b1p)
    _upd(beta2_pow, b2p)
    _upd(param, new)
    if master_param is not None and multi_precision:
        _upd(master_param, new)
    return param, moment1, moment2, beta1_pow, beta2_pow, master_param


# ------------------------------------------------------------------------------ more adapters
def _fill_diagonal(x, value=0.0, offset=0, wrap=False):
    t = _raw(x).clone()
    from .. import Tensor

    y = Tensor._wrap(t)
    return y.fill_diagonal_(value, offset, wrap)


def _fill_diagonal_tensor(x, y, offset=0, dim1=0, dim2=1):
    t = _raw(x).clone()
    d = torch.diagonal(t, offset, dim1, dim2)
    d.copy_(_raw(y).expand_as(d))
    return _wrap(t)


def _spectral_norm(weight, u, v, dim=0, power_iters=1, eps=1e-12):
    w = _raw(weight)
    perm = [dim] + [i for i in range(w.dim()) if i != dim]
    mat = w.permute(perm).reshape(w.shape[dim], -1)
    uu, vv = _raw(u).clone(), _raw(v).clone()
    for _ in range(power_iters):
        vv = torch.nn.functional.normalize(mat.t() @ uu, dim=0, eps=eps)
        uu = torch.nn.functional.normalize(mat @ vv, dim=0, eps=eps)
    sigma = uu @ mat @ vv
    return _wrap(w / sigma)


def _set_value_with_tensor(x, values, starts, ends, steps, axes, decrease_axes=None, none_axes=None):
    t = _raw(x).clone()
    idx = [slice(None)] * t.dim()
    for a, s0, e0, st in zip(axes, starts, ends, steps):
        idx[a] = slice(int(s0), int(e0), int(st))
    t[tuple(idx)] = _raw(values)
    return _wrap(t)


def _assign_value_(output, shape, dtype, values, place=None):
    t = _raw(output)
    t.copy_(torch.as_tensor(values, dtype=t.dtype).reshape(list(shape)))
    return output


def _assign_out_(x, output):
    _raw(output).copy_(_raw(x))
    return output


def _gammaincc(x, y):
    return _wrap(torch.special.gammaincc(_raw(x), _raw(y)))


def _dirichlet(alpha):
    a = _raw(alpha)
    g = torch._standard_gamma(a)
    return _wrap(g / g.sum(-1, keepdim=True))


def _edit_distance(hyps, refs, hypslength=None, refslength=None, normalized=False):
    """Levenshtein distance per sequence pair -> (sequence count, distances [B, 1])."""
    H, R = _raw(hyps), _raw(refs)
    hl = _raw(hypslength).reshape(-1).tolist() if hypslength is not None else [H.shape[1]] * H.shape[0]
    rl = _raw(refslength).reshape(-1).tolist() if refslength is not None else [R.shape[1]] * R.shape[0]
    out = []
    for b in range(H.shape[0]):
        h, r = H[b, :int(hl[b])].tolist(), R[b, :int(rl[b])].tolist()
        prev = list(range(len(r) + 1))
        for i, hv in enumerate(h, 1):
            cur = [i] + [0] * len(r)
            for j, rv in enumerate(r, 1):
                cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (hv != rv))
            prev = cur
        d = float(prev[-1])
        out.append(d / max(len(r), 1) if normalized else d)
    return (_wrap(torch.tensor([H.shape[0]], dtype=torch.int64)),
            _wrap(torch.tensor(out, dtype=torch.float32).view(-1, 1)))


def _box_clip(input, im_info):
    b, info = _raw(input), _raw(im_info)
    h = torch.round(info[:, 0] / info[:, 2]) - 1
    w = torch.round(info[:, 1] / info[:, 2]) - 1
    shape = [-1] + [1] * (b.dim() - 2)
    h, w = h.view(shape), w.view(shape)
    out = torch.stack([b[..., 0].clamp(min=0).minimum(w), b[..., 1].clamp(min=0).minimum(h),
                       b[..., 2].clamp(min=0).minimum(w), b[..., 3].clamp(min=0).minimum(h)], -1)
    return _wrap(out)


def _fc(input, w, bias=None, in_num_col_dims=1, activation_type="", padding_weights=False):
    x = _raw(input)
    x2 = x.reshape(int(torch.tensor(x.shape[:in_num_col_dims]).prod()), -1)
    y = x2 @ _raw(w)
    if bias is not None:
        y = y + _raw(bias)
    if activation_type == "relu":
        y = torch.relu(y)
    elif activation_type == "gelu":
        y = torch.nn.functional.gelu(y)
    return _wrap(y.reshape(list(x.shape[:in_num_col_dims]) + [y.shape[-1]]))


def _skip_layernorm(x, y, scale, bias, epsilon=1e-5, begin_norm_axis=-1):
    s = _raw(x) + _raw(y)
    n = s.shape[-1]
    return _wrap(torch.nn.functional.layer_norm(s, (n,), _raw(scale), _raw(bias), epsilon))


def _fused_dot_product_attention(q, k, v, bias=None, cu_seqlen_q=None, cu_seqlen_kv=None, scaling_factor=None,
                                 dropout_probability=0.0, is_training=False, mask_type_str="none",
                                 bias_type_str="none"):
    from ..nn import functional as F

    out = F.scaled_dot_product_attention(q, k, v, attn_mask=bias, dropout_p=dropout_probability,
                                         is_causal=mask_type_str == "causal", training=is_training)
    return out


def _sparse_values(x):
    t = _raw(x)
    return _wrap(t.values() if t.layout in (torch.sparse_coo, torch.sparse_csr) else t)


def _sparse_indices(x):
    t = _raw(x)
    return _wrap(t.coalesce().indices() if t.layout == torch.sparse_coo else t.to_sparse().indices())


def _sparse_to_coo(x, sparse_dim=None):
    t = _raw(x)
    return _wrap(t.to_sparse(sparse_dim) if sparse_dim else t.to_sparse())


def _sparse_to_csr(x):
    return _wrap(_raw(x).to_sparse_csr())


def _sparse_scale(x, scale=1.0, bias=0.0, bias_after_scale=True):
    t = _raw(x)
    return _wrap(t * scale if bias == 0.0 else (t * scale + bias if bias_after_scale else (t + bias) * scale))


def _sparse_divide_scalar(x, scalar):
    return _wrap(_raw(x) / scalar)


# ------------------------------------------------------------------------------ quantization / misc fused ops
def _qround(v, round_type):
    """round_type 0: ties to even (rint); 1: ties away from zero."""
    return torch.round(v) if round_type == 0 else torch.sign(v) * torch.floor(v.abs() + 0.5)


def _bnt(bit_length):
    return float((1 << (bit_length - 1)) - 1)


def fake_quantize_abs_max(x, bit_length=8, round_type=1):
    t = _raw(x)
    scale = t.abs().max().reshape(1)
    b = _bnt(bit_length)
    q = _qround(t / scale.clamp_min(1e-30) * b, round_type).clamp(-b, b)
    return _wrap(q), _wrap(scale)


def fake_quantize_dequantize_abs_max(x, bit_length=8, round_type=1):
    q, scale = fake_quantize_abs_max(x, bit_length, round_type)
    return _wrap(_raw(q) * _raw(scale) / _bnt(bit_length)), scale


def _chan_scale(t, quant_axis):
    dims = [d for d in range(t.dim()) if d != quant_axis]
    return t.abs().amax(dims)


def fake_channel_wise_quantize_abs_max(x, bit_length=8, round_type=1, quant_axis=0, is_test=False):
    t = _raw(x)
    sc = _chan_scale(t, quant_axis)
    shape = [1] * t.dim()
    shape[quant_axis] = -1
    b = _bnt(bit_length)
    q = _qround(t / sc.clamp_min(1e-30).view(shape) * b, round_type).clamp(-b, b)
    return _wrap(q), _wrap(sc)


def fake_channel_wise_quantize_dequantize_abs_max(x, bit_length=8, round_type=1, quant_axis=0):
    q, sc = fake_channel_wise_quantize_abs_max(x, bit_length, round_type, quant_axis)
    shape = [1] * _raw(q).dim()
    shape[quant_axis] = -1
    return _wrap(_raw(q) * _raw(sc).view(shape) / _bnt(bit_length)), sc


def fake_dequantize_max_abs(x, scale, max_range):
    return _wrap(_raw(x).float() * _raw(scale).float() / max_range)


def fake_channel_wise_dequantize_max_abs(x, scales, quant_bits=(8,), quant_axis=0, x_num_col_dims=1):
    t = _raw(x).float()
    sc = _raw(scales[0]).float()
    shape = [1] * t.dim()
    shape[quant_axis] = -1
    return _wrap(t * sc.view(shape) / _bnt(quant_bits[0]))


def fake_quantize_moving_average_abs_max(x, in_scale, in_accum=None, in_state=None, moving_rate=0.9,
                                         bit_length=8, is_test=False, round_type=1):
    t = _raw(x)
    if is_test or in_accum is None:
        scale = _raw(in_scale).reshape(1)
        accum, state = in_accum, in_state
    else:
        acc = moving_rate * _raw(in_accum) + t.abs().max()
        st = moving_rate * _raw(in_state) + 1
        scale = (acc / st).reshape(1)
        _raw(in_accum).copy_(acc)
        _raw(in_state).copy_(st)
        accum, state = in_accum, in_state
    b = _bnt(bit_length)
    q = _qround(t / scale.clamp_min(1e-30) * b, round_type).clamp(-b, b)
    return _wrap(q), _wrap(scale), state, accum


def fake_quantize_dequantize_moving_average_abs_max(x, in_scale, in_accum=None, in_state=None, moving_rate=0.9,
                                                    bit_length=8, is_test=False, round_type=1):
    q, scale, state, accum = fake_quantize_moving_average_abs_max(x, in_scale, in_accum, in_state, moving_rate,
                                                                  bit_length, is_test, round_type)
    return _wrap(_raw(q) * _raw(scale) / _bnt(bit_length)), scale, state, accum


def dequantize_log(x, dict):
    t = _raw(x).long()
    d = _raw(dict).float()
    v = d[t.abs() % d.numel()]
    return _wrap(torch.where(t < 0, -v, v))


def _fused_bias_dropout_residual_layer_norm(x, residual, bias=None, ln_scale=None, ln_bias=None, dropout_rate=0.5,
                                            ln_epsilon=1e-5, training=True, mode="upscale_in_train", name=None):
    from ..nn import functional as F

    h = x if bias is None else x + bias
    h = F.dropout(h, dropout_rate, training=training, mode=mode)
    y = _raw(h) + _raw(residual)
    n = y.shape[-1]
    return _wrap(torch.nn.functional.layer_norm(y, (n,), _raw(ln_scale) if ln_scale is not None else None,
                                                _raw(ln_bias) if ln_bias is not None else None, ln_epsilon))


@torch.no_grad()
def adadelta_(param, grad, avg_squared_grad, avg_squared_update, learning_rate, master_param=None, rho=0.95,
              epsilon=1e-6, multi_precision=False):
    p = _raw(master_param if (multi_precision and master_param is not None) else param).float()
    g = _raw(grad).float()
    asg = rho * _raw(avg_squared_grad).float() + (1 - rho) * g * g
    upd = -torch.sqrt((_raw(avg_squared_update).float() + epsilon) / (asg + epsilon)) * g
    asu = rho * _raw(avg_squared_update).float() + (1 - rho) * upd * upd
    new = p + _lr(learning_rate) * upd
    _upd(avg_squared_grad, asg)
    _upd(avg_squared_update, asu)
    _upd(param, new)
    if master_param is not None and multi_precision:
        _upd(master_param, new)
    return param, avg_squared_grad, avg_squared_update, master_param


def merged_adam_(param, grad, learning_rate, moment1, moment2, beta1_pow, beta2_pow, master_param=None, beta1=0.9,
                 beta2=0.999, epsilon=1e-8, multi_precision=False, use_global_beta_pow=False):
    mp = master_param or [None] * len(param)
    lrs = learning_rate if isinstance(learning_rate, (list, tuple)) else [learning_rate] * len(param)
    for i in range(len(param)):
        adam_(param[i], grad[i], lrs[i], moment1[i], moment2[i], beta1_pow[i], beta2_pow[i], mp[i], None, beta1,
              beta2, epsilon, multi_precision=multi_precision, use_global_beta_pow=use_global_beta_pow)
    return param, moment1, moment2, beta1_pow, beta2_pow, master_param


def merged_momentum_(param, grad, velocity, learning_rate, master_param=None, mu=0.9, use_nesterov=False,
                     regularization_method=(), regularization_coeff=(), multi_precision=False, rescale_grad=1.0):
    mp = master_param or [None] * len(param)
    lrs = learning_rate if isinstance(learning_rate, (list, tuple)) else [learning_rate] * len(param)
    for i in range(len(param)):
        rm = regularization_method[i] if regularization_method else ""
        rc = regularization_coeff[i] if regularization_coeff else 0.0
        momentum_(param[i], grad[i], velocity[i], lrs[i], mp[i], mu, use_nesterov, rm, rc, multi_precision,
                  rescale_grad)
    return param, velocity, master_param


def _c_allreduce_avg(x, ring_id=0, use_calc_stream=False, use_model_parallel=False):
    from ..distributed import ReduceOp

    return _c_allreduce(ReduceOp.AVG)(x)


def _tril_triu(x, diagonal=0, lower=True):
    from .. import tril, triu

    return tril(x, diagonal) if lower else triu(x, diagonal)


def _soft_relu(x, threshold=40.0):
    t = _raw(x)
    return _wrap(torch.log1p(torch.exp(t.clamp(-threshold, threshold))))


def quantize_linear(x, scale, zero_point=None, quant_axis=-1, bit_length=8, round_type=0, is_test=True,
                    only_observer=False):
    t, sc = _raw(x), _raw(scale)
    b = _bnt(bit_length)
    if sc.numel() > 1 and quant_axis >= 0:
        shape = [1] * t.dim()
        shape[quant_axis] = -1
        sc = sc.view(shape)
    zp = _raw(zero_point) if zero_point is not None else 0.0
    if only_observer:
        return x
    return _wrap((_qround(t / sc.clamp_min(1e-30) * b, round_type) + zp).clamp(-b - 1, b))


def dequantize_linear(x, scale, zero_point=None, quant_axis=-1, bit_length=8, round_type=0, is_test=True,
                      only_observer=False):
    t, sc = _raw(x).float(), _raw(scale).float()
    if only_observer:
        return x
    if sc.numel() > 1 and quant_axis >= 0:
        shape = [1] * t.dim()
        shape[quant_axis] = -1
        sc = sc.view(shape)
    zp = _raw(zero_point).float() if zero_point is not None else 0.0
    return _wrap((t - zp) * sc / _bnt(bit_length))


def _fused_gemm_epilogue(x, y, bias, trans_x=False, trans_y=False, activation="none"):
    from . import fused

    xt, yt = _raw(x), _raw(y)
    xt = xt.transpose(-1, -2) if trans_x else xt
    yt = yt.transpose(-1, -2) if trans_y else yt
    act = {"none": "identity", "": "identity"}.get(activation, activation)
    return _wrap(fused.bias_act(xt @ yt, _raw(bias), act))


def _selected_rows_value(x):
    from ..framework.tensor_types import SelectedRows

    return x.get_tensor() if isinstance(x, SelectedRows) else x


# ------------------------------------------------------------------------------ resolution
@functools.lru_cache(maxsize=1)
def reference_names():
    with open(os.path.join(_HERE, "reference_op_names.txt")) as f:
        return tuple(l.strip() for l in f if l.strip())


def _lookup(path):
    import paddle2_amd as root

    obj = root
    parts = path.split(".")
    for i, p in enumerate(parts):
        if not hasattr(obj, p):
            try:
                obj = importlib.import_module("paddle2_amd." + ".".join(parts[:i + 1]))
                continue
            except ImportError:
                return None
        obj = getattr(obj, p)
    return obj if callable(obj) else None


def resolve(name):
    """Reference op name -> callable (or None when this framework has no implementation)."""
    if name in ALIASES:
        path, kw = ALIASES[name]
        fn = _lookup(path)
        if fn is None:
            return None
        return functools.partial(fn, **kw) if kw else fn
    import paddle2_amd as root

    base = name[:-1] if name.endswith("_") and not name.endswith("__") else name
    if base.startswith("sparse_"):
        fn = getattr(root.sparse, base[len("sparse_"):], None) or getattr(root.sparse.nn.functional,
                                                                             base[len("sparse_"):], None)
        return fn if callable(fn) else None
    for mod in (root, root.nn.functional, root.linalg, root.fft, root.incubate.nn.functional, root.incubate,
                root.signal, root.geometric, root.vision.ops):
        fn = getattr(mod, base, None)
        if callable(fn) and not inspect.isclass(fn) and not inspect.ismodule(fn):
            if base != name and hasattr(root.Tensor, name):   # in-place variant: the Tensor method
                return getattr(root.Tensor, name)
            return fn
    meth = getattr(root.Tensor, name, None)
    return meth if callable(meth) else None


# ops whose implementation dispatches to a hand-written HIP kernel in paddle2_amd._C on the MI355X
NATIVE = {"matmul": "gemm", "fused_gemm_epilogue": "gemm", "fc": "gemm", "gemm_epilogue": "gemm",
          "fused_bias_act": "bias_act", "fused_dropout_add": "dropout_add", "batch_norm": "bn_fwd_train",
          "fused_batch_norm_act": "bn_fwd_train", "fused_bn_add_activation": "bn_fwd_train",
          "weight_only_linear": "wo_gemm", "masked_multihead_attention": "decode_attn",
          "block_multihead_attention": "decode_attn", "fused_moe": "gemm_grouped", "rms_norm": "norm_fwd",
          "layer_norm": "norm_fwd", "fused_bias_residual_layernorm": "norm_fwd", "softmax_mask_fuse": "softmax_mask_fwd",
          "memory_efficient_attention": "flash_fwd_ext", "variable_length_memory_efficient_attention": "flash_fwd_ext",
          "flash_attn_varlen_qkvpacked": "flash_fwd_ext", "flash_attn_qkvpacked": "flash_fwd",
          "merged_adam_": None}

_POPULATED = [False]


def populate():
    """Register every resolvable reference op in the op table; -> (registered, missing names)."""
    from .registry import _TABLE, register_op

    missing = []
    n = 0
    for name in reference_names():
        if _out_of_scope(name):
            continue
        if name in _TABLE:
            n += 1
            continue
        fn = resolve(name)
        if fn is None:
            missing.append(name)
            continue
        register_op(name, fn, native_kernel=NATIVE.get(name), inplace=name.endswith("_"))
        n += 1
    _POPULATED[0] = True
    return n, missing


def coverage():
    """Counts over the reference inventory minus the XPU-only fused kernels (out of scope)."""
    n, missing = populate()
    in_scope = [x for x in reference_names() if not _out_of_scope(x)]
    return {"reference_ops": len(in_scope), "implemented": n, "missing": missing,
            "out_of_scope": len(reference_names()) - len(in_scope)}


# ------------------------------------------------------------------------------ schema + infer_meta
def op_schema(name):
    """A reference-style schema record for ``name``: args (with defaults), inplace-ness, backing kernel."""
    from .registry import kernel_info, select

    if not _POPULATED[0]:
        populate()
    e = select(name)
    fn = e.fn.func if isinstance(e.fn, functools.partial) else e.fn
    try:
        sig = inspect.signature(fn)
        args = [{"name": p.name, "default": None if p.default is inspect.Parameter.empty else repr(p.default),
                 "kind": str(p.kind).split(".")[-1]} for p in sig.parameters.values()]
    except (TypeError, ValueError):
        args = []
    info = kernel_info(name)
    impl = getattr(fn, "__module__", "") + "." + getattr(fn, "__qualname__", getattr(fn, "__name__", ""))
    from .registry import has_op

    base = name[:-1] if name.endswith("_") else name
    inplace_variant = base + "_" if (not name.endswith("_") and has_op(base + "_")) else None
    return {"op": name, "args": args, "inplace": e.inplace, "inplace_variant": inplace_variant,
            "inplace_of": base if name.endswith("_") and has_op(base) else None, "impl": impl,
            "native_kernel": info["native_kernel"], "backward": backward_info(base)}


# no gradient flows through these (reference backward.yaml has no *_grad entry for them): comparisons, logical /
# bitwise ops, index-valued outputs, constants, random sources, shape / metadata queries, optimizer updates
_NO_GRAD_PREFIX = ("equal", "not_equal", "less", "greater", "logical_", "bitwise_", "is", "arg", "full", "zeros",
                   "ones", "empty", "arange", "linspace", "logspace", "eye", "randint", "randperm", "uniform",
                   "gaussian", "bernoulli", "multinomial", "poisson", "shape", "numel", "rank", "accuracy", "auc",
                   "one_hot", "unique", "nonzero", "histogram", "bincount", "searchsorted", "bucketize", "sign",
                   "floor", "ceil", "round", "trunc", "c_", "send", "recv", "barrier", "all_", "reduce_scatter",
                   "broadcast", "fake_", "dequantize", "quantize", "check_", "memcpy", "print", "top_p", "nms",
                   "sgd_", "momentum_", "adam", "adamw", "lamb_", "rmsprop_", "adagrad_", "adamax_", "adadelta_",
                   "merged_", "update_loss_scaling", "check_finite")


def backward_info(name):
    """How ``name`` is differentiated here (the reference declares it in backward.yaml as ``<name>_grad``):
    ``none`` (not differentiable), ``prim_vjp`` (a primitive VJP rule over PIR, decomposition/vjp.py),
    ``composite`` (decomposed into primitives that carry VJP rules, decomposition/rules.py) or ``autograd``
    (dygraph autograd through the implementation: a torch.autograd.Function with a hand-written / native
    backward, or differentiable torch ops)."""
    from .. import decomposition as D
    from ..decomposition import vjp as V

    if name.startswith(_NO_GRAD_PREFIX):
        return {"kind": "none", "grad_op": None}
    key = "pd_op." + name
    if key in V.VJP:
        kind = "none" if V.VJP[key] is V._v_none else "prim_vjp"
    elif D.has_rule(key):
        kind = "composite"
    else:
        kind = "autograd"
    return {"kind": kind, "grad_op": None if kind == "none" else name + "_grad"}


def _to_meta(x):
    from ..framework.tensor import Tensor

    if isinstance(x, Tensor):
        t = x._t
        return Tensor._wrap(torch.empty(t.shape, dtype=t.dtype, device="meta"))
    if isinstance(x, torch.Tensor):
        return torch.empty(x.shape, dtype=x.dtype, device="meta")
    if isinstance(x, (list, tuple)):
        return type(x)(_to_meta(v) for v in x)
    return x


class MetaTensor:
    """Output description from infer_meta (reference phi::MetaTensor: dims + dtype)."""

    def __init__(self, shape, dtype):
        self.shape, self.dtype = list(shape), dtype

    def __repr__(self):
        return f"MetaTensor(shape={self.shape}, dtype={str(self.dtype).replace('torch.', '')})"

    def __eq__(self, other):
        return isinstance(other, MetaTensor) and self.shape == other.shape and self.dtype == other.dtype


def infer_meta(name, *args, **kwargs):
    """Output shapes / dtypes of op ``name`` for these inputs, computed on meta tensors (no data, no device
    work) -> MetaTensor or a tuple of them."""
    from ..framework.tensor import Tensor
    from .registry import has_op, select

    if not has_op(name):
        populate()
    fn = select(name).fn
    margs = [_to_meta(a) for a in args]
    mkw = {k: _to_meta(v) for k, v in kwargs.items()}
    out = fn(*margs, **mkw)

    def desc(o):
        t = o._t if isinstance(o, Tensor) else o
        if isinstance(t, torch.Tensor):
            return MetaTensor(t.shape, t.dtype)
        if isinstance(t, (list, tuple)):
            return type(t)(desc(v) for v in t)
        return t

    return desc(out)
