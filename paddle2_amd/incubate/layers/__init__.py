"""paddle.incubate.layers (reference: python/paddle/incubate/layers/nn.py): the fused / sequence / recommender
layers of the legacy static API, over the framework's op table (ops/extra_ops.py and friends)."""
from __future__ import annotations

from ...ops import op_schema as _S

__all__ = ["fused_seqpool_cvm", "search_pyramid_hash", "shuffle_batch", "partial_concat", "partial_sum",
           "tdm_child", "tdm_sampler", "rank_attention", "batch_fc", "correlation", "fused_bn_add_act",
           "pow2_decay_with_linear_warmup", "multiclass_nms2", "fused_embedding_seq_pool", "bilateral_slice"]


def _op(name):
    fn = _S.resolve(name)
    if fn is None:
        raise NotImplementedError(name)
    return fn


def fused_seqpool_cvm(input, pool_type, cvm, pad_value=0.0, use_cvm=True, cvm_offset=2):
    return _op("fused_seqpool_cvm")(input, cvm, pooltype=pool_type.upper(), pad_value=pad_value, use_cvm=use_cvm,
                                    cvm_offset=cvm_offset)


def search_pyramid_hash(input, num_emb, space_len, pyramid_layer, rand_len, drop_out_percent, is_training,
                        use_filter, white_list_len, black_list_len, seed, lr, param_attr=None,
                        param_attr_wl=None, param_attr_bl=None, name=None, distribute_update_vars=None,
                        dtype="float32"):
    return _op("pyramid_hash")(input, num_emb=num_emb, space_len=space_len, pyramid_layer=pyramid_layer,
                               rand_len=rand_len, drop_out_percent=drop_out_percent, is_training=is_training,
                               use_filter=use_filter, white_list_len=white_list_len,
                               black_list_len=black_list_len, seed=seed, lr=lr)


def shuffle_batch(x, seed=None):
    return _op("shuffle_batch")(x, seed)


def partial_concat(input, start_index=0, length=-1):
    return _op("partial_concat")(input, start_index, length)


def partial_sum(input, start_index=0, length=-1):
    return _op("partial_sum")(input, start_index, length)


def tdm_child(x, node_nums, child_nums, param_attr=None, dtype="int32"):
    return _op("tdm_child")(x, node_nums=node_nums, child_nums=child_nums, param_attr=param_attr, dtype=dtype)


def tdm_sampler(x, neg_samples_num_list, layer_node_num_list, leaf_node_num, tree_travel_attr=None,
                tree_layer_attr=None, output_positive=True, output_list=True, seed=0, tree_dtype="int32",
                dtype="int32"):
    return _op("tdm_sampler")(x, neg_samples_num_list, layer_node_num_list, leaf_node_num,
                              tree_travel_attr=tree_travel_attr, tree_layer_attr=tree_layer_attr,
                              output_positive=output_positive, output_list=output_list, seed=seed)


def rank_attention(input, rank_offset, rank_param_shape, rank_param_attr=None, max_rank=3, max_size=0):
    return _op("rank_attention")(input, rank_offset, rank_param_shape=rank_param_shape,
                                 rank_param_attr=rank_param_attr, max_rank=max_rank, max_size=max_size)


def batch_fc(input, param_size, param_attr=None, bias_size=None, bias_attr=None, act=None):
    return _op("batch_fc")(input, param_size=param_size, param_attr=param_attr, bias_size=bias_size,
                           bias_attr=bias_attr, act=act)


def correlation(x, y, pad_size, kernel_size, max_displacement, stride1, stride2, corr_type_multiply=1):
    return _op("correlation")(x, y, pad_size, kernel_size, max_displacement, stride1, stride2, corr_type_multiply)


def fused_bn_add_act(x, y, momentum=0.9, epsilon=1e-05, param_attr=None, bias_attr=None,
                     moving_mean_name=None, moving_variance_name=None, act=None, name=None):
    """BN(x) + y -> act (ReLU) on channels-last input (the fused BN+add+ReLU kernel)."""
    from ... import nn
    from ...nn.functional.norm import fused_bn_add_activation

    c = x.shape[-1]
    bn = nn.BatchNorm(c, momentum=momentum, epsilon=epsilon, data_layout="NHWC")
    return fused_bn_add_activation(x, y, bn.weight, bn.bias, bn._mean, bn._variance, momentum=momentum,
                                   epsilon=epsilon, act_type=act or "relu")


def pow2_decay_with_linear_warmup(warmup_steps, total_steps, base_lr, end_lr, dtype="float32", name=None):
    """LR schedule: linear warm-up to base_lr, then (1 - t / T)^2 decay to end_lr (reference nn.py)."""
    from ...optimizer.lr import LRScheduler

    class _Pow2Decay(LRScheduler):
        def get_lr(self):
            step = self.last_epoch
            if step < warmup_steps:
                return base_lr * step / max(warmup_steps, 1)
            if step >= total_steps:
                return end_lr
            frac = 1.0 - (step - warmup_steps) / max(total_steps - warmup_steps, 1)
            return (base_lr - end_lr) * frac * frac + end_lr

    return _Pow2Decay(learning_rate=base_lr)


def multiclass_nms2(bboxes, scores, score_threshold, nms_top_k, keep_top_k, nms_threshold=0.3, normalized=True,
                    nms_eta=1.0, background_label=0, return_index=False, name=None):
    out = _op("multiclass_nms")(bboxes, scores, score_threshold=score_threshold, nms_top_k=nms_top_k,
                                keep_top_k=keep_top_k, nms_threshold=nms_threshold, normalized=normalized,
                                nms_eta=nms_eta, background_label=background_label)
    if isinstance(out, (tuple, list)):
        return (out[0], out[1]) if return_index and len(out) > 1 else out[0]
    return out


def fused_embedding_seq_pool(input, size, is_sparse=False, padding_idx=None, combiner="sum", param_attr=None,
                             dtype="float32"):
    """Embedding lookup of a LoD id sequence summed per sequence (fusion of lookup_table + sequence_pool)."""
    from ... import nn
    from ...static import sequence as _seq

    emb = nn.Embedding(size[0], size[1], padding_idx=padding_idx, sparse=is_sparse)
    e = emb(input)
    if getattr(input, "lod", None) is not None:
        return _seq.sequence_pool(e, "sum" if combiner == "sum" else combiner)
    return e.sum(axis=-2) if e.ndim > 2 else e


def bilateral_slice(x, guide, grid, has_offset, name=None):
    """HDRNet bilateral grid slicing: trilinear lookup of per-pixel affine coefficients from ``grid``
    [N, C*(D+1 if offset), gd, gh, gw] at (x, y, guide) and their application to ``x`` [N, D, H, W]."""
    import torch
    import torch.nn.functional as F

    from ...framework.tensor import Tensor

    xt, gt, gr = x._t.float(), guide._t.float(), grid._t.float()
    n, d, h, w = xt.shape
    coeffs = gr.shape[1]
    ys = torch.linspace(-1, 1, h, device=xt.device)
    xs = torch.linspace(-1, 1, w, device=xt.device)
    yy, xx = torch.meshgrid(ys, xs, indexing="ij")
    zz = gt * 2 - 1
    samp = torch.stack([xx.expand(n, h, w), yy.expand(n, h, w), zz], -1)[:, None]   # [N, 1, H, W, 3]
    co = F.grid_sample(gr, samp, mode="bilinear", align_corners=True)[:, :, 0]     # [N, coeffs, H, W]
    out_c = coeffs // (d + 1) if has_offset else coeffs // d
    co = co.view(n, out_c, d + 1 if has_offset else d, h, w)
    y = (co[:, :, :d] * xt[:, None]).sum(2)
    if has_offset:
        y = y + co[:, :, d]
    return Tensor._wrap(y.to(x._t.dtype))
