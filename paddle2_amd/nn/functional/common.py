"""Common functional ops: linear, dropout, pad, interpolate, embedding, one_hot ...

Reference: python/paddle/nn/functional/{common,input}.py.  Paddle stores Linear weights as
``[in_features, out_features]`` so ``linear(x, W, b) = x @ W + b``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor
from ...tensor._helpers import shape_arg, ut
from ...amp import amp_op as _amp_op  # noqa: E402

_wrap = Tensor._wrap


@_amp_op("linear")
def linear(x, weight, bias=None, name=None):
    t = x._t
    w = weight._t
    from ...ops import torch_ops as T

    if isinstance(t, T._DTensor) or isinstance(w, T._DTensor):   # DistTensor: SPMD dispatch (matmul rule)
        return _wrap(T.linear(t, w, None if bias is None else bias._t))

    if (t.is_cuda and t.dtype in (torch.bfloat16, torch.float16) and w.dim() == 2) or \
            getattr(w, "_p2_gt", None) is not None or T.WeightGradStore.route:  # main grad / zero-bubble split
        return _wrap(T.linear(t, w, None if bias is None else bias._t))
    if bias is not None:
        b = bias._t
        if t.dim() == 2:
            return _wrap(torch.addmm(b, t, w))
        return _wrap(torch.matmul(t, w) + b)
    return _wrap(torch.matmul(t, w))


def bilinear(x1, x2, weight, bias=None, name=None):
    return _wrap(F.bilinear(x1._t, x2._t, weight._t, None if bias is None else bias._t.reshape(-1)))


def dropout(x, p=0.5, axis=None, training=True, mode="upscale_in_train", name=None):
    t = x._t
    if not training or p == 0.0:
        if mode == "downscale_in_infer" and not training:
            return _wrap(t * (1.0 - p))
        return x
    if p == 1.0:
        return _wrap(torch.zeros_like(t))
    if axis is None:
        if mode == "upscale_in_train":
            return _wrap(F.dropout(t, p, True))
        mask = torch.bernoulli(torch.full_like(t, 1.0 - p))
        return _wrap(t * mask)
    axes = [axis] if isinstance(axis, int) else list(axis)
    mshape = [t.shape[i] if i in [a % t.dim() for a in axes] else 1 for i in range(t.dim())]
    mask = torch.bernoulli(torch.full(mshape, 1.0 - p, device=t.device, dtype=t.dtype))
    if mode == "upscale_in_train":
        return _wrap(t * mask / (1.0 - p))
    return _wrap(t * mask)


def dropout2d(x, p=0.5, training=True, data_format="NCHW", name=None):
    return dropout(x, p, axis=[0, 1] if data_format == "NCHW" else [0, 3], training=training)


def dropout3d(x, p=0.5, training=True, data_format="NCDHW", name=None):
    return dropout(x, p, axis=[0, 1] if data_format == "NCDHW" else [0, 4], training=training)


def alpha_dropout(x, p=0.5, training=True, name=None):
    return _wrap(F.alpha_dropout(x._t, p, training))


def feature_alpha_dropout(x, p=0.5, training=True, name=None):
    return _wrap(F.feature_alpha_dropout(x._t, p, training))


def pad(x, pad, mode="constant", value=0.0, data_format="NCHW", pad_from_left_axis=True, name=None):
    t = x._t
    p = shape_arg(pad) if not isinstance(pad, (list, tuple)) else [int(v.item()) if isinstance(v, Tensor) else int(v) for v in pad]
    nd = t.dim()
    if len(p) == 2 * nd and mode == "constant":
        # paddle full-rank pad: [d0_lo, d0_hi, d1_lo, d1_hi, ...] from first axis
        tp = []
        for i in reversed(range(nd)):
            tp += [p[2 * i], p[2 * i + 1]]
        return _wrap(F.pad(t, tp, "constant", value))
    # spatial pad: paddle order [left, right, top, bottom, front, back] on the last dims
    channel_last = data_format in ("NHWC", "NLC", "NDHWC")
    if channel_last:
        t = t.movedim(-1, 1)
    mode_map = {"constant": "constant", "reflect": "reflect", "replicate": "replicate", "circular": "circular"}
    out = F.pad(t, p, mode_map[mode], value if mode == "constant" else None)
    if channel_last:
        out = out.movedim(1, -1)
    return _wrap(out)


def zeropad2d(x, padding, data_format="NCHW", name=None):
    return pad(x, padding, "constant", 0.0, data_format)


def interpolate(x, size=None, scale_factor=None, mode="nearest", align_corners=False, align_mode=0,
                data_format="NCHW", name=None):
    t = x._t
    channel_last = data_format in ("NHWC", "NLC", "NDHWC")
    if channel_last:
        t = t.movedim(-1, 1)
    if isinstance(size, Tensor):
        size = size._t.tolist()
    if isinstance(size, (list, tuple)):
        size = [int(s.item()) if isinstance(s, Tensor) else int(s) for s in size]
    m = {"nearest": "nearest", "bilinear": "bilinear", "trilinear": "trilinear", "bicubic": "bicubic",
         "linear": "linear", "area": "area"}[mode.lower()]
    kw = {}
    if m in ("bilinear", "trilinear", "bicubic", "linear"):
        kw["align_corners"] = align_corners
    out = F.interpolate(t, size=size, scale_factor=scale_factor, mode=m, **kw)
    if channel_last:
        out = out.movedim(1, -1)
    return _wrap(out)


upsample = interpolate


def embedding(x, weight, padding_idx=None, sparse=False, max_norm=None, norm_type=2.0, scale_grad_by_freq=False, name=None):
    from ...ops import embedding as _emb

    if sparse:
        # row-sparse weight gradient (SelectedRows): the optimizers update only the looked-up rows
        return _wrap(F.embedding(x._t.long(), weight._t, padding_idx=padding_idx, sparse=True))
    return _emb(x, weight, padding_idx)


def one_hot(x, num_classes, name=None):
    return _wrap(F.one_hot(x._t.long(), num_classes).to(torch.float32))


def label_smooth(label, prior_dist=None, epsilon=0.1, name=None):
    t = label._t
    k = t.shape[-1]
    if prior_dist is None:
        return _wrap((1 - epsilon) * t + epsilon / k)
    return _wrap((1 - epsilon) * t + epsilon * prior_dist._t)


def cosine_similarity(x1, x2, axis=1, eps=1e-8):
    return _wrap(F.cosine_similarity(x1._t, x2._t, axis, eps))


def pairwise_distance(x, y, p=2.0, epsilon=1e-6, keepdim=False, name=None):
    return _wrap(F.pairwise_distance(x._t, y._t, p, epsilon, keepdim))


def normalize(x, p=2, axis=1, epsilon=1e-12, name=None):
    return _wrap(F.normalize(x._t, p, axis, epsilon))


def unfold(x, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return _wrap(F.unfold(x._t, kernel_sizes, dilations, paddings, strides))


def fold(x, output_sizes, kernel_sizes, strides=1, paddings=0, dilations=1, name=None):
    return _wrap(F.fold(x._t, output_sizes, kernel_sizes, dilations, paddings, strides))


def pixel_shuffle(x, upscale_factor, data_format="NCHW", name=None):
    t = x._t
    if data_format == "NHWC":
        return _wrap(F.pixel_shuffle(t.permute(0, 3, 1, 2), upscale_factor).permute(0, 2, 3, 1))
    return _wrap(F.pixel_shuffle(t, upscale_factor))


def pixel_unshuffle(x, downscale_factor, data_format="NCHW", name=None):
    t = x._t
    if data_format == "NHWC":
        return _wrap(F.pixel_unshuffle(t.permute(0, 3, 1, 2), downscale_factor).permute(0, 2, 3, 1))
    return _wrap(F.pixel_unshuffle(t, downscale_factor))


def channel_shuffle(x, groups, data_format="NCHW", name=None):
    t = x._t
    if data_format == "NHWC":
        return _wrap(F.channel_shuffle(t.permute(0, 3, 1, 2), groups).permute(0, 2, 3, 1))
    return _wrap(F.channel_shuffle(t, groups))


def grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=True, name=None):
    return _wrap(F.grid_sample(x._t, grid._t, mode, padding_mode, align_corners))


def affine_grid(theta, out_shape, align_corners=True, name=None):
    return _wrap(F.affine_grid(theta._t, shape_arg(out_shape), align_corners))


def class_center_sample(label, num_classes, num_samples, group=None):
    t = label._t
    pos = torch.unique(t)
    if pos.numel() < num_samples:
        perm = torch.randperm(num_classes, device=t.device)
        extra = perm[~torch.isin(perm, pos)][: num_samples - pos.numel()]
        sampled = torch.cat([pos, extra]).sort().values
    else:
        sampled = pos
    remap = torch.full((num_classes,), -1, dtype=torch.long, device=t.device)
    remap[sampled] = torch.arange(sampled.numel(), device=t.device)
    return _wrap(remap[t]), _wrap(sampled)


def sequence_mask(x, maxlen=None, dtype="int64", name=None):
    from ...framework.dtype import convert_dtype

    t = x._t
    m = int(t.max().item()) if maxlen is None else int(maxlen)
    r = torch.arange(m, device=t.device)
    return _wrap((r < t.unsqueeze(-1)).to(convert_dtype(dtype)))


def temporal_shift(x, seg_num, shift_ratio=0.25, data_format="NCHW", name=None):
    t = x._t
    nt, c, h, w = t.shape
    n = nt // seg_num
    t = t.reshape(n, seg_num, c, h, w)
    fold_ = int(c * shift_ratio)
    out = torch.zeros_like(t)
    out[:, :-1, :fold_] = t[:, 1:, :fold_]
    out[:, 1:, fold_:2 * fold_] = t[:, :-1, fold_:2 * fold_]
    out[:, :, 2 * fold_:] = t[:, :, 2 * fold_:]
    return _wrap(out.reshape(nt, c, h, w))


def _ut(x):
    return ut(x)
