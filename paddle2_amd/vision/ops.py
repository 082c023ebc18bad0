"""paddle.vision.ops — detection / region operators (reference: python/paddle/vision/ops.py with the phi CPU
kernels yolo_box_kernel.cc + funcs/yolo_box_util.h, yolo_loss_kernel.cc, prior_box_kernel.cc,
box_coder_kernel.cc, roi_align_kernel.cc, roi_pool_kernel.cc, psroi_pool_kernel.cc, nms_kernel.cc,
matrix_nms_kernel.cc, generate_proposals_kernel.cc (+ funcs/detection/nms_util.h),
distribute_fpn_proposals_kernel.cc, funcs/deformable_conv_functor.cc).

Everything is written as batched tensor math (gathers, masks, segment reductions) so the same code runs on
the MI355X and on the CPU; only the inherently sequential greedy NMS walks run as host loops over a
precomputed IoU matrix.  Differentiable ops (roi_align, roi_pool, psroi_pool, deform_conv2d, yolo_loss, box
coding) get their gradients from autograd of the forward math.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from ..framework.tensor import Tensor
from ..nn.layer.layers import Layer

_w = Tensor._wrap

__all__ = ["yolo_loss", "yolo_box", "prior_box", "box_coder", "deform_conv2d", "DeformConv2D",
           "distribute_fpn_proposals", "generate_proposals", "read_file", "decode_jpeg", "roi_pool", "RoIPool",
           "psroi_pool", "PSRoIPool", "roi_align", "RoIAlign", "nms", "matrix_nms", "ConvNormActivation"]


def _t(x):
    if x is None:
        return None
    if isinstance(x, Tensor):
        return x._t
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x))


def _pair(v):
    return (v, v) if isinstance(v, int) else tuple(v)


# ================================================================================================ YOLO
def _yolo_parts(x, an_num, class_num, iou_aware):
    n, c, h, w = x.shape
    if iou_aware:
        iou = x[:, :an_num]
        rest = x[:, an_num:].reshape(n, an_num, 5 + class_num, h, w)
        return rest, iou
    return x.reshape(n, an_num, 5 + class_num, h, w), None


def yolo_box(x, img_size, anchors, class_num, conf_thresh, downsample_ratio, clip_bbox=True, name=None,
             scale_x_y=1.0, iou_aware=False, iou_aware_factor=0.5):
    """YOLOv3 head -> boxes [N, an*H*W, 4] (x1, y1, x2, y2 in image pixels) and scores [N, an*H*W, class_num];
    entries whose confidence is below ``conf_thresh`` are zero."""
    xt, sz = _t(x), _t(img_size)
    an_num = len(anchors) // 2
    n, _, h, w = xt.shape
    rest, iou = _yolo_parts(xt, an_num, class_num, iou_aware)
    dt = xt.dtype
    conf = torch.sigmoid(rest[:, :, 4])
    if iou_aware:
        conf = conf.pow(1.0 - iou_aware_factor) * torch.sigmoid(iou).pow(iou_aware_factor)
    bias = -0.5 * (scale_x_y - 1.0)
    img_h = sz[:, 0].to(dt).view(n, 1, 1, 1)
    img_w = sz[:, 1].to(dt).view(n, 1, 1, 1)
    gx = torch.arange(w, device=xt.device, dtype=dt).view(1, 1, 1, w)
    gy = torch.arange(h, device=xt.device, dtype=dt).view(1, 1, h, 1)
    an = torch.as_tensor(anchors, dtype=dt, device=xt.device).view(an_num, 2)
    cx = (gx + torch.sigmoid(rest[:, :, 0]) * scale_x_y + bias) * img_w / w
    cy = (gy + torch.sigmoid(rest[:, :, 1]) * scale_x_y + bias) * img_h / h
    bw = torch.exp(rest[:, :, 2]) * an[:, 0].view(1, an_num, 1, 1) * img_w / (downsample_ratio * w)
    bh = torch.exp(rest[:, :, 3]) * an[:, 1].view(1, an_num, 1, 1) * img_h / (downsample_ratio * h)
    x1, y1, x2, y2 = cx - bw / 2, cy - bh / 2, cx + bw / 2, cy + bh / 2
    if clip_bbox:
        x1 = x1.clamp_min(0)
        y1 = y1.clamp_min(0)
        x2 = torch.minimum(x2, img_w - 1)
        y2 = torch.minimum(y2, img_h - 1)
    keep = (conf >= conf_thresh).to(dt)
    boxes = torch.stack([x1, y1, x2, y2], -1) * keep.unsqueeze(-1)
    scores = conf.unsqueeze(2) * torch.sigmoid(rest[:, :, 5:]) * keep.unsqueeze(2)
    boxes = boxes.reshape(n, an_num * h * w, 4)
    scores = scores.permute(0, 1, 3, 4, 2).reshape(n, an_num * h * w, class_num)
    return _w(boxes), _w(scores)


def _sce(x, label):
    """sigmoid cross-entropy with logits (reference SigmoidCrossEntropy)."""
    return x.clamp_min(0) - x * label + torch.log1p(torch.exp(-x.abs()))


def _iou_cxcywh(b1, b2):
    def ov(c1, w1, c2, w2):
        return torch.minimum(c1 + w1 / 2, c2 + w2 / 2) - torch.maximum(c1 - w1 / 2, c2 - w2 / 2)

    iw = ov(b1[..., 0], b1[..., 2], b2[..., 0], b2[..., 2])
    ih = ov(b1[..., 1], b1[..., 3], b2[..., 1], b2[..., 3])
    inter = torch.where((iw < 0) | (ih < 0), torch.zeros_like(iw), iw * ih)
    union = b1[..., 2] * b1[..., 3] + b2[..., 2] * b2[..., 3] - inter
    return inter / union


def yolo_loss(x, gt_box, gt_label, anchors, anchor_mask, class_num, ignore_thresh, downsample_ratio, gt_score=None,
              use_label_smooth=True, name=None, scale_x_y=1.0):
    """YOLOv3 loss per image [N]: location (sigmoid-CE on x/y, L1 on log w/h, weighted by 2 - w*h), class
    sigmoid-CE and objectness sigmoid-CE with predictions overlapping any GT above ``ignore_thresh`` ignored.
    ``gt_box`` is [N, B, 4] normalized (cx, cy, w, h); boxes with w or h <= 0 are padding."""
    xt = _t(x)
    gtb = _t(gt_box).to(xt.dtype)
    gtl = _t(gt_label).long()
    n, _, h, w = xt.shape
    b = gtb.shape[1]
    an_num = len(anchors) // 2
    mask_num = len(anchor_mask)
    dev, dt = xt.device, xt.dtype
    gts = _t(gt_score).to(dt) if gt_score is not None else torch.ones(n, b, dtype=dt, device=dev)
    input_size = downsample_ratio * h
    stride_bias = -0.5 * (scale_x_y - 1.0)
    pred = xt.reshape(n, mask_num, 5 + class_num, h, w)
    an_all = torch.as_tensor(anchors, dtype=dt, device=dev).view(an_num, 2)
    an_m = an_all[torch.as_tensor(anchor_mask, device=dev)]
    if use_label_smooth:
        sw = min(1.0 / class_num, 1.0 / 40)
        pos, neg = 1.0 - sw, sw
    else:
        pos, neg = 1.0, 0.0
    valid = (gtb[..., 2] > 1e-6) & (gtb[..., 3] > 1e-6)   # LessEqualZero uses a 1e-6 tolerance
    with torch.no_grad():
        gx = torch.arange(w, device=dev, dtype=dt).view(1, 1, 1, w)
        gy = torch.arange(h, device=dev, dtype=dt).view(1, 1, h, 1)
        px = (gx + torch.sigmoid(pred[:, :, 0]) * scale_x_y + stride_bias) / w
        py = (gy + torch.sigmoid(pred[:, :, 1]) * scale_x_y + stride_bias) / h
        pw = torch.exp(pred[:, :, 2]) * an_m[:, 0].view(1, mask_num, 1, 1) / input_size
        ph = torch.exp(pred[:, :, 3]) * an_m[:, 1].view(1, mask_num, 1, 1) / input_size
        pboxes = torch.stack([px, py, pw, ph], -1)                          # [n, m, h, w, 4]
        ious = _iou_cxcywh(pboxes.unsqueeze(-2), gtb.view(n, 1, 1, 1, b, 4))  # [n, m, h, w, b]
        ious = torch.where(valid.view(n, 1, 1, 1, b), ious, torch.zeros_like(ious))
        best = ious.amax(-1) if b else torch.zeros(n, mask_num, h, w, dtype=dt, device=dev)
        obj_mask = torch.where(best > ignore_thresh, torch.full_like(best, -1.0), torch.zeros_like(best))
        # anchor matching on shape only
        an_box = torch.cat([torch.zeros(an_num, 2, dtype=dt, device=dev), an_all / input_size], -1)
        gt_shift = torch.cat([torch.zeros(n, b, 2, dtype=dt, device=dev), gtb[..., 2:]], -1)
        an_iou = _iou_cxcywh(an_box.view(1, 1, an_num, 4), gt_shift.unsqueeze(2))   # [n, b, an]
        # first index of the maximum (strictly greater wins), as the reference's scan
        best_n = an_iou.argmax(-1)
        lut = torch.full((an_num,), -1, dtype=torch.long, device=dev)
        lut[torch.as_tensor(anchor_mask, device=dev)] = torch.arange(mask_num, device=dev)
        mask_idx = torch.where(valid, lut[best_n], torch.full_like(best_n, -1))
        gi = (gtb[..., 0] * w).long().clamp(0, w - 1)
        gj = (gtb[..., 1] * h).long().clamp(0, h - 1)
    loss = torch.zeros(n, dtype=dt, device=dev)
    hit = mask_idx >= 0
    if bool(hit.any()):
        bi, ti = hit.nonzero(as_tuple=True)
        mi, cj, ci = mask_idx[bi, ti], gj[bi, ti], gi[bi, ti]
        g = gtb[bi, ti]
        sc = gts[bi, ti]
        anc = an_all[best_n[bi, ti]]
        p = pred[bi, mi, :, cj, ci]                                   # [k, 5 + C]
        tx = g[:, 0] * w - ci.to(dt)
        ty = g[:, 1] * h - cj.to(dt)
        tw = torch.log(g[:, 2] * input_size / anc[:, 0])
        th = torch.log(g[:, 3] * input_size / anc[:, 1])
        scale = (2.0 - g[:, 2] * g[:, 3]) * sc
        loc = (_sce(p[:, 0], tx) + _sce(p[:, 1], ty) + (p[:, 2] - tw).abs() + (p[:, 3] - th).abs()) * scale
        onehot = F.one_hot(gtl[bi, ti], class_num).to(dt)
        lab = onehot * pos + (1 - onehot) * neg
        cls = (_sce(p[:, 5:], lab) * sc.unsqueeze(1)).sum(1)
        loss = loss.index_add(0, bi, loc + cls)
        with torch.no_grad():
            # later GTs overwrite earlier ones on the same cell (sequential scan order)
            order = torch.arange(bi.numel(), device=dev)
            key = ((bi * mask_num + mi) * h + cj) * w + ci
            last = torch.full((n * mask_num * h * w,), -1, dtype=torch.long, device=dev)
            last.scatter_reduce_(0, key, order, reduce="amax")
            win = last[key] == order
            obj_mask.view(-1)[key[win]] = sc[win]
    obj_logit = pred[:, :, 4]
    pos_m = obj_mask > 1e-5
    neg_m = (~pos_m) & (obj_mask > -0.5)
    obj = torch.where(pos_m, _sce(obj_logit, torch.ones_like(obj_logit)) * obj_mask, torch.zeros_like(obj_logit))
    obj = obj + torch.where(neg_m, _sce(obj_logit, torch.zeros_like(obj_logit)), torch.zeros_like(obj_logit))
    loss = loss + obj.reshape(n, -1).sum(1)
    return _w(loss)


# ================================================================================================ SSD priors / coding
def _expand_ars(ars, flip):
    out = [1.0]
    for ar in ars:
        if all(abs(ar - o) >= 1e-6 for o in out):
            out.append(ar)
            if flip:
                out.append(1.0 / ar)
    return out


def prior_box(input, image, min_sizes, max_sizes=None, aspect_ratios=[1.0], variance=[0.1, 0.1, 0.2, 0.2],
              flip=False, clip=False, steps=[0.0, 0.0], offset=0.5, min_max_aspect_ratios_order=False, name=None):
    """SSD prior boxes -> (boxes [H, W, P, 4] normalized, variances [H, W, P, 4])."""
    it, im = _t(input), _t(image)
    min_sizes = [float(m) for m in (min_sizes if isinstance(min_sizes, (list, tuple)) else [min_sizes])]
    max_sizes = [float(m) for m in (max_sizes if isinstance(max_sizes, (list, tuple)) else
                                    ([] if max_sizes is None else [max_sizes]))]
    ars = _expand_ars([float(a) for a in (aspect_ratios if isinstance(aspect_ratios, (list, tuple))
                                          else [aspect_ratios])], flip)
    fh, fw = it.shape[2], it.shape[3]
    ih, iw = im.shape[2], im.shape[3]
    sw, sh = float(steps[0]), float(steps[1])
    if sw == 0 or sh == 0:
        sw, sh = iw / fw, ih / fh
    # per-location list of (half width, half height) in the reference's order
    halves = []
    for s, ms in enumerate(min_sizes):
        if min_max_aspect_ratios_order:
            halves.append((ms / 2.0, ms / 2.0))
            if max_sizes:
                v = math.sqrt(ms * max_sizes[s]) / 2.0
                halves.append((v, v))
            for ar in ars:
                if abs(ar - 1.0) < 1e-6:
                    continue
                halves.append((ms * math.sqrt(ar) / 2.0, ms / math.sqrt(ar) / 2.0))
        else:
            for ar in ars:
                halves.append((ms * math.sqrt(ar) / 2.0, ms / math.sqrt(ar) / 2.0))
            if max_sizes:
                v = math.sqrt(ms * max_sizes[s]) / 2.0
                halves.append((v, v))
    dt = it.dtype if it.is_floating_point() else torch.float32
    hv = torch.as_tensor(halves, dtype=dt, device=it.device)                   # [P, 2]
    cx = (torch.arange(fw, dtype=dt, device=it.device) + offset) * sw
    cy = (torch.arange(fh, dtype=dt, device=it.device) + offset) * sh
    cx = cx.view(1, fw, 1)
    cy = cy.view(fh, 1, 1)
    P = hv.shape[0]
    cx = cx.expand(fh, fw, P)
    cy = cy.expand(fh, fw, P)
    boxes = torch.stack([(cx - hv[:, 0]) / iw, (cy - hv[:, 1]) / ih, (cx + hv[:, 0]) / iw, (cy + hv[:, 1]) / ih],
                        -1).contiguous()
    if clip:
        boxes = boxes.clamp(0.0, 1.0)
    var = torch.as_tensor(variance, dtype=dt, device=it.device).expand_as(boxes).contiguous()
    return _w(boxes), _w(var)


def box_coder(prior_box, prior_box_var, target_box, code_type="encode_center_size", box_normalized=True, axis=0,
              name=None):
    """Encode target boxes against priors (-> [T, P, 4]) or decode deltas ([T, P, 4] -> boxes)."""
    pb, tb = _t(prior_box), _t(target_box)
    off = 0.0 if box_normalized else 1.0
    var_t = _t(prior_box_var) if isinstance(prior_box_var, (Tensor, torch.Tensor)) else None
    var_l = list(prior_box_var) if isinstance(prior_box_var, (list, tuple)) else None
    pw = pb[:, 2] - pb[:, 0] + off
    ph = pb[:, 3] - pb[:, 1] + off
    pcx = pb[:, 0] + pw / 2
    pcy = pb[:, 1] + ph / 2
    if code_type.lower() in ("encode_center_size", "encodecentersize"):
        tw = tb[:, 2] - tb[:, 0] + off
        th = tb[:, 3] - tb[:, 1] + off
        tcx = (tb[:, 2] + tb[:, 0]) / 2
        tcy = (tb[:, 3] + tb[:, 1]) / 2
        out = torch.stack([(tcx[:, None] - pcx[None]) / pw[None], (tcy[:, None] - pcy[None]) / ph[None],
                           torch.log((tw[:, None] / pw[None]).abs()), torch.log((th[:, None] / ph[None]).abs())], -1)
        if var_t is not None:
            out = out / var_t.view(1, -1, 4)
        elif var_l:
            out = out / torch.as_tensor(var_l, dtype=out.dtype, device=out.device)
        return _w(out)
    # decode: target [T, P, 4]; priors broadcast along `axis`
    shape = (1, -1) if axis == 0 else (-1, 1)
    pw, ph, pcx, pcy = (v.view(*shape) for v in (pw, ph, pcx, pcy))
    if var_t is not None:
        vv = var_t.view(*shape, 4)
        vx, vy, vw, vh = vv[..., 0], vv[..., 1], vv[..., 2], vv[..., 3]
    elif var_l:
        vx, vy, vw, vh = var_l
    else:
        vx = vy = vw = vh = 1.0
    cx = vx * tb[..., 0] * pw + pcx
    cy = vy * tb[..., 1] * ph + pcy
    ww = torch.exp(vw * tb[..., 2]) * pw
    hh = torch.exp(vh * tb[..., 3]) * ph
    out = torch.stack([cx - ww / 2, cy - hh / 2, cx + ww / 2 - off, cy + hh / 2 - off], -1)
    return _w(out)


# ================================================================================================ RoI ops
def _roi_batch_ids(boxes_num, n_rois, batch, device):
    if boxes_num is None:
        if batch != 1:
            raise ValueError("boxes_num is required when the batch has more than one image")
        return torch.zeros(n_rois, dtype=torch.long, device=device)
    bn = _t(boxes_num).to(device).long()
    if bn.numel() != batch:
        raise ValueError(f"The batch size of rois and the batch size of images must be the same. But received the "
                         f"batch size of rois is {bn.numel()}, and the batch size of images is {batch}")
    return torch.repeat_interleave(torch.arange(batch, device=device), bn)


def _bilinear(img, y, x):
    """img [C, H, W]; y, x [...] float (already clamped to the valid sample window) -> [C, ...]."""
    H, W = img.shape[-2:]
    y0 = y.floor().long().clamp(0, H - 1)
    x0 = x.floor().long().clamp(0, W - 1)
    y1 = (y0 + 1).clamp(max=H - 1)
    x1 = (x0 + 1).clamp(max=W - 1)
    ly, lx = y - y0.to(y.dtype), x - x0.to(x.dtype)
    hy, hx = 1 - ly, 1 - lx
    flat = img.reshape(img.shape[0], -1)

    def g(yy, xx):
        return flat[:, (yy * W + xx).reshape(-1)].reshape(img.shape[0], *y.shape)

    return hy * hx * g(y0, x0) + hy * lx * g(y0, x1) + ly * hx * g(y1, x0) + ly * lx * g(y1, x1)


def roi_align(x, boxes, boxes_num, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=True, name=None):
    """RoIAlign: average of bilinear samples on a regular grid per output bin -> [R, C, ph, pw]."""
    xt, bt = _t(x), _t(boxes)
    ph, pw = _pair(output_size)
    n, c, H, W = xt.shape
    R = bt.shape[0]
    out = xt.new_zeros(R, c, ph, pw)
    if R == 0:
        return _w(out)
    bid = _roi_batch_ids(boxes_num, R, n, xt.device)
    off = 0.5 if aligned else 0.0
    b = bt.to(xt.dtype) * spatial_scale - off
    rw = b[:, 2] - b[:, 0]
    rh = b[:, 3] - b[:, 1]
    if not aligned:
        rw = rw.clamp_min(1.0)
        rh = rh.clamp_min(1.0)
    if sampling_ratio > 0:
        gh = torch.full((R,), sampling_ratio, dtype=torch.long, device=xt.device)
        gw = gh.clone()
    else:
        gh = torch.ceil(rh / ph).long().clamp_min(1)
        gw = torch.ceil(rw / pw).long().clamp_min(1)
    outs = []
    for r in range(R):   # grids differ per roi: one vectorized sample per roi
        Gh, Gw = int(gh[r]), int(gw[r])
        iy = (torch.arange(ph, device=xt.device, dtype=xt.dtype).view(ph, 1) +
              (torch.arange(Gh, device=xt.device, dtype=xt.dtype).view(1, Gh) + 0.5) / Gh)   # [ph, Gh]
        ix = (torch.arange(pw, device=xt.device, dtype=xt.dtype).view(pw, 1) +
              (torch.arange(Gw, device=xt.device, dtype=xt.dtype).view(1, Gw) + 0.5) / Gw)
        ys = b[r, 1] + rh[r] / ph * iy
        xs = b[r, 0] + rw[r] / pw * ix
        Y = ys.view(ph, Gh, 1, 1).expand(ph, Gh, pw, Gw)
        X = xs.view(1, 1, pw, Gw).expand(ph, Gh, pw, Gw)
        inside = (Y >= -1.0) & (Y <= H) & (X >= -1.0) & (X <= W)
        Yc = Y.clamp_min(0)
        Xc = X.clamp_min(0)
        Yc = torch.where(Yc >= H - 1, torch.full_like(Yc, H - 1), Yc)
        Xc = torch.where(Xc >= W - 1, torch.full_like(Xc, W - 1), Xc)
        v = _bilinear(xt[bid[r]], Yc, Xc) * inside.to(xt.dtype)
        outs.append(v.sum((2, 4)) / (Gh * Gw))
    return _w(torch.stack(outs))


def roi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    """RoIPool (Fast R-CNN): max over integer-quantized bins; empty bins are 0 -> [R, C, ph, pw]."""
    xt, bt = _t(x), _t(boxes)
    ph, pw = _pair(output_size)
    n, c, H, W = xt.shape
    R = bt.shape[0]
    if R == 0:
        return _w(xt.new_zeros(0, c, ph, pw))
    bid = _roi_batch_ids(boxes_num, R, n, xt.device)
    q = torch.round(bt.double() * spatial_scale).long()
    sw, sh, ew, eh = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    bh = (eh - sh + 1).clamp_min(1).double() / ph
    bw = (ew - sw + 1).clamp_min(1).double() / pw
    ar_h = torch.arange(ph, device=xt.device).double()
    ar_w = torch.arange(pw, device=xt.device).double()
    hs = (torch.floor(ar_h[None] * bh[:, None]).long() + sh[:, None]).clamp(0, H)
    he = (torch.ceil((ar_h[None] + 1) * bh[:, None]).long() + sh[:, None]).clamp(0, H)
    ws = (torch.floor(ar_w[None] * bw[:, None]).long() + sw[:, None]).clamp(0, W)
    we = (torch.ceil((ar_w[None] + 1) * bw[:, None]).long() + sw[:, None]).clamp(0, W)
    neg = torch.finfo(xt.dtype).min if xt.is_floating_point() else torch.iinfo(xt.dtype).min
    out = xt.new_zeros(R, c, ph, pw)
    for r in range(R):   # crop each roi's window, then one masked max over all its bins
        h0, h1 = int(hs[r].min()), int(he[r].max())
        w0, w1 = int(ws[r].min()), int(we[r].max())
        if h1 <= h0 or w1 <= w0:
            continue
        crop = xt[bid[r], :, h0:h1, w0:w1]                                                # [C, h, w]
        hh = torch.arange(h0, h1, device=xt.device)
        ww = torch.arange(w0, w1, device=xt.device)
        mh = (hh[None] >= hs[r][:, None]) & (hh[None] < he[r][:, None])                    # [ph, h]
        mw = (ww[None] >= ws[r][:, None]) & (ww[None] < we[r][:, None])                    # [pw, w]
        m = mh[:, None, :, None] & mw[None, :, None, :]                                    # [ph, pw, h, w]
        vals = torch.where(m[None], crop[:, None, None], torch.full((), neg, dtype=xt.dtype, device=xt.device))
        o = vals.amax((-2, -1))
        empty = ~m.flatten(-2).any(-1)
        out[r] = torch.where(empty[None], torch.zeros_like(o), o)
    return _w(out)


def psroi_pool(x, boxes, boxes_num, output_size, spatial_scale=1.0, name=None):
    """Position-sensitive RoI average pooling: bin (i, j) of output channel k reads input channel
    (k * ph + i) * pw + j -> [R, C / (ph * pw), ph, pw]."""
    xt, bt = _t(x), _t(boxes)
    ph, pw = _pair(output_size)
    n, c, H, W = xt.shape
    if c % (ph * pw):
        raise ValueError("the channel of input X should be divisible by pooled_height * pooled_width")
    oc = c // (ph * pw)
    R = bt.shape[0]
    if R == 0:
        return _w(xt.new_zeros(0, oc, ph, pw))
    bid = _roi_batch_ids(boxes_num, R, n, xt.device)
    dt = xt.dtype
    rb = torch.round(bt.to(dt))
    x1, y1 = rb[:, 0] * spatial_scale, rb[:, 1] * spatial_scale
    x2, y2 = (rb[:, 2] + 1) * spatial_scale, (rb[:, 3] + 1) * spatial_scale
    rh = (y2 - y1).clamp_min(0.1)
    rw = (x2 - x1).clamp_min(0.1)
    bh, bw = rh / ph, rw / pw
    ar_h = torch.arange(ph, device=xt.device, dtype=dt)
    ar_w = torch.arange(pw, device=xt.device, dtype=dt)
    hs = torch.floor(ar_h[None] * bh[:, None] + y1[:, None]).long().clamp(0, H)
    he = torch.ceil((ar_h[None] + 1) * bh[:, None] + y1[:, None]).long().clamp(0, H)
    ws = torch.floor(ar_w[None] * bw[:, None] + x1[:, None]).long().clamp(0, W)
    we = torch.ceil((ar_w[None] + 1) * bw[:, None] + x1[:, None]).long().clamp(0, W)
    outs = []
    for r in range(R):
        h0, h1 = int(hs[r].min()), max(int(he[r].max()), int(hs[r].min()) + 1)
        w0, w1 = int(ws[r].min()), max(int(we[r].max()), int(ws[r].min()) + 1)
        h1, w1 = min(h1, H), min(w1, W)
        hh = torch.arange(h0, h1, device=xt.device)
        ww = torch.arange(w0, w1, device=xt.device)
        mh = ((hh[None] >= hs[r][:, None]) & (hh[None] < he[r][:, None])).to(dt)          # [ph, h]
        mw = ((ww[None] >= ws[r][:, None]) & (ww[None] < we[r][:, None])).to(dt)          # [pw, w]
        feat = xt[bid[r], :, h0:h1, w0:w1].reshape(oc, ph, pw, h1 - h0, w1 - w0)
        ssum = torch.einsum("kijhw,ih,jw->kij", feat, mh, mw)
        area = ((he[r] - hs[r]).clamp_min(0)[:, None] * (we[r] - ws[r]).clamp_min(0)[None]).to(dt)
        outs.append(torch.where(area[None] > 0, ssum / area.clamp_min(1)[None], torch.zeros_like(ssum)))
    out = torch.stack(outs)
    return _w(out)


class RoIAlign(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self._output_size, self._spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num, aligned=True):
        return roi_align(x, boxes, boxes_num, self._output_size, self._spatial_scale, aligned=aligned)


class RoIPool(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self._output_size, self._spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return roi_pool(x, boxes, boxes_num, self._output_size, self._spatial_scale)


class PSRoIPool(Layer):
    def __init__(self, output_size, spatial_scale=1.0):
        super().__init__()
        self.output_size, self.spatial_scale = output_size, spatial_scale

    def forward(self, x, boxes, boxes_num):
        return psroi_pool(x, boxes, boxes_num, self.output_size, self.spatial_scale)


# ================================================================================================ NMS family
def _iou_matrix(b, offset=0.0):
    x1, y1, x2, y2 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    area = ((x2 - x1 + offset).clamp_min(0) * (y2 - y1 + offset).clamp_min(0))
    iw = (torch.minimum(x2[:, None], x2[None]) - torch.maximum(x1[:, None], x1[None]) + offset).clamp_min(0)
    ih = (torch.minimum(y2[:, None], y2[None]) - torch.maximum(y1[:, None], y1[None]) + offset).clamp_min(0)
    inter = iw * ih
    return inter / (area[:, None] + area[None] - inter).clamp_min(1e-12)


def _greedy(iou, thresh):
    """Greedy suppression over boxes already in priority order: keep i unless a kept j < i overlaps > thresh."""
    n = iou.shape[0]
    over = (iou > thresh).cpu().numpy()
    removed = np.zeros(n, dtype=bool)
    keep = []
    for i in range(n):
        if removed[i]:
            continue
        keep.append(i)
        removed |= over[i]
    return keep


def _nms_sorted(boxes, thresh):
    keep = _greedy(_iou_matrix(boxes), thresh)
    return torch.as_tensor(keep, dtype=torch.long, device=boxes.device)


def nms(boxes, iou_threshold=0.3, scores=None, category_idxs=None, categories=None, top_k=None):
    """Non-maximum suppression -> int64 indices of kept boxes (by descending score when ``scores`` is given;
    per category when ``category_idxs`` / ``categories`` are)."""
    b = _t(boxes)
    if scores is None:
        return _w(_nms_sorted(b, iou_threshold))
    s = _t(scores)
    if category_idxs is None:
        order = torch.argsort(s, descending=True)
        return _w(order[_nms_sorted(b[order], iou_threshold)])
    if top_k is not None and top_k > s.shape[0]:
        raise ValueError("top_k should be smaller equal than the number of boxes")
    if categories is None:
        raise ValueError("if category_idxs is given, categories which is a list of unique id of all categories is "
                         "necessary")
    cidx = _t(category_idxs)
    mask = torch.zeros(s.shape[0], dtype=torch.bool, device=s.device)
    for cat in categories:
        idx = (cidx == int(cat)).nonzero(as_tuple=True)[0]
        if idx.numel() == 0:
            continue
        order = torch.argsort(s[idx], descending=True)
        kept = idx[order[_nms_sorted(b[idx][order], iou_threshold)]]
        mask[kept] = True
    keep = mask.nonzero(as_tuple=True)[0]
    order = torch.argsort(s[keep], descending=True)
    if top_k is not None:
        order = order[:min(top_k, keep.numel())]
    return _w(keep[order])


def matrix_nms(bboxes, scores, score_threshold, post_threshold, nms_top_k, keep_top_k, use_gaussian=False,
               gaussian_sigma=2.0, background_label=0, normalized=True, return_index=False, return_rois_num=True,
               name=None):
    """Matrix NMS (SOLOv2): per class, scores decay by the worst IoU ratio against higher-scored boxes instead
    of hard suppression -> (out [K, 6] = (label, score, x1, y1, x2, y2), rois_num [N] | None, index [K, 1] |
    None)."""
    bb, sc = _t(bboxes), _t(scores)
    N, C, M = sc.shape
    offset = 0.0 if normalized else 1.0
    outs, idxs, nums = [], [], []
    for i in range(N):
        dets = []   # (score, class, box index)
        for c in range(C):
            if c == background_label:
                continue
            s = sc[i, c]
            cand = (s > score_threshold).nonzero(as_tuple=True)[0]
            if cand.numel() == 0:
                continue
            order = cand[torch.argsort(s[cand], descending=True, stable=True)]
            if nms_top_k > -1:
                order = order[:nms_top_k]
            boxes = bb[i, order]
            iou = _iou_matrix(boxes, offset)
            # only pairs (i, j) with j ranked above i count
            iou = torch.triu(iou, diagonal=1).t()            # iou[i, j] for j < i
            iou_max = iou.amax(1)                            # max IoU of each box with higher-ranked ones
            if use_gaussian:
                decay = torch.exp((iou_max[None, :] ** 2 - iou ** 2) * gaussian_sigma)
            else:
                decay = (1 - iou) / (1 - iou_max[None, :])
            lower = torch.tril(torch.ones_like(iou, dtype=torch.bool), diagonal=-1)
            decay = torch.where(lower, decay, torch.ones_like(decay))
            min_decay = decay.amin(1)
            ds = min_decay * s[order]
            ds[0] = s[order[0]]
            keepm = ds > post_threshold
            for sc_v, bi in zip(ds[keepm].tolist(), order[keepm].tolist()):
                dets.append((sc_v, c, bi))
        # stable order: by score (class scan order breaks ties, as the reference's partial sort of appended dets)
        dets_sorted = sorted(range(len(dets)), key=lambda k: -dets[k][0])
        if keep_top_k > -1:
            dets_sorted = dets_sorted[:keep_top_k]
        for k in dets_sorted:
            sv, cl, bi = dets[k]
            outs.append(torch.cat([torch.tensor([float(cl), sv], dtype=bb.dtype, device=bb.device), bb[i, bi]]))
            idxs.append(i * M + bi)
        nums.append(len(dets_sorted))
    out = torch.stack(outs) if outs else bb.new_zeros(0, bb.shape[-1] + 2)
    index = torch.tensor(idxs, dtype=torch.int32, device=bb.device).view(-1, 1)
    rois_num = torch.tensor(nums, dtype=torch.int32, device=bb.device)
    return _w(out), (_w(rois_num) if return_rois_num else None), (_w(index) if return_index else None)


_BBOX_CLIP = math.log(1000.0 / 16.0)


def _detection_nms(boxes, scores, thresh, eta, pixel_offset):
    order = torch.argsort(scores, descending=True, stable=True)
    iou = _iou_matrix(boxes[order], 1.0 if pixel_offset else 0.0).cpu().numpy()
    keep = []
    adaptive = thresh
    for i in range(order.numel()):
        ok = all(iou[i, j] <= adaptive for j in keep)
        if ok:
            keep.append(i)
            if eta < 1 and adaptive > 0.5:
                adaptive *= eta
    return order[torch.as_tensor(keep, dtype=torch.long, device=boxes.device)]


def generate_proposals(scores, bbox_deltas, img_size, anchors, variances, pre_nms_top_n=6000, post_nms_top_n=1000,
                       nms_thresh=0.5, min_size=0.1, eta=1.0, pixel_offset=False, return_rois_num=False, name=None):
    """RPN proposals: decode anchors with the deltas, clip to the image, drop small boxes, NMS per image ->
    (rois [K, 4], probs [K, 1], rois_num [N] | None)."""
    s, d, im = _t(scores), _t(bbox_deltas), _t(img_size)
    an, var = _t(anchors).reshape(-1, 4), _t(variances).reshape(-1, 4)
    N = s.shape[0]
    s = s.permute(0, 2, 3, 1).reshape(N, -1)
    d = d.permute(0, 2, 3, 1).reshape(N, -1, 4)
    off = 1.0 if pixel_offset else 0.0
    rois, probs, nums = [], [], []
    for i in range(N):
        sc = s[i]
        if 0 < pre_nms_top_n < sc.numel():
            idx = torch.topk(sc, pre_nms_top_n).indices
        else:
            idx = torch.argsort(sc, descending=True)
        a, dl, v = an[idx], d[i, idx], var[idx]
        aw = a[:, 2] - a[:, 0] + off
        ah = a[:, 3] - a[:, 1] + off
        acx, acy = a[:, 0] + 0.5 * aw, a[:, 1] + 0.5 * ah
        cx = v[:, 0] * dl[:, 0] * aw + acx
        cy = v[:, 1] * dl[:, 1] * ah + acy
        bw = torch.exp(torch.clamp(v[:, 2] * dl[:, 2], max=_BBOX_CLIP)) * aw
        bh = torch.exp(torch.clamp(v[:, 3] * dl[:, 3], max=_BBOX_CLIP)) * ah
        prop = torch.stack([cx - bw / 2, cy - bh / 2, cx + bw / 2 - off, cy + bh / 2 - off], -1)
        h, w = float(im[i, 0]), float(im[i, 1])
        prop = torch.stack([prop[:, 0].clamp(0, w - off), prop[:, 1].clamp(0, h - off),
                            prop[:, 2].clamp(0, w - off), prop[:, 3].clamp(0, h - off)], -1)
        ms = max(min_size, 1.0)
        ws = prop[:, 2] - prop[:, 0] + off
        hs = prop[:, 3] - prop[:, 1] + off
        keep = (ws >= ms) & (hs >= ms)
        if pixel_offset:
            keep &= (prop[:, 0] + ws / 2 <= w) & (prop[:, 1] + hs / 2 <= h)
        kidx = keep.nonzero(as_tuple=True)[0]
        if kidx.numel() == 0:
            rois.append(prop.new_zeros(1, 4))
            probs.append(prop.new_zeros(1, 1))
            nums.append(1)
            continue
        bsel, ssel = prop[kidx], sc[idx][kidx]
        if nms_thresh > 0:
            k2 = _detection_nms(bsel, ssel, nms_thresh, eta, pixel_offset)
            if 0 < post_nms_top_n < k2.numel():
                k2 = k2[:post_nms_top_n]
            bsel, ssel = bsel[k2], ssel[k2]
        rois.append(bsel)
        probs.append(ssel.view(-1, 1))
        nums.append(bsel.shape[0])
    out_rois, out_probs = torch.cat(rois), torch.cat(probs)
    rn = torch.tensor(nums, dtype=torch.int32, device=out_rois.device)
    return _w(out_rois), _w(out_probs), (_w(rn) if return_rois_num else None)


def distribute_fpn_proposals(fpn_rois, min_level, max_level, refer_level, refer_scale, pixel_offset=False,
                             rois_num=None, name=None):
    """Assign each RoI to an FPN level by sqrt(area) -> (per-level rois, restore index [R, 1], per-level rois
    num | None)."""
    r = _t(fpn_rois)
    R = r.shape[0]
    off = 1.0 if pixel_offset else 0.0
    w = r[:, 2] - r[:, 0] + off
    h = r[:, 3] - r[:, 1] + off
    area = torch.where((r[:, 2] < r[:, 0]) | (r[:, 3] < r[:, 1]), torch.zeros_like(w), w * h)
    lvl = torch.floor(torch.log2(torch.sqrt(area) / refer_scale + 1e-6) + refer_level).long()
    lvl = lvl.clamp(min_level, max_level)
    if rois_num is not None:
        bid = torch.repeat_interleave(torch.arange(_t(rois_num).numel(), device=r.device),
                                      _t(rois_num).to(r.device).long())
        nb = _t(rois_num).numel()
    else:
        bid = torch.zeros(R, dtype=torch.long, device=r.device)
        nb = 1
    outs, per_level_nums, order_all = [], [], []
    for L in range(min_level, max_level + 1):
        sel = (lvl == L).nonzero(as_tuple=True)[0]            # image-major, original order within an image
        sel = sel[torch.argsort(bid[sel], stable=True)]
        outs.append(_w(r[sel]))
        order_all.append(sel)
        per_level_nums.append(_w(torch.bincount(bid[sel], minlength=nb).to(torch.int32)))
    cat = torch.cat(order_all)
    restore = torch.empty(R, dtype=torch.int32, device=r.device)
    restore[cat] = torch.arange(R, dtype=torch.int32, device=r.device)
    return outs, _w(restore.view(-1, 1)), (per_level_nums if rois_num is not None else None)


# ================================================================================================ deformable conv
def deform_conv2d(x, offset, weight, bias=None, stride=1, padding=0, dilation=1, deformable_groups=1, groups=1,
                  mask=None, name=None):
    """Deformable convolution v1 (``mask`` None) / v2: each kernel tap samples the input bilinearly at its
    learned offset (zero outside the image), optionally modulated by ``mask``, then a grouped GEMM."""
    xt, ot, wt = _t(x), _t(offset), _t(weight)
    bt = _t(bias)
    mt = _t(mask)
    sh, sw = _pair(stride)
    ph, pw = _pair(padding)
    dh, dw = _pair(dilation)
    N, C, H, W = xt.shape
    Co, Cg, kh, kw = wt.shape
    Ho = (H + 2 * ph - (dh * (kh - 1) + 1)) // sh + 1
    Wo = (W + 2 * pw - (dw * (kw - 1) + 1)) // sw + 1
    K = kh * kw
    dg = deformable_groups
    off = ot.view(N, dg, K, 2, Ho, Wo)
    ky = torch.arange(kh, device=xt.device, dtype=xt.dtype).repeat_interleave(kw) * dh       # [K]
    kx = torch.arange(kw, device=xt.device, dtype=xt.dtype).repeat(kh) * dw
    oy = torch.arange(Ho, device=xt.device, dtype=xt.dtype) * sh - ph
    ox = torch.arange(Wo, device=xt.device, dtype=xt.dtype) * sw - pw
    py = oy.view(1, 1, 1, Ho, 1) + ky.view(1, 1, K, 1, 1) + off[:, :, :, 0]                 # [N, dg, K, Ho, Wo]
    px = ox.view(1, 1, 1, 1, Wo) + kx.view(1, 1, K, 1, 1) + off[:, :, :, 1]
    valid = (py > -1) & (py < H) & (px > -1) & (px < W)
    y0 = torch.floor(py)
    x0 = torch.floor(px)
    ly, lx = py - y0, px - x0
    y0, x0 = y0.long(), x0.long()
    xg = xt.view(N, dg, C // dg, H * W)

    def corner(yy, xx, wgt):
        inb = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W) & valid
        idx = (yy.clamp(0, H - 1) * W + xx.clamp(0, W - 1)).view(N, dg, 1, -1).expand(-1, -1, C // dg, -1)
        v = torch.gather(xg, 3, idx).view(N, dg, C // dg, K, Ho, Wo)
        return v * (wgt * inb.to(xt.dtype)).unsqueeze(2)

    cols = (corner(y0, x0, (1 - ly) * (1 - lx)) + corner(y0, x0 + 1, (1 - ly) * lx) +
            corner(y0 + 1, x0, ly * (1 - lx)) + corner(y0 + 1, x0 + 1, ly * lx))          # [N, dg, C/dg, K, Ho, Wo]
    if mt is not None:
        cols = cols * mt.view(N, dg, 1, K, Ho, Wo)
    cols = cols.reshape(N, groups, C // groups * K, Ho * Wo)
    wg = wt.reshape(groups, Co // groups, Cg * K)
    out = torch.einsum("gok,ngkl->ngol", wg, cols).reshape(N, Co, Ho, Wo)
    if bt is not None:
        out = out + bt.view(1, -1, 1, 1)
    return _w(out)


class DeformConv2D(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, deformable_groups=1,
                 groups=1, weight_attr=None, bias_attr=None):
        super().__init__()
        kh, kw = _pair(kernel_size)
        self._stride, self._padding, self._dilation = stride, padding, dilation
        self._deformable_groups, self._groups = deformable_groups, groups
        fan_in = in_channels // groups * kh * kw
        from ..nn import initializer as I

        std = (2.0 / fan_in) ** 0.5
        self.weight = self.create_parameter([out_channels, in_channels // groups, kh, kw], attr=weight_attr,
                                            default_initializer=I.Normal(0.0, std))
        self.bias = None if bias_attr is False else self.create_parameter([out_channels], attr=bias_attr,
                                                                          is_bias=True)

    def forward(self, x, offset, mask=None):
        return deform_conv2d(x, offset, self.weight, self.bias, self._stride, self._padding, self._dilation,
                             self._deformable_groups, self._groups, mask)


# ================================================================================================ IO
def read_file(filename, name=None):
    """File bytes -> uint8 tensor [num_bytes]."""
    with open(filename, "rb") as f:
        data = np.frombuffer(f.read(), dtype=np.uint8).copy()
    return _w(torch.from_numpy(data))


def decode_jpeg(x, mode="unchanged", name=None):
    """JPEG bytes (uint8 tensor) -> CHW uint8 image; ``mode`` 'unchanged' | 'gray' | 'rgb'."""
    import io as _io

    from PIL import Image

    buf = _t(x).detach().cpu().numpy().astype(np.uint8).tobytes()
    img = Image.open(_io.BytesIO(buf))
    if mode == "gray":
        img = img.convert("L")
    elif mode == "rgb":
        img = img.convert("RGB")
    arr = np.asarray(img)
    if arr.ndim == 2:
        arr = arr[None]
    else:
        arr = arr.transpose(2, 0, 1)
    return _w(torch.from_numpy(np.ascontiguousarray(arr)))


# ================================================================================================ blocks
class ConvNormActivation(Layer):
    """Conv2D -> norm -> activation (reference ConvNormActivation, a Sequential)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=None, groups=1, norm_layer=None,
                 activation_layer=None, dilation=1, bias=None):
        super().__init__()
        from .. import nn

        norm_layer = nn.BatchNorm2D if norm_layer is None else norm_layer
        activation_layer = nn.ReLU if activation_layer is None else activation_layer
        if padding is None:
            padding = (kernel_size - 1) // 2 * dilation
        if bias is None:
            bias = norm_layer is None
        layers = [nn.Conv2D(in_channels, out_channels, kernel_size, stride, padding, dilation=dilation,
                            groups=groups, bias_attr=None if bias else False)]
        if norm_layer is not None:
            layers.append(norm_layer(out_channels))
        if activation_layer is not None:
            layers.append(activation_layer())
        self.layers = nn.Sequential(*layers)

    def forward(self, x):
        return self.layers(x)
