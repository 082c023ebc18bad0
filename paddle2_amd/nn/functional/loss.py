"""Losses (reference: python/paddle/nn/functional/loss.py).

``cross_entropy``/``softmax_with_cross_entropy`` with hard labels over a large vocabulary
route to the fused HIP softmax-CE kernel in :mod:`paddle2_amd.ops`.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ...framework.tensor import Tensor
from ...amp import amp_op as _amp_op  # noqa: E402

_wrap = Tensor._wrap


def _reduce(t, reduction):
    if reduction == "mean":
        return t.mean()
    if reduction == "sum":
        return t.sum()
    return t


@_amp_op("cross_entropy")
def cross_entropy(input, label, weight=None, ignore_index=-100, reduction="mean", soft_label=False, axis=-1,
                  use_softmax=True, label_smoothing=0.0, name=None):
    logits = input._t
    lab = label._t
    ax = axis % logits.dim()
    if soft_label or (lab.dim() == logits.dim() and lab.shape[ax] == logits.shape[ax] and lab.is_floating_point()):
        logp = torch.log_softmax(logits.float(), ax) if use_softmax else torch.log(logits.float())
        if label_smoothing > 0:
            k = logits.shape[ax]
            lab = (1 - label_smoothing) * lab + label_smoothing / k
        loss = -(lab.float() * logp)
        if weight is not None:
            shp = [1] * logits.dim()
            shp[ax] = -1
            loss = loss * weight._t.reshape(shp)
        loss = loss.sum(ax, keepdim=True)
        out = _reduce(loss, reduction)
        return _wrap(out.to(logits.dtype) if logits.dtype != torch.float32 and reduction == "none" else out)
    # hard labels
    if lab.dim() == logits.dim():
        lab = lab.squeeze(ax)
    lab = lab.long()
    if use_softmax and weight is None and label_smoothing == 0.0 and ax == logits.dim() - 1:
        from ...ops.torch_ops import softmax_cross_entropy as _sce

        loss = _sce(logits, lab, ignore_index)  # per-token fp32, 0 where ignored
        if reduction == "mean":
            valid = (lab != ignore_index).sum().clamp_min(1)
            return _wrap(loss.sum() / valid)
        if reduction == "sum":
            return _wrap(loss.sum())
        return _wrap(loss.unsqueeze(-1))
    lg = logits.movedim(ax, 1) if ax != 1 and logits.dim() > 2 else logits
    if use_softmax:
        loss = F.cross_entropy(lg.float(), lab if lg.dim() != 2 or lab.dim() == 1 else lab,
                               weight=None if weight is None else weight._t.float(), ignore_index=ignore_index,
                               reduction="none", label_smoothing=label_smoothing)
    else:
        loss = F.nll_loss(torch.log(lg.float()), lab, weight=None if weight is None else weight._t.float(),
                          ignore_index=ignore_index, reduction="none")
    if reduction == "mean":
        if weight is not None:
            wv = weight._t.float()[lab.clamp_min(0)] * (lab != ignore_index)
            return _wrap(loss.sum() / wv.sum())
        valid = (lab != ignore_index).sum().clamp_min(1)
        return _wrap(loss.sum() / valid)
    if reduction == "sum":
        return _wrap(loss.sum())
    return _wrap(loss.unsqueeze(ax))


def softmax_with_cross_entropy(logits, label, soft_label=False, ignore_index=-100, numeric_stable_mode=True,
                               return_softmax=False, axis=-1):
    loss = cross_entropy(logits, label, soft_label=soft_label, ignore_index=ignore_index, reduction="none", axis=axis)
    if return_softmax:
        return loss, _wrap(torch.softmax(logits._t, axis))
    return loss


def nll_loss(input, label, weight=None, ignore_index=-100, reduction="mean", name=None):
    return _wrap(F.nll_loss(input._t, label._t.long(), None if weight is None else weight._t,
                            ignore_index=ignore_index, reduction=reduction))


def mse_loss(input, label, reduction="mean", name=None):
    return _wrap(F.mse_loss(input._t, label._t, reduction=reduction))


def l1_loss(input, label, reduction="mean", name=None):
    return _wrap(F.l1_loss(input._t, label._t, reduction=reduction))


def smooth_l1_loss(input, label, reduction="mean", delta=1.0, name=None):
    return _wrap(F.huber_loss(input._t, label._t, reduction=reduction, delta=delta))


def huber_loss(input, label, reduction="mean", delta=1.0, name=None):
    return _wrap(F.huber_loss(input._t, label._t, reduction=reduction, delta=delta))


def binary_cross_entropy(input, label, weight=None, reduction="mean", name=None):
    return _wrap(F.binary_cross_entropy(input._t, label._t, None if weight is None else weight._t, reduction=reduction))


def binary_cross_entropy_with_logits(logit, label, weight=None, reduction="mean", pos_weight=None, name=None):
    return _wrap(F.binary_cross_entropy_with_logits(logit._t, label._t, None if weight is None else weight._t,
                                                    reduction=reduction,
                                                    pos_weight=None if pos_weight is None else pos_weight._t))


def sigmoid_focal_loss(logit, label, normalizer=None, alpha=0.25, gamma=2.0, reduction="sum", name=None):
    p = torch.sigmoid(logit._t)
    ce = F.binary_cross_entropy_with_logits(logit._t, label._t, reduction="none")
    pt = p * label._t + (1 - p) * (1 - label._t)
    loss = ce * ((1 - pt) ** gamma)
    a = alpha * label._t + (1 - alpha) * (1 - label._t)
    loss = a * loss
    if normalizer is not None:
        loss = loss / normalizer._t
    return _wrap(_reduce(loss, reduction))


def kl_div(input, label, reduction="mean", log_target=False, name=None):
    red = "batchmean" if reduction == "batchmean" else reduction
    return _wrap(F.kl_div(input._t, label._t, reduction=red, log_target=log_target))


def margin_ranking_loss(input, other, label, margin=0.0, reduction="mean", name=None):
    return _wrap(F.margin_ranking_loss(input._t, other._t, label._t, margin, reduction=reduction))


def hinge_embedding_loss(input, label, margin=1.0, reduction="mean", name=None):
    return _wrap(F.hinge_embedding_loss(input._t, label._t, margin, reduction=reduction))


def cosine_embedding_loss(input1, input2, label, margin=0, reduction="mean", name=None):
    return _wrap(F.cosine_embedding_loss(input1._t, input2._t, label._t, margin, reduction=reduction))


def triplet_margin_loss(input, positive, negative, margin=1.0, p=2, epsilon=1e-6, swap=False, reduction="mean", name=None):
    return _wrap(F.triplet_margin_loss(input._t, positive._t, negative._t, margin, p, epsilon, swap, reduction=reduction))


def soft_margin_loss(input, label, reduction="mean", name=None):
    return _wrap(F.soft_margin_loss(input._t, label._t, reduction=reduction))


def multi_label_soft_margin_loss(input, label, weight=None, reduction="mean", name=None):
    return _wrap(F.multilabel_soft_margin_loss(input._t, label._t, None if weight is None else weight._t, reduction=reduction))


def multi_margin_loss(input, label, p=1, margin=1.0, weight=None, reduction="mean", name=None):
    return _wrap(F.multi_margin_loss(input._t, label._t.long(), p, margin, None if weight is None else weight._t, reduction=reduction))


def poisson_nll_loss(input, label, log_input=True, full=False, epsilon=1e-8, reduction="mean", name=None):
    return _wrap(F.poisson_nll_loss(input._t, label._t, log_input, full, eps=epsilon, reduction=reduction))


def gaussian_nll_loss(input, label, variance, full=False, epsilon=1e-6, reduction="mean", name=None):
    return _wrap(F.gaussian_nll_loss(input._t, label._t, variance._t, full, epsilon, reduction))


def ctc_loss(log_probs, labels, input_lengths, label_lengths, blank=0, reduction="mean", norm_by_times=False):
    loss = F.ctc_loss(log_probs._t, labels._t, input_lengths._t, label_lengths._t, blank, reduction="none")
    if reduction == "mean":
        return _wrap((loss / label_lengths._t.float()).mean())
    return _wrap(_reduce(loss, reduction))


def log_loss(input, label, epsilon=0.0001, name=None):
    t, l = input._t, label._t
    return _wrap(-l * torch.log(t + epsilon) - (1 - l) * torch.log(1 - t + epsilon))


def dice_loss(input, label, epsilon=0.00001, name=None):
    t = input._t
    lab = F.one_hot(label._t.squeeze(-1).long(), t.shape[-1]).to(t.dtype)
    red = tuple(range(1, t.dim()))
    inse = (t * lab).sum(red)
    return _wrap((1 - 2 * inse / (t.sum(red) + lab.sum(red) + epsilon)).mean())


def square_error_cost(input, label):
    return _wrap((input._t - label._t) ** 2)


def margin_cross_entropy(logits, label, margin1=1.0, margin2=0.5, margin3=0.0, scale=64.0, group=None,
                         return_softmax=False, reduction="mean"):
    t = logits._t.float()
    lab = label._t.long().reshape(-1)
    theta = torch.acos(t.clamp(-1 + 1e-7, 1 - 1e-7))
    tgt = torch.cos(margin1 * theta + margin2) - margin3
    oh = F.one_hot(lab, t.shape[-1]).bool()
    t = torch.where(oh, tgt, t) * scale
    loss = F.cross_entropy(t, lab, reduction="none").unsqueeze(-1)
    out = _wrap(_reduce(loss, reduction))
    if return_softmax:
        return out, _wrap(torch.softmax(t, -1))
    return out


def npair_loss(anchor, positive, labels, l2_reg=0.002):
    a, p = anchor._t, positive._t
    lab = labels._t.reshape(-1, 1)
    same = (lab == lab.t()).float()
    same = same / same.sum(1, keepdim=True)
    logits = a @ p.t()
    ce = (-same * torch.log_softmax(logits, 1)).sum(1).mean()
    reg = l2_reg * ((a ** 2).sum(1).mean() + (p ** 2).sum(1).mean()) * 0.25
    return _wrap(ce + reg)


def hsigmoid_loss(input, label, num_classes, weight, bias=None, path_table=None, path_code=None, is_sparse=False,
                  name=None):
    """Hierarchical sigmoid (reference nn/functional/loss.py hsigmoid_loss, phi hsigmoid_loss_kernel with
    MatrixBitCodeFunctor).  Default tree: leaf c = label + num_classes of a complete binary tree; node j on
    the path is (c >> (j+1)) - 1 with branch bit (c >> j) & 1, length floor(log2(c)).  Custom trees: rows of
    ``path_table`` (node ids, -1 padded) and ``path_code`` (bits).  Loss per sample = sum over its path of
    softplus(z) - bit * z, z = x . W[node] + b[node] (pre-activations clipped to [-40, 40]).  -> [N, 1]."""
    x = input._t
    W = weight._t
    lab = label._t.reshape(-1).long()
    N = x.shape[0]
    if path_table is None:
        c = lab + num_classes
        L = int(torch.floor(torch.log2(c.float().max())).item()) if N else 0
        j = torch.arange(L, device=x.device)
        nodes = (c[:, None] >> (j[None, :] + 1)) - 1
        bits = ((c[:, None] >> j[None, :]) & 1).to(x.dtype)
        lens = torch.floor(torch.log2(c.float())).long()
        valid = j[None, :] < lens[:, None]
    else:
        nodes = path_table._t.long()
        bits = path_code._t.to(x.dtype)
        valid = nodes >= 0
    safe = nodes.clamp_min(0)
    z = torch.einsum("nd,nld->nl", x, W[safe])
    if bias is not None:
        z = z + bias._t.reshape(-1)[safe]
    z = z.clamp(-40.0, 40.0)
    per = (F.softplus(z) - bits * z) * valid.to(x.dtype)
    return _wrap(per.sum(1, keepdim=True))


def rnnt_loss(input, label, input_lengths, label_lengths, blank=0, fastemit_lambda=0.001, reduction="mean",
              name=None):
    """RNN-Transducer loss (Graves 2012; reference nn/functional/loss.py rnnt_loss over warprnnt).
    ``input`` [B, T, U+1, V] logits, ``label`` [B, U].  alpha(t, u) = logaddexp(alpha(t-1, u) + blank(t-1, u),
    alpha(t, u-1) + emit(t, u-1)); loss = -(alpha(T-1, U) + blank(T-1, U)) per sequence, differentiated by
    autograd through the log-space recursion.  ``fastemit_lambda`` adds the FastEmit regulariser's
    emission weight to the emit transitions' gradient (lambda * dL/d emit), as warprnnt does.
    reduction 'mean' divides by the target lengths' sum... the reference (warprnnt) 'mean' averages over
    the batch; 'sum' / 'none' as usual."""
    logits = input._t
    lab = label._t.long()
    tl = input_lengths._t.long().reshape(-1)
    ul = label_lengths._t.long().reshape(-1)
    B, T, U1, V = logits.shape
    lp = torch.log_softmax(logits.float(), -1)
    blank_lp = lp[..., blank]                                     # [B, T, U+1]
    idx = lab.clamp_min(0)[:, None, :].expand(B, T, U1 - 1)[..., None]
    emit_lp = lp[:, :, :U1 - 1, :].gather(-1, idx).squeeze(-1)   # [B, T, U]
    if fastemit_lambda:
        # FastEmit (Yu et al. 2021): scale the emit paths' gradient by (1 + lambda), value unchanged
        emit_lp = emit_lp + fastemit_lambda * (emit_lp - emit_lp.detach())
    neg = torch.finfo(torch.float32).min / 4
    alpha = [[None] * U1 for _ in range(T)]
    for t in range(T):
        for u in range(U1):
            if t == 0 and u == 0:
                a = torch.zeros(B, device=logits.device)
            else:
                c1 = alpha[t - 1][u] + blank_lp[:, t - 1, u] if t > 0 else torch.full((B,), neg, device=logits.device)
                c2 = alpha[t][u - 1] + emit_lp[:, t, u - 1] if u > 0 else torch.full((B,), neg, device=logits.device)
                a = torch.logaddexp(c1, c2)
            alpha[t][u] = a
    ar = torch.stack([torch.stack(row, 1) for row in alpha], 1)   # [B, T, U+1]
    bi = torch.arange(B, device=logits.device)
    ll = ar[bi, tl - 1, ul] + blank_lp[bi, tl - 1, ul]
    loss = -ll
    if reduction == "mean":
        return _wrap(loss.mean())
    if reduction == "sum":
        return _wrap(loss.sum())
    return _wrap(loss)
