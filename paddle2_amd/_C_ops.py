"""``paddle._C_ops`` — positional, Paddle-signature op entry points over the single-backend op table.

Reference: python/paddle/_C_ops.py (generated ``eager_api_<op>`` bindings, python_c_gen.py:113) with
argument orders from paddle/phi/ops/yaml/ops.yaml (e.g. ``rms_norm``, ``flash_attn`` :1945,
``swiglu`` :4780, ``adamw_`` :118), fused_ops.yaml (``fused_rotary_position_embedding`` :409) and
inconsistent/dygraph_ops.yaml (``c_embedding`` :59).

Every name resolves through ``paddle2_amd.ops.registry``: the hot ops below are registered with the
HIP kernel that backs them on the MI355X (``native_kernel``); any other name falls back to the
public ``paddle.*`` / ``paddle.nn.functional.*`` function of the same name (so ``_C_ops.relu``,
``_C_ops.add`` ... work), and unknown names raise ``NotImplementedError``.
"""
from __future__ import annotations

import torch

from .framework.tensor import Tensor
from .ops import torch_ops as T
from .ops.registry import call, has_op, kernel_info, list_ops, register_op  # noqa: F401


def _t(x):
    return None if x is None else (x._t if isinstance(x, Tensor) else x)


def _w(t):
    return None if t is None else Tensor._wrap(t)


# ----------------------------------------------------------------------------- normalisation / act
@register_op("rms_norm", native_kernel="norm_fwd")
def _rms_norm(x, bias, residual, norm_weight, norm_bias, epsilon, begin_norm_axis, quant_scale=-1.0,
              quant_round_type=0, quant_max_bound=0.0, quant_min_bound=0.0):
    """RMSNorm (+bias, +residual add); returns (out, residual_out, inv_var)."""
    from .incubate.nn.functional import fused_rms_norm

    out, res = fused_rms_norm(x, norm_weight, norm_bias, epsilon, begin_norm_axis, bias, residual, quant_scale,
                              quant_round_type, quant_max_bound, quant_min_bound)
    src = res if res is not None else x
    h = _t(src).float()
    inv = torch.rsqrt(h.reshape(*h.shape[:begin_norm_axis], -1).pow(2).mean(-1) + epsilon)
    return out, res, _w(inv)


@register_op("layer_norm", native_kernel="norm_fwd")
def _layer_norm(x, scale, bias, epsilon=1e-5, begin_norm_axis=1):
    """LayerNorm over dims >= begin_norm_axis; returns (out, mean, variance)."""
    t = _t(x)
    lead = t.shape[:begin_norm_axis]
    t2 = t.reshape(*lead, -1)
    n = t2.shape[-1]
    w = _t(scale).reshape(-1) if scale is not None else torch.ones(n, dtype=t.dtype, device=t.device)
    b = _t(bias).reshape(-1) if bias is not None else torch.zeros(n, dtype=t.dtype, device=t.device)
    y = T.layer_norm(t2, w, b, epsilon)
    f = t2.float()
    return _w(y.reshape(t.shape)), _w(f.mean(-1).reshape(-1)), _w(f.var(-1, unbiased=False).reshape(-1))


@register_op("swiglu", native_kernel="swiglu_fwd")
def _swiglu(x, y=None):
    """silu(x) * y (y None: split x in half on the last dim)."""
    return _w(T.swiglu(_t(x), _t(y)))


@register_op("fused_rotary_position_embedding", native_kernel="rope")
def _rope(q, k=None, v=None, sin=None, cos=None, position_ids=None, use_neox_rotary_style=True, time_major=False,
          rotary_emb_base=10000.0):
    """RoPE on q/k/v; returns (out_q, out_k, out_v)."""
    from .incubate.nn.functional import fused_rotary_position_embedding

    return fused_rotary_position_embedding(q, k, v, sin, cos, position_ids, use_neox_rotary_style, time_major,
                                           rotary_emb_base)


# ----------------------------------------------------------------------------- attention
@register_op("flash_attn", native_kernel="flash_fwd")
def _flash_attn(q, k, v, fixed_seed_offset=None, attn_mask=None, dropout=0.0, causal=False, return_softmax=False,
                is_test=False, rng_name=""):
    """Flash attention [b, s, h, d]; returns (out, softmax, softmax_lse, seed_offset)."""
    from .nn.functional.attention import flash_attention, scaled_dot_product_attention

    if attn_mask is not None:
        out = scaled_dot_product_attention(q, k, v, attn_mask, dropout, causal, training=not is_test)
        return out, None, None, None
    out, sm = flash_attention(q, k, v, dropout, causal, return_softmax, fixed_seed_offset=fixed_seed_offset,
                              rng_name=rng_name, training=not is_test)
    return out, sm, None, fixed_seed_offset


@register_op("flash_attn_unpadded", native_kernel="flash_fwd_ext")
def _flash_attn_unpadded(q, k, v, cu_seqlens_q, cu_seqlens_k, fixed_seed_offset=None, attn_mask=None,
                         max_seqlen_q=0, max_seqlen_k=0, scale=None, dropout=0.0, causal=False, return_softmax=False,
                         is_test=False, rng_name=""):
    """Varlen flash attention over packed tokens; returns (out, softmax, softmax_lse, seed_offset)."""
    from .nn.functional.attention import flash_attn_unpadded

    if scale is None:
        scale = float(_t(q).shape[-1]) ** -0.5
    out, sm = flash_attn_unpadded(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, scale, dropout,
                                  causal, return_softmax, fixed_seed_offset=fixed_seed_offset, rng_name=rng_name,
                                  training=not is_test)
    return out, sm, None, fixed_seed_offset


@register_op("flashmask_attention", native_kernel="flash_fwd_ext")
def _flashmask(q, k, v, startend_row_indices, fixed_seed_offset=None, dropout=0.0, causal=False,
               return_softmax=False, is_test=False, rng_name=""):
    """FlashMask row-range sparse-mask attention; returns (out, softmax, softmax_lse, seed_offset)."""
    from .nn.functional.attention import flashmask_attention

    out = flashmask_attention(q, k, v, startend_row_indices, dropout=dropout, causal=causal,
                              fixed_seed_offset=fixed_seed_offset, rng_name=rng_name, training=not is_test)
    return out, None, None, fixed_seed_offset


# ----------------------------------------------------------------------------- GEMM / embedding / loss
@register_op("matmul")
def _matmul(x, y, transpose_x=False, transpose_y=False):
    """Batched GEMM with optional transposes (hipBLASLt through the layout-aware linear path)."""
    a, b = _t(x), _t(y)
    if transpose_x:
        a = a.transpose(-1, -2)
    if transpose_y:
        b = b.transpose(-1, -2)
    return _w(torch.matmul(a, b))


@register_op("embedding", native_kernel="embed_fwd")
def _embedding(x, weight, padding_idx=-1, sparse=False):
    """Row gather from ``weight``; ``padding_idx`` rows get zero gradient."""
    from .nn import functional as F

    return F.embedding(x, weight, padding_idx=None if padding_idx is None or padding_idx < 0 else padding_idx)


@register_op("c_embedding", native_kernel="embed_fwd")
def _c_embedding(weight, x, start_index=0, vocab_size=-1):
    """Vocab-parallel lookup: ids outside [start, start + rows) give zero rows."""
    w, ids = _t(weight), _t(x)
    local = ids - start_index
    ok = (local >= 0) & (local < w.shape[0])
    out = torch.nn.functional.embedding(torch.where(ok, local, torch.zeros_like(local)), w)
    return _w(out * ok.unsqueeze(-1).to(out.dtype))


@register_op("cross_entropy_with_softmax", native_kernel="ce_stats")
def _ce_softmax(input, label, soft_label=False, use_softmax=True, numeric_stable_mode=True, ignore_index=-100,
                axis=-1):
    """Softmax + cross entropy; returns (softmax, loss) with loss keeping a trailing 1 dim."""
    x, lab = _t(input), _t(label)
    if axis not in (-1, x.dim() - 1):
        x = x.movedim(axis, -1)
        lab = lab.movedim(axis, -1)
    sm = torch.softmax(x.float(), -1) if use_softmax else x.float()
    if soft_label:
        loss = -(lab.float() * torch.log(sm.clamp_min(1e-30))).sum(-1, keepdim=True)
    else:
        li = lab.reshape(x.shape[:-1]).long()
        if use_softmax and x.dim() == 2:
            loss = T.softmax_cross_entropy(x, li, ignore_index).float().unsqueeze(-1)
        else:
            valid = li != ignore_index
            pick = torch.gather(sm, -1, torch.where(valid, li, torch.zeros_like(li)).unsqueeze(-1))
            loss = torch.where(valid.unsqueeze(-1), -torch.log(pick.clamp_min(1e-30)), torch.zeros_like(pick))
    if axis not in (-1, x.dim() - 1):
        sm, loss = sm.movedim(-1, axis), loss.movedim(-1, axis)
    return _w(sm.to(_t(input).dtype)), _w(loss)


# ----------------------------------------------------------------------------- optimizer / AMP kernels
@register_op("fused_softmax_mask", native_kernel="softmax_mask_fwd")
def _fused_softmax_mask(x, mask):
    return _w(T.softmax_mask(_t(x), _t(mask), causal=False))


@register_op("fused_softmax_mask_upper_triangle", native_kernel="softmax_mask_fwd")
def _fused_softmax_mask_ut(x):
    return _w(T.softmax_mask(_t(x), None, causal=True))


@register_op("fused_linear_param_grad_add", inplace=True)
def _fused_linear_param_grad_add(x, dout, dweight=None, dbias=None, multi_precision=True, has_bias=True):
    """dW += x^T dy (fp32 main_grad when multi_precision), db += sum(dy); returns (dweight, dbias).
    Reference: phi/kernels/fusion/gpu/fused_linear_param_grad_add_kernel.cu:282 (use_addto into MT=fp32).
    The product is accumulated straight into the fp32 main grad (native MFMA GEMM fp32 epilogue with
    beta = 1 on the GPU; fp32 addmm on the CPU) — never rounded to bf16 first, no [K, N] temporary."""
    xt, dy = _t(x), _t(dout)
    x2 = xt.reshape(-1, xt.shape[-1])
    d2 = dy.reshape(-1, dy.shape[-1])
    acc_dt = torch.float32 if multi_precision else dy.dtype
    fresh = dweight is None
    if fresh:
        dw = torch.empty(x2.shape[1], d2.shape[1], dtype=acc_dt, device=dy.device)
        dweight = _w(dw)
    dw = _t(dweight)
    if dw.dtype == torch.float32:
        if not x2.is_contiguous():
            x2 = x2.contiguous()
        if not d2.is_contiguous():
            d2 = d2.contiguous()
        T.wgrad_accumulate(dw, x2, d2, 0.0 if fresh else 1.0)
    elif fresh:
        torch.matmul(x2.t(), d2, out=dw)
    else:
        dw.addmm_(x2.t(), d2)
    if has_bias:
        db_new = d2.sum(0, dtype=torch.float32).to(acc_dt)
        if dbias is None:
            dbias = _w(db_new)
        else:
            _t(dbias).add_(db_new.to(_t(dbias).dtype))
    return dweight, dbias


@register_op("squared_l2_norm", native_kernel="sqnorm_mt")
def _sq_l2(x):
    """sum(x^2) as a 1-element fp32 tensor."""
    t = _t(x).float()
    return _w(torch.dot(t.reshape(-1), t.reshape(-1)).reshape(1))


@register_op("adamw_", native_kernel="adamw_mt", inplace=True)
def _adamw_(param, grad, learning_rate, moment1, moment2, beta1_pow, beta2_pow, master_param=None, skip_update=None,
            beta1=0.9, beta2=0.999, epsilon=1e-8, lr_ratio=1.0, coeff=0.01, with_decay=False, lazy_mode=False,
            min_row_size_to_use_multithread=1000, multi_precision=False, use_global_beta_pow=False):
    """In-place AdamW on one parameter (reference gpu/adamw_kernel.cu:35 semantics); returns the updated
    (param, moment1, moment2, beta1_pow, beta2_pow, master_param)."""
    p, g, m, v = _t(param), _t(grad).float(), _t(moment1), _t(moment2)
    b1p, b2p = _t(beta1_pow), _t(beta2_pow)
    if skip_update is not None and bool(_t(skip_update).reshape(-1)[0]):
        return param, moment1, moment2, beta1_pow, beta2_pow, master_param
    lr = float(_t(learning_rate).reshape(-1)[0]) if isinstance(learning_rate, Tensor) else float(learning_rate)
    lr *= lr_ratio
    tgt = _t(master_param) if (multi_precision and master_param is not None) else p
    with torch.no_grad():
        if with_decay:
            tgt.mul_(1.0 - lr * coeff)
        m.mul_(beta1).add_(g, alpha=1 - beta1)
        v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
        bc1 = 1 - b1p.float()
        bc2 = 1 - b2p.float()
        upd = (m / bc1) / ((v / bc2).sqrt() + epsilon)
        tgt.sub_((lr * upd).to(tgt.dtype))
        if tgt is not p:
            p.copy_(tgt)
        if not use_global_beta_pow:
            b1p.mul_(beta1)
            b2p.mul_(beta2)
    return param, moment1, moment2, beta1_pow, beta2_pow, master_param


@register_op("check_finite_and_unscale_", native_kernel="unscale_mt", inplace=True)
def _check_finite_and_unscale_(x, scale):
    """x_i /= scale in place; returns (x, found_inf[1] bool)."""
    inv = 1.0 / _t(scale).float()
    found = torch.zeros(1, dtype=torch.bool, device=_t(scale).device)
    with torch.no_grad():
        for t in x:
            tt = _t(t)
            found |= ~torch.isfinite(tt).all().reshape(1)
            tt.mul_(inv.to(tt.dtype))
    return x, _w(found)


@register_op("update_loss_scaling_", native_kernel="update_loss_scaling", inplace=True)
def _update_loss_scaling_(x, found_infinite, prev_loss_scaling, in_good_steps, in_bad_steps, incr_every_n_steps,
                          decr_every_n_nan_or_inf, incr_ratio, decr_ratio, stop_update=False):
    """Dynamic loss-scale state machine (reference gpu/amp_kernel.cu:85); zeroes x on overflow."""
    s, good, bad = _t(prev_loss_scaling), _t(in_good_steps), _t(in_bad_steps)
    with torch.no_grad():
        if bool(_t(found_infinite).reshape(-1)[0]):
            for t in x:
                _t(t).zero_()
            if not stop_update:
                good.zero_()
                bad.add_(1)
                if int(bad.reshape(-1)[0]) >= decr_every_n_nan_or_inf:
                    s.mul_(decr_ratio).clamp_(min=1.0)
                    bad.zero_()
        elif not stop_update:
            bad.zero_()
            good.add_(1)
            if int(good.reshape(-1)[0]) >= incr_every_n_steps:
                ns = s * incr_ratio
                if bool(torch.isfinite(ns).all()):
                    s.copy_(ns)
                good.zero_()
    return x, prev_loss_scaling, in_good_steps, in_bad_steps


# ----------------------------------------------------------------------------- fallback to the public API
def __getattr__(name):
    if has_op(name):
        from .ops.registry import select

        return select(name).fn
    import paddle2_amd as _p

    base = name[:-1] if name.endswith("_") and not name.endswith("__") else name
    for mod in (_p, _p.nn.functional, getattr(_p, "linalg", None), getattr(_p, "fft", None)):
        if mod is not None and hasattr(mod, base):
            fn = getattr(mod, base)
            if callable(fn):
                register_op(name, fn, inplace=base != name)
                return fn
    from .ops.op_schema import NATIVE, resolve

    fn = resolve(name)   # reference op names whose public API is spelled differently (ops/op_schema.py)
    if fn is not None:
        register_op(name, fn, native_kernel=NATIVE.get(name), inplace=name.endswith("_"))
        return fn
    raise AttributeError(f"paddle2_amd._C_ops has no op '{name}'")
