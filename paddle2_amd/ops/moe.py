"""Expert-grouped GEMMs for Mixture-of-Experts FFNs (reference: phi/kernels/fusion/cutlass/fused_moe_kernel.cu,
moe_gemm; python/paddle/incubate/nn/functional/fused_moe.py).

Rows (token, expert) assignments are sorted by expert ONCE on the device; ``goff`` [E + 1] int32 (device)
delimits every expert's slice.  On the MI355X each projection is ONE launch of the native MFMA GEMM in
grouped mode (csrc/kernels/gemm.hip pd_gemm_grouped) — forward, dgrad and the per-expert weight gradients
alike — and the per-expert row counts are never read by the host, so routing + experts + combine run
without a device->host sync.  CPU: a per-expert loop of the same math.
"""
from __future__ import annotations

import torch

from . import _native as N
from . import gemm as G
from . import torch_ops as T


def _native_ok(*ts):
    return all(t.device.type == "cuda" and t.dtype == torch.bfloat16 for t in ts) and N.use_native(ts[0])


def _slices(goff):
    o = goff.tolist()
    return [(e, o[e], o[e + 1]) for e in range(len(o) - 1) if o[e + 1] > o[e]]


class _GroupedLinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xs, w, goff, bias):
        ctx.native = _native_ok(xs, w) and xs.shape[1] % 8 == 0 and w.shape[2] % 8 == 0
        ctx.has_bias = bias is not None
        if ctx.native:
            xs, w = xs.contiguous(), w.contiguous()
            out = G.grouped_fwd(xs, w, goff, None if bias is None else bias.contiguous())
        else:
            out = torch.zeros(xs.shape[0], w.shape[2], dtype=xs.dtype, device=xs.device)
            for e, a, b in _slices(goff):
                y = xs[a:b] @ w[e]
                out[a:b] = y + bias[e] if bias is not None else y
        ctx.save_for_backward(xs, w, goff)
        return out

    @staticmethod
    def backward(ctx, dy):
        xs, w, goff = ctx.saved_tensors
        dy = dy.contiguous()
        db = None
        if ctx.native:
            dx = G.grouped_dgrad(dy, w, goff)
            dw = G.grouped_wgrad(xs, dy, goff, torch.empty_like(w))
            if ctx.has_bias:
                db = _segment_sum(dy, goff, w.shape[0])
        else:
            dx = torch.zeros_like(xs)
            dw = torch.zeros_like(w)
            db = torch.zeros(w.shape[0], w.shape[2], dtype=dy.dtype, device=dy.device) if ctx.has_bias else None
            for e, a, b in _slices(goff):
                dx[a:b] = dy[a:b] @ w[e].t()
                dw[e] = xs[a:b].t() @ dy[a:b]
                if db is not None:
                    db[e] = dy[a:b].sum(0)
        return dx, dw, None, db


def _segment_sum(x, goff, E):
    """Per-expert row sums [E, N] without host sync: segment ids from goff by searchsorted."""
    rows = torch.arange(x.shape[0], device=x.device, dtype=torch.int32)
    seg = torch.searchsorted(goff[1:].contiguous(), rows, right=True).long()
    out = torch.zeros(E, x.shape[1], dtype=torch.float32, device=x.device)
    out.index_add_(0, seg, x.float())
    return out.to(x.dtype)


class _GroupedSwiGLUFn(torch.autograd.Function):
    """a = silu(xs @ w_e[:, :F]) * (xs @ w_e[:, F:]) per expert; one grouped launch with the SwiGLU epilogue."""

    @staticmethod
    def forward(ctx, xs, w, goff):
        F2 = w.shape[2]
        ctx.native = (_native_ok(xs, w) and xs.shape[1] % 8 == 0 and F2 % 64 == 0)
        if ctx.native:
            xs, w = xs.contiguous(), w.contiguous()
            a, gu = G.grouped_swiglu(xs, w, goff)
        else:
            gu = torch.zeros(xs.shape[0], F2, dtype=xs.dtype, device=xs.device)
            for e, lo, hi in _slices(goff):
                gu[lo:hi] = xs[lo:hi] @ w[e]
            a = T.swiglu(gu)
        ctx.save_for_backward(xs, w, goff, gu)
        return a

    @staticmethod
    def backward(ctx, da):
        xs, w, goff, gu = ctx.saved_tensors
        with torch.enable_grad():
            g = gu.detach().requires_grad_(True)
            (dgu,) = torch.autograd.grad(T.swiglu(g), g, da)
        dgu = dgu.contiguous()
        if ctx.native:
            dx = G.grouped_dgrad(dgu, w, goff)
            dw = G.grouped_wgrad(xs, dgu, goff, torch.empty_like(w))
        else:
            dx, dw = torch.zeros_like(xs), torch.zeros_like(w)
            for e, lo, hi in _slices(goff):
                dx[lo:hi] = dgu[lo:hi] @ w[e].t()
                dw[e] = xs[lo:hi].t() @ dgu[lo:hi]
        return dx, dw, None


def grouped_linear(xs, w, goff, bias=None):
    """xs [T, K] rows sorted by expert, w [E, K, N], goff [E + 1] int32 -> [T, N]."""
    return _GroupedLinearFn.apply(xs, w, goff, bias)


def grouped_swiglu(xs, w, goff):
    """xs [T, K], w [E, K, 2F] packed [gate | up] -> silu(gate) * up [T, F]."""
    return _GroupedSwiGLUFn.apply(xs, w, goff)


def route_topk(logits, k, norm_topk_prob=True):
    """softmax -> top-k -> expert-sorted assignment, all on the device.

    Returns (token_of_row [T*k], gate_of_row [T*k] fp32, goff [E + 1] int32): row r of the sorted
    activation matrix is token ``token_of_row[r]`` routed to the expert whose slice holds r."""
    E = logits.shape[-1]
    probs = torch.softmax(logits.float(), -1)
    w, idx = torch.topk(probs, k, -1)
    if norm_topk_prob:
        w = w / w.sum(-1, keepdim=True)
    flat_e = idx.reshape(-1)
    order = torch.argsort(flat_e, stable=True)
    tok = order // k
    gate = w.reshape(-1)[order]
    counts = torch.bincount(flat_e, minlength=E)
    goff = torch.zeros(E + 1, dtype=torch.int32, device=logits.device)
    goff[1:] = counts.cumsum(0).to(torch.int32)
    return tok, gate, goff


def moe_ffn(x2, gate_weight, w1, w2, k, norm_topk_prob=True, b1=None, b2=None):
    """Token-choice top-k MoE FFN on x2 [T, H]: router, expert-sorted gather, grouped SwiGLU FFN, weighted
    scatter-add combine.  w1 [E, H, 2F] (packed gate|up), w2 [E, F, H]."""
    tok, gate, goff = route_topk(x2.float() @ gate_weight.float(), k, norm_topk_prob)
    xs = x2.index_select(0, tok)
    if b1 is None:
        h = grouped_swiglu(xs, w1, goff)
    else:
        h = T.swiglu(grouped_linear(xs, w1, goff, b1))
    ys = grouped_linear(h, w2, goff, b2)
    out = torch.zeros(x2.shape[0], ys.shape[1], dtype=torch.float32, device=x2.device)
    out = out.index_add(0, tok, ys.float() * gate[:, None])
    return out.to(x2.dtype)
