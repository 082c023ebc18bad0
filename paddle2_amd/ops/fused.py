"""Fused elementwise training ops on the native kernels (csrc/kernels/fused_act.hip): bias + activation
(plain and gated: swiglu / geglu) and dropout + residual add with a counter-hash mask regenerated in the
backward (reference: phi/kernels/fusion/gpu/fused_bias_act_kernel.cu, fused_dropout_add_kernel.cu).
CPU: the same math in PyTorch, with the bit-identical mask (``dropout_keep``)."""
from __future__ import annotations

import torch

from . import _native as N

ACTS = {"identity": 0, "relu": 1, "gelu": 2, "gelu_tanh": 3, "silu": 4, "swish": 4, "sigmoid": 5}
GATED = {"swiglu": "silu", "geglu": "gelu"}
_M32 = 0xFFFFFFFF


def _act_torch(name, v):
    F = torch.nn.functional
    return {"identity": lambda t: t, "relu": torch.relu, "gelu": F.gelu,
            "gelu_tanh": lambda t: F.gelu(t, approximate="tanh"), "silu": F.silu, "swish": F.silu,
            "sigmoid": torch.sigmoid}[name](v)


def _native_ok(*ts):
    return all(t is None or (t.is_cuda and t.dtype in N.DT_CODE) for t in ts) and N.use_native(ts[0])


class _BiasActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act, gated):
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).contiguous()
        W = shp[-1]
        H = W // 2 if gated else W
        e = 4 if x.dtype == torch.float32 else 8
        ctx.native = _native_ok(x2, bias) and H % e == 0
        if ctx.native:
            b = None if bias is None else bias.contiguous().to(x.dtype)
            out = torch.empty(x2.shape[0], H, dtype=x.dtype, device=x.device)
            N.native().bias_act(N.DT_CODE[x.dtype], int(gated), ACTS[act], x2.data_ptr(), N.ptr(b), out.data_ptr(),
                                x2.shape[0], H, x2.stride(0), out.stride(0), N.stream())
        else:
            t = x2.float() + (0 if bias is None else bias.float())
            out = (_act_torch(act, t[:, :H]) * t[:, H:] if gated else _act_torch(act, t)).to(x.dtype)
        ctx.save_for_backward(x, bias)   # the input itself: under create_graph it carries the graph back to x
        ctx.meta = (act, gated, shp, H)
        return out.reshape(*shp[:-1], H)

    @staticmethod
    def backward(ctx, dout):
        x, bias = ctx.saved_tensors
        act, gated, shp, H = ctx.meta
        x2 = x.reshape(-1, shp[-1]).contiguous()
        d2 = dout.reshape(-1, H).contiguous()
        if torch.is_grad_enabled():
            # create_graph (double backward, incubate.autograd Hessian / jvp): a differentiable backward in torch
            # ops — the native kernel writes dx through raw pointers, with no graph for the second-order terms
            t = x2.float() + (0 if bias is None else bias.float())
            y = _act_torch(act, t[:, :H]) * t[:, H:] if gated else _act_torch(act, t)
            (dx,) = torch.autograd.grad(y, t, d2.float(), create_graph=True)
            dx = dx.to(x2.dtype)
        elif ctx.native:
            b = None if bias is None else bias.contiguous().to(x2.dtype)
            dx = torch.empty_like(x2)
            N.native().bias_act_bwd(N.DT_CODE[x2.dtype], int(gated), ACTS[act], x2.data_ptr(), N.ptr(b),
                                    d2.data_ptr(), dx.data_ptr(), x2.shape[0], H, x2.stride(0), d2.stride(0),
                                    N.stream())
        else:
            with torch.enable_grad():
                t = (x2.float() + (0 if bias is None else bias.float())).detach().requires_grad_(True)
                y = _act_torch(act, t[:, :H]) * t[:, H:] if gated else _act_torch(act, t)
                (dx,) = torch.autograd.grad(y, t, d2.float())
            dx = dx.to(x2.dtype)
        db = None if bias is None else dx.float().sum(0).to(bias.dtype)
        return dx.reshape(shp), db, None, None


def bias_act(x, bias=None, act="gelu"):
    """act(x + bias); act may be a gated name (swiglu / geglu: x = [a | g], out = act(a) * g)."""
    gated = act in GATED
    return _BiasActFn.apply(x, bias, GATED.get(act, act), gated)


def _mul32(x, c):
    return (x * (c & 0xFFFF) + (((x * (c >> 16)) & 0xFFFF) << 16)) & _M32


def dropout_keep(seed32, n, p, device="cpu"):
    """The kernel's keep mask over flat element indices 0..n-1 (bit-identical host model)."""
    idx = torch.arange(n, dtype=torch.int64, device=device)
    x = (int(seed32) & _M32) ^ _mul32(idx >> 32, 0x27D4EB2D)
    x = (x + _mul32(idx & _M32, 0x9E3779B1)) & _M32
    x = x ^ (x >> 15)
    x = _mul32(x, 0x85EBCA77)
    x = x ^ (x >> 13)
    x = _mul32(x, 0x27D4EB2F)
    x = x ^ (x >> 16)
    thresh = int(min(float(torch.tensor(p, dtype=torch.float32) * torch.tensor(4294967296.0)), 4294967040.0))
    return x >= thresh


class _DropoutAddFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y, p, seed):
        xc, yc = x.contiguous(), y.contiguous()
        e = 4 if x.dtype == torch.float32 else 8
        ctx.native = _native_ok(xc, yc) and xc.numel() % e == 0 and x.dtype == y.dtype
        ctx.meta = (p, seed, x.shape)
        if ctx.native:
            out = torch.empty_like(xc)
            N.native().dropout_add(N.DT_CODE[x.dtype], 0, xc.data_ptr(), yc.data_ptr(), out.data_ptr(), xc.numel(),
                                   seed, float(p), N.stream())
            return out
        keep = dropout_keep(seed, xc.numel(), p, x.device).reshape(x.shape)
        return (xc.float() * keep / (1.0 - p) + yc.float()).to(x.dtype)

    @staticmethod
    def backward(ctx, dout):
        p, seed, shape = ctx.meta
        d = dout.contiguous()
        if ctx.native:
            dx = torch.empty_like(d)
            N.native().dropout_add(N.DT_CODE[d.dtype], 1, d.data_ptr(), 0, dx.data_ptr(), d.numel(), seed, float(p),
                                   N.stream())
        else:
            keep = dropout_keep(seed, d.numel(), p, d.device).reshape(shape)
            dx = (d.float() * keep / (1.0 - p)).to(d.dtype)
        return dx, dout, None, None


def dropout_add(x, y, p, seed=None):
    """dropout(x, p) + y (upscale_in_train), mask regenerated from ``seed`` in the backward."""
    if seed is None:
        from .torch_ops import attn_dropout_seed

        seed = attn_dropout_seed()
    return _DropoutAddFn.apply(x, y, float(p), int(seed) & _M32)
