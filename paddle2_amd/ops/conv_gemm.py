"""Channels-last convolutions as GEMMs on the hand-written MFMA kernels (reference: paddle/phi/kernels/gpudnn/
conv_kernel.cu:305 / conv_grad_kernel.cu — cuDNN / MIOpen; this replaces MIOpen for the bottleneck convolutions).

* 1x1 (any stride: a stride subsamples the input first): forward y = x . W^T is the TN GEMM with both operands
  K-major as stored (x [pixels, Cin], W [Cout, Cin]), dgrad the forward GEMM node with W read as [K, N], wgrad a
  split-K GEMM over the pixels.
* 3x3, stride 1, padding 1 — implicit GEMM by row shifts.  The input is laid out with a one-pixel zero border and
  flattened to [padded pixels, Cin]; output pixel p of the padded grid reads input rows p + (kh - 1) * Wp + (kw - 1)
  for its 9 taps, so with K = 9 x Cin in tap-major order the A operand of K-tile kt is the input matrix with its base
  moved by a tap-dependent number of rows (gemm7.hip SCHED bit 11: only the LDS-DMA descriptor base changes).
  The border rows of the padded output are computed and dropped.  The input gradient is the same kernel with the
  shifts negated over the zero-bordered output gradient and the weight transposed to [Cin, 9 x Cout]; the weight
  gradient is 9 split-K GEMMs (one per tap) between the bordered output gradient and the shifted bordered input.
* Split-K weight gradients: the pixel reduction is cut into E slices run as one grouped GEMM (gemm.hip gmode 1,
  fp32 slab per slice) and summed — a [Cout, Cin] result is 1-4 tiles, which a plain GEMM would run on 1-4 CUs.
"""
from __future__ import annotations

import math
import os

import torch

from . import _native as N
from . import gemm as G

# auto (default) | native | miopen.  auto: per layer shape the faster of the native kernels and MIOpen, from one
# timed forward + backward of each (profiles/r4_secondary_configs.md: whole-network native 5,922 vs MIOpen
# 7,295 images/s on ResNet50 b=256, so the choice is made per shape, not globally)
MODE = os.environ.get("PADDLE2_AMD_CONV", "auto")
_ROUTE = {}
_CUS = {}
calls = {"1x1": 0, "3x3": 0}


def _cus(dev):
    c = _CUS.get(dev.index)
    if c is None:
        c = _CUS[dev.index] = torch.cuda.get_device_properties(dev).multi_processor_count
    return c


def wgrad_splitk(a, b):
    """fp32 [M, N] = a[R, M]^T . b[R, N] (rows = the reduction), the reduction split over E grouped slices."""
    R, M = a.shape
    Nn = b.shape[1]
    tiles = math.ceil(M / 256) * math.ceil(Nn / 256)
    E = max(1, min(max(1, 1024 // tiles), R // 1024))
    bounds = torch.div(torch.arange(E + 1, dtype=torch.int64) * R, E, rounding_mode="floor").to(torch.int32)
    goff = bounds.to(a.device, non_blocking=True)
    out = torch.empty(E, M, Nn, dtype=torch.float32, device=a.device)
    G.grouped_wgrad(a, b, goff, out)
    return out.sum(0)


# ---------------------------------------------------------------------------------------------------- 1x1
class Conv1x1Fn(torch.autograd.Function):
    """y[P, Co] = x[P, Ci] . W[Co, Ci]^T for NHWC x (stride-1 pixels; the caller subsamples strided inputs)."""

    @staticmethod
    def forward(ctx, x, w, b):
        calls["1x1"] += 1
        Nb, H, W_, Ci = x.shape
        Co = w.shape[0]
        x2 = x.reshape(-1, Ci)
        w2 = w.reshape(Co, Ci)
        y = torch.empty(x2.shape[0], Co, dtype=x.dtype, device=x.device)
        G._launch(G.LAYOUT_AK | G.LAYOUT_BK, G.EPI_BF16, x2, Ci, w2, Ci, y, Co, None, 0,
                  None if b is None else b.contiguous(), x2.shape[0], Co, Ci, name="fwd")
        ctx.save_for_backward(x2, w2)
        ctx.meta = (x.shape, w.shape, b is not None)
        return y.view(Nb, H, W_, Co)

    @staticmethod
    def backward(ctx, dy):
        from .torch_ops import bias_grad

        x2, w2 = ctx.saved_tensors
        xshape, wshape, has_b = ctx.meta
        dy2 = dy.reshape(-1, w2.shape[0])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = G.mm_fwd(dy2, w2).view(xshape)
        if ctx.needs_input_grad[1]:
            dw = wgrad_splitk(dy2, x2).to(w2.dtype).view(wshape)
        if has_b and ctx.needs_input_grad[2]:
            db = bias_grad(dy2)
        return dx, dw, db


# ---------------------------------------------------------------------------------------------------- 3x3
def _pow2_64(c):
    return c >= 64 and c % 64 == 0 and (c // 64) & (c // 64 - 1) == 0


def _bordered(x):
    """NHWC [N, H, W, C] -> (flat buffer [g + N*Hp*Wp + g, C] with a one-pixel zero border and g guard rows on both
    sides, g, Hp, Wp)."""
    Nb, H, W_, C = x.shape
    Hp, Wp = H + 2, W_ + 2
    g = Wp + 1
    M = Nb * Hp * Wp
    buf = torch.empty(g + M + g, C, dtype=x.dtype, device=x.device)
    buf[:g].zero_()
    buf[g + M:].zero_()
    grid = buf[g:g + M].view(Nb, Hp, Wp, C)
    grid[:, 0].zero_()
    grid[:, Hp - 1].zero_()
    grid[:, :, 0].zero_()
    grid[:, :, Wp - 1].zero_()
    grid[:, 1:H + 1, 1:W_ + 1].copy_(x)
    return buf, g, Hp, Wp


def _tap_weight(w_taps, C):
    """[Nout, 9, C] tap-major weight -> [Nout, K] with K rounded up to an even number of 64-wide K-tiles."""
    Nout = w_taps.shape[0]
    K = 9 * C
    Kp = K if (K // 64) % 2 == 0 else K + 64
    if Kp == K:
        return w_taps.reshape(Nout, K).contiguous(), K
    out = torch.zeros(Nout, Kp, dtype=w_taps.dtype, device=w_taps.device)
    out[:, :K] = w_taps.reshape(Nout, K)
    return out, Kp


def _conv_gemm(buf, g, C, Hp, Wp, M, wmat, K, Nout, sign):
    out = torch.empty(M, Nout, dtype=buf.dtype, device=buf.device)
    es = buf.element_size()
    base = buf.data_ptr()
    rc = N.native().gemm_conv(base + g * C * es, C, base, base + buf.numel() * es, wmat.data_ptr(), K,
                              out.data_ptr(), Nout, M, Nout, K, 9, 3, Wp, 1, 1, sign, int(math.log2(C // 64)), 4,
                              _cus(buf.device), N.stream())
    if rc != 0:
        raise RuntimeError(f"native implicit-GEMM conv failed ({rc})")
    return out


class Conv3x3Fn(torch.autograd.Function):
    """3x3 / stride 1 / padding 1 NHWC convolution on the implicit-GEMM kernel (see the module doc)."""

    @staticmethod
    def forward(ctx, x, w):
        calls["3x3"] += 1
        Nb, H, W_, Ci = x.shape
        Co = w.shape[0]
        buf, g, Hp, Wp = _bordered(x)
        M = Nb * Hp * Wp
        wmat, K = _tap_weight(w.permute(0, 2, 3, 1).reshape(Co, 9, Ci), Ci)
        yp = _conv_gemm(buf, g, Ci, Hp, Wp, M, wmat, K, Co, 1)
        ctx.save_for_backward(buf, w)
        ctx.meta = (Nb, H, W_, Ci, Co, g, Hp, Wp)
        return yp.view(Nb, Hp, Wp, Co)[:, 1:H + 1, 1:W_ + 1].contiguous()

    @staticmethod
    def backward(ctx, dy):
        buf, w = ctx.saved_tensors
        Nb, H, W_, Ci, Co, g, Hp, Wp = ctx.meta
        M = Nb * Hp * Wp
        dbuf, gd, _, _ = _bordered(dy.contiguous())
        dx = dw = None
        if ctx.needs_input_grad[0]:
            wd, Kd = _tap_weight(w.permute(1, 2, 3, 0).reshape(Ci, 9, Co), Co)
            dxp = _conv_gemm(dbuf, gd, Co, Hp, Wp, M, wd, Kd, Ci, -1)
            dx = dxp.view(Nb, Hp, Wp, Ci)[:, 1:H + 1, 1:W_ + 1].contiguous()
        if ctx.needs_input_grad[1]:
            dy_rows = dbuf[gd:gd + M]
            taps = []
            for kh in range(3):
                for kw in range(3):
                    s = (kh - 1) * Wp + (kw - 1)
                    taps.append(wgrad_splitk(dy_rows, buf[g + s:g + s + M]))   # [Co, Ci]
            dw = torch.stack(taps, 1).view(Co, 3, 3, Ci).permute(0, 3, 1, 2).contiguous().to(w.dtype)
        return dx, dw


def eligible_3x3(t_nhwc, w, stride, padding, dilation, groups):
    if MODE not in ("native", "auto") or not t_nhwc.is_cuda or t_nhwc.dtype != torch.bfloat16 \
            or w.dtype != torch.bfloat16:
        return False
    if not N.use_native(t_nhwc) or groups != 1 or tuple(w.shape[2:]) != (3, 3):
        return False
    if list(stride) != [1, 1] or list(dilation) != [1, 1] or list(padding) != [1, 1]:
        return False
    return _pow2_64(w.shape[1]) and _pow2_64(w.shape[0]) and route("3x3", t_nhwc, w, [1, 1], [1, 1])


def _time_fwd_bwd(fn, x, w, iters=5):
    from ..incubate.autotune import _bench

    with torch.enable_grad():
        xx = x.detach().requires_grad_(x.is_floating_point())
        ww = w.detach().requires_grad_(True)
        dy = torch.randn_like(fn(xx, ww))

        def run():
            torch.autograd.backward(fn(xx, ww), dy)
            xx.grad = ww.grad = None

        return _bench(run, iters)


def route(kind, x, w, stride, padding):
    """True -> the native kernel runs this NHWC conv.  MODE native: always; auto: timed once per (kind, shapes)
    against MIOpen (torch conv2d on the channels-last view), forward + backward, and cached."""
    if MODE == "native":
        return True
    key = (kind, tuple(x.shape), tuple(w.shape), tuple(stride))
    r = _ROUTE.get(key)
    if r is None:
        if torch.cuda.is_current_stream_capturing():
            return True                               # no timing inside a graph capture
        s = list(stride)
        if kind == "1x1":
            def nat(a, b):
                a = a[:, ::s[0], ::s[1], :] if s != [1, 1] else a
                return Conv1x1Fn.apply(a.contiguous(), b, None)
        else:
            def nat(a, b):
                return Conv3x3Fn.apply(a.contiguous(), b)

        def lib(a, b):
            return torch.nn.functional.conv2d(a.movedim(-1, 1), b, None, s, list(padding)).movedim(1, -1)

        r = _ROUTE[key] = _time_fwd_bwd(nat, x, w) <= _time_fwd_bwd(lib, x, w)
    return r
