"""torch-level fused ops: HIP kernel on the MI355X, PyTorch reference on CPU.

Each op is a ``torch.autograd.Function`` whose forward/backward call the CDNA4 kernels of
``paddle2_amd._C`` when the inputs are on the GPU (``_native.use_native`` raises if the extension
is missing there, so GPU runs never silently fall back).  The CPU branches are the fp32
reference implementations that the numerics tests compare against.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from . import _native as N

_DT = N.DT_CODE

_DT_CLS = []


class _DTensorMeta(type):
    """``isinstance(x, _DTensor)`` is the framework's DistTensor, resolved on first use (the distributed package
    imports this module, so it cannot be imported here)."""

    def __instancecheck__(cls, obj):
        if type(obj) is torch.Tensor or not isinstance(obj, torch.Tensor):
            return False
        if not _DT_CLS:
            from ..distributed.auto_parallel.dist_tensor import DistTensor

            _DT_CLS.append(DistTensor)
        return isinstance(obj, _DT_CLS[0])


class _DTensor(metaclass=_DTensorMeta):
    """DistTensor arguments take the SPMD dispatch at op entry (distributed/auto_parallel/dist_ops.py)."""


def _dist_ops():
    from ..distributed.auto_parallel import dist_ops

    return dist_ops


def _rows(x: torch.Tensor):
    n = x.shape[-1]
    return x.numel() // max(n, 1), n


# ============================================================================ RMSNorm / LayerNorm
class _NormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, residual, eps, layernorm):
        shape = x.shape
        M, Nn = _rows(x)
        x2 = x.reshape(M, Nn).contiguous()
        res2 = residual.reshape(M, Nn).contiguous() if residual is not None else None
        if w is None:
            w = torch.ones(Nn, dtype=x.dtype, device=x.device)
        wc = w.contiguous()
        if wc.dtype not in (x.dtype, torch.float32):
            wc = wc.to(x.dtype)
        bc = None
        if b is not None:
            bc = b.contiguous().to(wc.dtype)
        if N.use_native(x) and x.dtype in _DT and (Nn % (4 if x.dtype == torch.float32 else 8) == 0) and \
                Nn <= (4096 if x.dtype == torch.float32 else 8192):
            C = N.native()
            y = torch.empty_like(x2)
            rstd = torch.empty(M, dtype=torch.float32, device=x.device)
            mean = torch.empty(M, dtype=torch.float32, device=x.device) if layernorm else None
            h = torch.empty_like(x2) if res2 is not None else None
            C.norm_fwd(int(layernorm), _DT[x.dtype], _DT[wc.dtype], x2.data_ptr(), N.ptr(res2), wc.data_ptr(),
                       N.ptr(bc), y.data_ptr(), N.ptr(h), N.ptr(mean), rstd.data_ptr(), M, Nn, float(eps), N.stream())
            hh = h if h is not None else x2
            ctx.native = True
        else:
            hh = (x2.float() + res2.float()).to(x.dtype) if res2 is not None else x2
            hf = hh.float()
            if layernorm:
                mean = hf.mean(-1)
                var = ((hf - mean[:, None]) ** 2).mean(-1)
                rstd = torch.rsqrt(var + eps)
                yf = (hf - mean[:, None]) * rstd[:, None] * wc.float()
            else:
                mean = None
                rstd = torch.rsqrt((hf * hf).mean(-1) + eps)
                yf = hf * rstd[:, None] * wc.float()
            if bc is not None:
                yf = yf + bc.float()
            y = yf.to(x.dtype)
            h = hh if res2 is not None else None
            ctx.native = False
        ctx.save_for_backward(hh, wc, mean, rstd)
        ctx.layernorm = layernorm
        ctx.has_res = res2 is not None
        ctx.has_b = bc is not None
        ctx.shape = shape
        ctx.wdtype = w.dtype
        ctx.params = (w, b)
        if res2 is not None:
            return y.reshape(shape), h.reshape(shape)
        return y.reshape(shape), None

    @staticmethod
    def backward(ctx, dy, dh):
        hh, wc, mean, rstd = ctx.saved_tensors
        M, Nn = hh.shape
        dy2 = dy.reshape(M, Nn).contiguous()
        dh2 = dh.reshape(M, Nn).contiguous() if (dh is not None and ctx.has_res) else None
        if ctx.native:
            C = N.native()
            nb = C.norm_bwd_blocks(M)
            dx = torch.empty_like(hh)
            dw_part = torch.empty(nb, Nn, dtype=torch.float32, device=hh.device)
            db_part = torch.empty(nb, Nn, dtype=torch.float32, device=hh.device) if ctx.layernorm else None
            # weight (and bias) gradients straight into their fp32 main-grad slots when every one has a slot
            wp, bp = ctx.params
            slots = None
            if BIAS_MAIN and ctx.needs_input_grad[1] and (not ctx.has_b or ctx.needs_input_grad[2]):
                slots = [main_slot(wp)] + ([main_slot(bp)] if ctx.has_b else [])
                if any(sl is None for sl in slots):
                    slots = None
            if slots is not None:
                dw = slots[0][0]
                db = slots[1][0] if ctx.has_b else (
                    torch.empty(Nn, dtype=torch.float32, device=hh.device) if ctx.layernorm else None)
                accs = [int(sl[1] != 0) for sl in slots] + [0]
                odt = _DT[torch.float32]
            else:
                dw = torch.empty(Nn, dtype=wc.dtype, device=hh.device)
                db = torch.empty(Nn, dtype=wc.dtype, device=hh.device) if ctx.layernorm else None
                accs, odt = [0, 0], -1
            C.norm_bwd(int(ctx.layernorm), _DT[hh.dtype], _DT[wc.dtype], dy2.data_ptr(), hh.data_ptr(), wc.data_ptr(),
                       N.ptr(mean), rstd.data_ptr(), N.ptr(dh2), dx.data_ptr(), dw_part.data_ptr(), N.ptr(db_part),
                       dw.data_ptr(), N.ptr(db), M, Nn, nb, N.stream(), odt=odt, acc_w=accs[0], acc_b=accs[1])
            if slots is not None:
                for _v, _b, owner, idx in slots:
                    owner.param_grad_done(idx)
                dx = dx.reshape(ctx.shape)
                return dx, None, None, (dx if ctx.has_res else None), None, None
        else:
            hf = hh.float()
            xh = (hf - mean[:, None]) * rstd[:, None] if ctx.layernorm else hf * rstd[:, None]
            g = dy2.float() * wc.float()
            dxf = g - xh * (g * xh).mean(-1, keepdim=True)
            if ctx.layernorm:
                dxf = dxf - g.mean(-1, keepdim=True)
            dxf = dxf * rstd[:, None]
            if dh2 is not None:
                dxf = dxf + dh2.float()
            dx = dxf.to(hh.dtype)
            dw = (dy2.float() * xh).sum(0).to(wc.dtype)
            db = dy2.float().sum(0).to(wc.dtype) if ctx.layernorm else None
        dx = dx.reshape(ctx.shape)
        dres = dx if ctx.has_res else None
        dw = dw.to(ctx.wdtype)
        return dx, dw, (db if ctx.has_b else None), dres, None, None


def rms_norm(x, w, eps=1e-6, residual=None):
    if isinstance(x, _DTensor) or isinstance(residual, _DTensor):   # DistTensor: SPMD dispatch at op entry
        return _dist_ops().rms_norm(x, w, eps, residual)
    y, h = _NormFn.apply(x, w, None, residual, eps, False)
    return (y, h) if residual is not None else y


def rms_norm_partials(p, w, eps, residual):
    """rms_norm(x, w, eps, residual) -> (y, x + residual) where x arrives as a decode GEMM's unreduced split-K partials
    (ops.weight_only.DecodePartials): the partials are summed and rounded inside the norm kernel, bit-identical to
    reducing them first.  Falls back to materialising x when the rows are outside the kernel's form."""
    r2 = residual.reshape(p.M, p.N) if residual.is_contiguous() else None
    wdt = _DT.get(w.dtype)
    if (r2 is None or p.dtype != torch.bfloat16 or residual.dtype != torch.bfloat16 or wdt not in (_DT[torch.bfloat16],
            _DT[torch.float32]) or not w.is_contiguous() or p.N % 8 or p.N > 8192 or not N.use_native(residual)):
        return rms_norm(p.materialize(), w, eps, residual)
    y = torch.empty(p.M, p.N, dtype=residual.dtype, device=residual.device)
    h = torch.empty_like(y)
    N.native().norm_fwd_part(wdt, p.ws.data_ptr(), p.S, r2.data_ptr(), w.data_ptr(), y.data_ptr(), h.data_ptr(),
                             p.M, p.N, float(eps), N.stream())
    return y.view(p.shape), h.view(p.shape)


def layer_norm(x, w, b, eps=1e-5, residual=None):
    if isinstance(x, _DTensor) or isinstance(residual, _DTensor):
        return _dist_ops().rms_norm(x, w, eps, residual, layer=True, b=b)
    y, h = _NormFn.apply(x, w, b, residual, eps, True)
    return (y, h) if residual is not None else y


# ============================================================================ SwiGLU
class _SwiGLUFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, y):
        packed = y is None
        if packed:
            H = x.shape[-1] // 2
            rows = x.numel() // x.shape[-1]
            xc = x.contiguous()
            out_shape = list(x.shape[:-1]) + [H]
        else:
            H = x.shape[-1]
            rows = x.numel() // H
            xc, yc = x.contiguous(), y.contiguous()
            out_shape = list(x.shape)
        ctx.packed, ctx.H, ctx.rows = packed, H, rows
        if N.use_native(x) and x.dtype in _DT and H % (4 if x.dtype == torch.float32 else 8) == 0:
            C = N.native()
            out = torch.empty(out_shape, dtype=x.dtype, device=x.device)
            if packed:
                C.swiglu_fwd(_DT[x.dtype], xc.data_ptr(), xc.data_ptr() + H * xc.element_size(), out.data_ptr(), rows, H,
                             2 * H, 2 * H, N.stream())
                ctx.save_for_backward(xc)
            else:
                C.swiglu_fwd(_DT[x.dtype], xc.data_ptr(), yc.data_ptr(), out.data_ptr(), rows, H, H, H, N.stream())
                ctx.save_for_backward(xc, yc)
            ctx.native = True
            return out
        ctx.native = False
        if packed:
            a, b = xc[..., :H], xc[..., H:]
            ctx.save_for_backward(xc)
        else:
            a, b = xc, yc
            ctx.save_for_backward(xc, yc)
        return (F.silu(a.float()) * b.float()).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        H, rows = ctx.H, ctx.rows
        gc = g.contiguous()
        if ctx.packed:
            (xc,) = ctx.saved_tensors
        else:
            xc, yc = ctx.saved_tensors
        if ctx.native:
            C = N.native()
            es = xc.element_size()
            if ctx.packed:
                dxy = torch.empty_like(xc)
                C.swiglu_bwd(_DT[xc.dtype], xc.data_ptr(), xc.data_ptr() + H * es, gc.data_ptr(), dxy.data_ptr(),
                             dxy.data_ptr() + H * es, rows, H, 2 * H, 2 * H, 2 * H, 2 * H, N.stream())
                return dxy, None
            dx = torch.empty_like(xc)
            dy = torch.empty_like(yc)
            C.swiglu_bwd(_DT[xc.dtype], xc.data_ptr(), yc.data_ptr(), gc.data_ptr(), dx.data_ptr(), dy.data_ptr(), rows,
                         H, H, H, H, H, N.stream())
            return dx, dy
        if ctx.packed:
            a, b = xc[..., :H].float(), xc[..., H:].float()
        else:
            a, b = xc.float(), yc.float()
        s = torch.sigmoid(a)
        gf = gc.float()
        da = gf * b * s * (1 + a * (1 - s))
        db = gf * a * s
        if ctx.packed:
            return torch.cat([da, db], -1).to(xc.dtype), None
        return da.to(xc.dtype), db.to(yc.dtype)


def swiglu(x, y=None):
    if isinstance(x, _DTensor) or isinstance(y, _DTensor):
        return _dist_ops().swiglu(x, y)
    return _SwiGLUFn.apply(x, y)


# ============================================================================ RoPE
def rope_tables(seq_len, head_dim, base=10000.0, interleaved=True, device=None, position_scale=1.0):
    """cos/sin fp32 tables [S, D] laid out for the chosen rotation style."""
    inv = 1.0 / (base ** (torch.arange(0, head_dim, 2, dtype=torch.float32, device=device) / head_dim))
    t = torch.arange(seq_len, dtype=torch.float32, device=device) * position_scale
    freqs = torch.outer(t, inv)  # [S, D/2]
    if interleaved:
        emb = torch.repeat_interleave(freqs, 2, dim=-1)
    else:
        emb = torch.cat([freqs, freqs], dim=-1)
    return emb.cos(), emb.sin()


class _RopeFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, cos, sin, pos, style, time_major):
        ctx.save_for_backward(cos, sin, pos)
        ctx.style, ctx.tm = style, time_major
        return _rope_apply(x, cos, sin, pos, style, time_major, False)

    @staticmethod
    def backward(ctx, g):
        cos, sin, pos = ctx.saved_tensors
        return _rope_apply(g, cos, sin, pos, ctx.style, ctx.tm, True), None, None, None, None, None


def _tok_view_ok(t):
    """[A, B, H, D] with unit stride on D, stride D on H and uniform token stride (A*B tokens)."""
    st = t.stride()
    return st[3] == 1 and st[2] == t.shape[3] and st[0] == t.shape[1] * st[1]


def _rope_apply(x, cos, sin, pos, style, time_major, bwd, out=None):
    """Rotate x ([B,S,H,D] or time-major); x and ``out`` may be token-strided views."""
    if time_major:
        S, B, Hn, D = x.shape
    else:
        B, S, Hn, D = x.shape
    if N.use_native(x) and x.dtype in _DT:
        xc = x if _tok_view_ok(x) else x.contiguous()
        C = N.native()
        if out is None:
            out = torch.empty(x.shape, dtype=x.dtype, device=x.device)
        C.rope(_DT[x.dtype], style, int(bwd), xc.data_ptr(), out.data_ptr(), cos.data_ptr(), sin.data_ptr(),
               N.ptr(pos), B, S, Hn, D, int(time_major), xc.stride(1), out.stride(1), N.stream())
        return out
    xc = x.contiguous()
    if out is not None:
        out.copy_(_rope_apply(xc, cos, sin, pos, style, time_major, bwd))
        return out
    # reference
    xf = xc.float()
    if pos is not None:
        c = cos[pos]  # [B, S, D]
        s_ = sin[pos]
        c = c[:, :, None, :]
        s_ = s_[:, :, None, :]
        if time_major:
            c, s_ = c.transpose(0, 1), s_.transpose(0, 1)
    else:
        c = cos[:S][:, None, :]
        s_ = sin[:S][:, None, :]
        if not time_major:
            c, s_ = c[None], s_[None]
    if style == 0:
        half = D // 2
        xa, xb = xf[..., :half], xf[..., half:]
        ca, cb = c[..., :half], c[..., half:]
        sa, sb = s_[..., :half], s_[..., half:]
    else:
        xa, xb = xf[..., 0::2], xf[..., 1::2]
        ca, cb = c[..., 0::2], c[..., 1::2]
        sa, sb = s_[..., 0::2], s_[..., 1::2]
    if not bwd:
        oa = xa * ca - xb * sa
        ob = xb * cb + xa * sb
    else:
        oa = xa * ca + xb * sb
        ob = xb * cb - xa * sa
    if style == 0:
        out = torch.cat([oa, ob], -1)
    else:
        out = torch.stack([oa, ob], -1).flatten(-2)
    return out.to(x.dtype)


def rope(x, cos, sin, pos=None, style=0, time_major=False):
    """Apply rotary embedding. style 0 = rotate-half, 1 = rotate-every-two (interleaved)."""
    if isinstance(x, _DTensor):
        return _dist_ops().rope(x, cos, sin, pos, style, time_major)
    cos = cos.reshape(-1, x.shape[-1]).float().contiguous()
    sin = sin.reshape(-1, x.shape[-1]).float().contiguous()
    if pos is not None:
        pos = pos.to(torch.int64).contiguous()
    return _RopeFn.apply(x, cos, sin, pos, style, time_major)


# ============================================================================ Linear (layout-aware GEMMs)
def transpose2d(x):
    """[M, N] (unit column stride) -> contiguous [N, M]; the HBM-speed HIP transpose for 16-bit tensors."""
    M, N_ = x.shape
    if (x.device.type == "cuda" and N.use_native(x) and x.element_size() == 2 and x.stride(1) == 1
            and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and M % 8 == 0):
        out = torch.empty(N_, M, dtype=x.dtype, device=x.device)
        N.native().transpose16(x.data_ptr(), out.data_ptr(), M, N_, x.stride(0), M, N.stream())
        return out
    return x.t().contiguous()


import os as _os  # noqa: E402

_LINEAR_LAYOUT = _os.environ.get("PADDLE2_AMD_LINEAR_LAYOUT", "auto")  # auto | off | all


def _linear_plan(M, K, Nn):
    """(fwd via W^T, dW via X^T / dY^T).  hipBLASLt runs the layout with both operands contiguous along the
    reduction dim fastest (profiles/r1_gemm_layouts.md); the transposes cost one HBM pass each, so they pay
    only on token-heavy GEMMs (W^T: M >= 4096; dW: M >= 8192 and the dY transpose amortised, N >= 2K)."""
    if _LINEAR_LAYOUT == "off":
        return False, False
    if _LINEAR_LAYOUT == "all":
        return True, True
    return M >= 4096 and K % 8 == 0, M >= 8192 and Nn >= 2 * K


class WeightGradStore:
    """Zero-bubble pipeline support (reference: the ZB-H1 / ZBV schedules' split of backward into B = input
    gradient and W = weight gradient, distributed/passes/pipeline_scheduler_pass/pipeline_zero_bubble.py).

    ``route``: set during a zero-bubble stage's forward so every Linear runs through ``_LinearFn`` (whose
    backward can split); ``defer``: set during a B unit — the Linear backward then computes only dX and
    queues its weight-gradient GEMM; ``take()`` hands the queue to the W unit, which runs it later to fill a
    pipeline bubble.  Weight grads land in ``param.grad`` (or the fp32 main-grad buffer) exactly as in a
    normal backward."""

    route = False
    defer = False
    _queue = []

    @classmethod
    def put(cls, fn):
        cls._queue.append(fn)

    @classmethod
    def take(cls):
        q, cls._queue = cls._queue, []
        return q

    @staticmethod
    def run(queue):
        for fn in queue:
            fn()


def _accumulate_grad(w, dw):
    with torch.no_grad():
        if w.grad is None:
            w.grad = dw.to(w.dtype)
        else:
            w.grad.add_(dw.to(w.grad.dtype))


class _LinearFn(torch.autograd.Function):
    """y = x @ W (+ b) with W [K, N] (Paddle layout) — GEMM layouts picked per shape (see _linear_plan)."""

    @staticmethod
    def forward(ctx, x, w, b):
        K, Nn = w.shape
        x2 = x.reshape(-1, K)
        M = x2.shape[0]
        fwd_t, dw_t = _linear_plan(M, K, Nn)
        from . import gemm as G

        if G.supported_fwd(x2, w) and (b is None or b.dtype == x2.dtype) and _pass_native("fwd", x2, w):
            y = G.mm_fwd(x2, w, bias=None if b is None else b.contiguous())
        else:
            if fwd_t:
                y = torch.matmul(x2, transpose2d(w).t())
            else:
                y = torch.matmul(x2, w)
            if b is not None:
                y += b
        ctx.save_for_backward(x2, w)
        ctx.meta = (x.shape, dw_t, b is not None)
        ctx.gt = getattr(w, "_p2_gt", None)
        ctx.bt = b
        ctx.w_leaf = w if WeightGradStore.route else None
        return y.view(*x.shape[:-1], Nn)

    @staticmethod
    def backward(ctx, dy):
        x2, w = ctx.saved_tensors
        xshape, dw_t, has_b = ctx.meta
        Nn = w.shape[1]
        dy2 = dy.reshape(-1, Nn)
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dx = dw = db = None
        from . import gemm as G

        if ctx.needs_input_grad[0]:
            if G.supported_dgrad(dy2, w) and _pass_native("dgrad", dy2, w):
                dx = G.mm_dgrad(dy2, w).view(xshape)
            else:
                dx = torch.matmul(dy2, w.t()).view(xshape)
        if ctx.needs_input_grad[1] and WeightGradStore.defer and (ctx.gt is not None or ctx.w_leaf is not None):
            gt, wl = ctx.gt, ctx.w_leaf

            def _w_pass(x2=x2, dy2=dy2, gt=gt, wl=wl):
                if gt is not None:
                    _main_grad_accumulate(gt, x2, dy2)
                else:
                    _accumulate_grad(wl, weight_grad(x2, dy2))

            WeightGradStore.put(_w_pass)
        elif ctx.needs_input_grad[1]:
            if ctx.gt is not None:
                _main_grad_accumulate(ctx.gt, x2, dy2)
            elif G.supported_wgrad(x2, dy2) and _pass_native("wgrad", x2, dy2):
                dw = G.mm_wgrad_bf16(x2, dy2)
            elif dw_t:
                dw = torch.matmul(transpose2d(x2), transpose2d(dy2).t())
            else:
                dw = torch.matmul(x2.t(), dy2)
        if has_b and ctx.needs_input_grad[2]:
            db = bias_grad(dy2, bt=ctx.bt)
        return dx, dw, db


def main_slot(t):
    """The fp32 main-grad slot of a 1-D parameter (a sharding unit's ``_p2_bt``: biases, norm weights) as
    (view, beta, owner, index), or None.  Its gradient kernel writes there (beta 1: accumulate) and calls
    ``owner.param_grad_done(index)``; autograd then gets None, so no bf16 gradient and no fp32 conversion pass."""
    bt = getattr(t, "_p2_bt", None) if t is not None else None
    if bt is None:
        return None
    owner, idx = bt
    view, beta = owner.grad_target(idx)
    if view.dtype != torch.float32 or not view.is_contiguous() or view.data_ptr() % 16 != 0:
        return None
    return view, beta, owner, idx


def bias_grad(dy2, out_dtype=None, bt=None):
    """db = dy2.sum(0) for a [M, N] gradient: the native two-pass column sum (csrc/kernels/norm.hip
    bias_grad_part_kernel + colsum, fp32 accumulation, deterministic) — torch's bf16 dim-0 reduce ran 5-30x slower
    on the GPT-3 13B step (24.9 ms / 160 calls).  ``out_dtype`` (default dy2's): the fp32 partials are rounded once,
    straight to it — an fp32 master bias gets the fp32 sum, not a bf16-rounded one.  ``bt``: the bias tensor; with
    an fp32 main-grad slot (main_slot) the sum lands there and None is returned."""
    M, Nn = dy2.shape
    odt = out_dtype or dy2.dtype
    if (N.use_native(dy2) and dy2.dtype in _DT and odt in _DT and Nn % 8 == 0 and dy2.is_contiguous() and M > 0
            and dy2.data_ptr() % 16 == 0):
        C = N.native()
        part = torch.empty(C.bias_grad_chunks(M, Nn) * Nn, dtype=torch.float32, device=dy2.device)
        slot = main_slot(bt) if bt is not None and BIAS_MAIN else None
        if slot is not None:
            view, beta, owner, idx = slot
            C.bias_grad(_DT[dy2.dtype], _DT[torch.float32], dy2.data_ptr(), part.data_ptr(), view.data_ptr(), M, Nn,
                        N.stream(), acc=int(beta != 0))
            owner.param_grad_done(idx)
            return None
        db = torch.empty(Nn, dtype=odt, device=dy2.device)
        C.bias_grad(_DT[dy2.dtype], _DT[odt], dy2.data_ptr(), part.data_ptr(), db.data_ptr(), M, Nn, N.stream())
        return db
    return dy2.sum(0, dtype=torch.float32).to(odt)


# 1-D parameter gradients (biases, norm weights) written straight into their fp32 main-grad slots
BIAS_MAIN = _os.environ.get("PADDLE2_AMD_BIAS_MAIN", "1") != "0"


def _pass_native(name, t, other=None):
    """Per-pass GEMM backend (PADDLE2_AMD_GEMM_{FWD,DGRAD,WGRAD} = native | blas): the hand-written MFMA
    kernel (ops/gemm.py) or hipBLASLt, chosen per pass from measured speed (profiles/r2_gemm_native.md) — or,
    with routing autotune on (incubate.autotune.enable_routing_autotune), per shape from timing both."""
    from . import gemm as G

    if not G.enabled(t):
        return False
    if other is not None:
        from ..incubate import autotune as _at

        r = _at.route(name, t, other)
        if r is not None:
            return r
    return _GEMM_PASS.get("wgrad" if name == "wgrad32" else name, "native") == "native"


_GEMM_PASS = {"fwd": _os.environ.get("PADDLE2_AMD_GEMM_FWD", "native"),
              "dgrad": _os.environ.get("PADDLE2_AMD_GEMM_DGRAD", "native"),
              "wgrad": _os.environ.get("PADDLE2_AMD_GEMM_WGRAD", "native")}


def wgrad_accumulate(out, x2, dy2, beta):
    """out[K, N] (fp32 main grad) = x2^T @ dy2 + beta * out, with the product accumulated in fp32 — never
    rounded to the activation dtype first (reference fused_linear_param_grad_add_kernel.cu:51, use_addto).
    GPU: the native MFMA GEMM's fp32 main-grad epilogue (M/N-major operands, no transpose pass)."""
    if out.device.type == "cuda":
        from . import gemm as G

        if (out.dtype == torch.float32 and out.is_contiguous() and G.supported_wgrad(x2, dy2)
                and _pass_native("wgrad32", x2, dy2)):
            G.mm_wgrad(x2, dy2, out, beta)
            return out
        torch.addmm(out, x2.t(), dy2, beta=float(beta), out_dtype=out.dtype, out=out)
        return out
    if beta == 0:
        out.zero_()
    out.addmm_(x2.t().to(out.dtype), dy2.to(out.dtype))
    return out


def mm(x2, w, b=None):
    """y[M, N] = x2[M, K] @ w[K, N] (+ b): the Linear forward GEMM (native MFMA kernel or hipBLASLt per
    _GEMM_PASS), shared by nn.Linear and the tensor-/sequence-parallel linears."""
    from . import gemm as G

    if x2.dim() == 2 and G.supported_fwd(x2, w) and (b is None or b.dtype == x2.dtype) and _pass_native("fwd", x2, w):
        return G.mm_fwd(x2, w, bias=None if b is None else b.contiguous())
    y = torch.matmul(x2, w)
    return y + b if b is not None else y


def mm_t(dy2, w):
    """dx[M, K] = dy2[M, N] @ w[K, N]^T (the Linear input-gradient GEMM)."""
    from . import gemm as G

    if dy2.dim() == 2 and G.supported_dgrad(dy2, w) and _pass_native("dgrad", dy2, w):
        return G.mm_dgrad(dy2, w)
    return torch.matmul(dy2, w.t())


def weight_grad(x2, dy2, gt=None):
    """dW = x2^T @ dy2.  With a main-grad target ``gt`` the product accumulates in fp32 straight into it
    and None is returned (the autograd engine then never materialises a 16-bit dW)."""
    if gt is not None:
        _main_grad_accumulate(gt, x2, dy2)
        return None
    from . import gemm as G

    if G.supported_wgrad(x2, dy2) and _pass_native("wgrad", x2, dy2):
        return G.mm_wgrad_bf16(x2, dy2)
    return torch.matmul(x2.t(), dy2)


def _main_grad_accumulate(gt, x2, dy2):
    """Weight gradient straight into the owner's fp32 main-grad buffer (group-sharded unit / main_grad):
    ``gt`` = (owner, index) with owner.grad_target(index) -> (fp32 view, beta) and owner.param_grad_done."""
    owner, idx = gt
    view, beta = owner.grad_target(idx)
    wgrad_accumulate(view, x2, dy2, beta)
    owner.param_grad_done(idx)


def linear(x, w, b=None):
    """Paddle-layout linear on bf16/fp16 GPU tensors through the layout-aware GEMM node (and on any device
    when the weight's gradient goes to an fp32 main-grad buffer); plain matmul otherwise."""
    if isinstance(x, _DTensor) or isinstance(w, _DTensor):
        return _dist_ops().linear(x, w, b)
    if (x.device.type == "cuda" and x.dtype in (torch.bfloat16, torch.float16) and w.dtype == x.dtype
            and w.dim() == 2 and x.shape[-1] == w.shape[0] and N.use_native(x)) or \
            (getattr(w, "_p2_gt", None) is not None and w.dim() == 2 and x.shape[-1] == w.shape[0]) or \
            (WeightGradStore.route and w.dim() == 2 and x.shape[-1] == w.shape[0] and w.requires_grad):
        return _LinearFn.apply(x, w, b)
    y = torch.matmul(x, w)
    return y + b if b is not None else y


class _TiedLogitsFn(torch.autograd.Function):
    """logits = h @ E^T for a tied word embedding E [V, H] (GPT's output layer) on the native GEMM: E as stored is
    the K-major B operand of the TN kernel (no transpose pass); backward dh = dlogits @ E (the forward form) and
    dE = dlogits^T @ h (the weight-gradient form, bf16, accumulated by autograd with the embedding's own grad).
    Reference: the tied-embedding matmul of test/auto_parallel/get_gpt_model.py (paddle.matmul(x, w,
    transpose_y=True))."""

    @staticmethod
    def forward(ctx, h2, E):
        from . import gemm as G

        ctx.save_for_backward(h2, E)
        return G.mm_dgrad(h2, E)

    @staticmethod
    def backward(ctx, dy):
        from . import gemm as G

        h2, E = ctx.saved_tensors
        dy2 = dy.contiguous()
        dh = G.mm_fwd(dy2, E) if ctx.needs_input_grad[0] else None
        dE = G.mm_wgrad_bf16(dy2, h2) if ctx.needs_input_grad[1] else None
        return dh, dE


def tied_logits(h, E):
    """h [..., H] @ E[V, H]^T: the native TN GEMM for bf16 GPU tensors of native-friendly shapes, torch.matmul
    otherwise."""
    from . import gemm as G

    h2 = h.reshape(-1, h.shape[-1])
    if (h.device.type == "cuda" and G.enabled(h2) and E.dtype == h2.dtype and E.dim() == 2
            and E.shape[1] == h2.shape[1] and E.shape[0] % 8 == 0 and G.supported_dgrad(h2, E)
            and _pass_native("dgrad", h2, E)):
        if not h2.is_contiguous():
            h2 = h2.contiguous()
        return _TiedLogitsFn.apply(h2, E).view(*h.shape[:-1], E.shape[0])
    return torch.matmul(h, E.t())


class _GeluMLPFn(torch.autograd.Function):
    """y = gelu(x @ W1 + b1) @ W2 + b2 (the GPT MLP) as one autograd node, so the GELU rides on the GEMM epilogues in
    both directions (reference funcs/fused_gemm_epilogue.h:382 GELU_AUX_BIAS forward, :580 gelu_grad backward;
    incubate fused_feedforward):
      forward   a, h = gelu(x W1 + b1), x W1 + b1       one GEMM, two outputs (h is what the backward needs)
                y = a W2 + b2                            bias epilogue
      backward  dh = (dy W2^T) * gelu'(h)               the dgrad GEMM with the dGELU epilogue
                dW2 = a^T dy, dW1 = x^T dh (fp32 main grads when the weights have them), db = column sums
                dx = dh W1^T"""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, approximate):
        from . import gemm as G

        K = w1.shape[0]
        x2 = x.reshape(-1, K)
        a, h = G.mm_gelu(x2, w1, None if b1 is None else b1.contiguous(), approximate)
        y = G.mm_fwd(a, w2, bias=None if b2 is None else b2.contiguous())
        ctx.save_for_backward(x2, w1, w2, a, h)
        ctx.meta = (x.shape, b1 is not None, b2 is not None, approximate)
        ctx.gt = (getattr(w1, "_p2_gt", None), getattr(w2, "_p2_gt", None))
        return y.view(*x.shape[:-1], w2.shape[1])

    @staticmethod
    def backward(ctx, dy):
        from . import gemm as G

        x2, w1, w2, a, h = ctx.saved_tensors
        xshape, has_b1, has_b2, approximate = ctx.meta
        gt1, gt2 = ctx.gt
        dy2 = dy.reshape(-1, w2.shape[1])
        if not dy2.is_contiguous():
            dy2 = dy2.contiguous()
        dh = G.mm_dgrad_dgelu(dy2, w2, h, approximate)
        need = ctx.needs_input_grad
        dw2 = weight_grad(a, dy2, gt2) if need[3] else None
        db2 = bias_grad(dy2) if has_b2 and need[4] else None
        dw1 = weight_grad(x2, dh, gt1) if need[1] else None
        db1 = bias_grad(dh) if has_b1 and need[2] else None
        dx = G.mm_dgrad(dh, w1).view(xshape) if need[0] else None
        return dx, dw1, db1, dw2, db2, None


_FUSED_GELU_MLP = _os.environ.get("PADDLE2_AMD_FUSED_GELU_MLP", "0") != "0"


def gelu_mlp_ok(x, w1, b1, w2, b2):
    """The fused GELU-MLP node applies: bf16 GPU tensors of one dtype, native GEMM shapes, no distributed or
    zero-bubble weight-gradient routing."""
    from . import gemm as G

    def _bias_ok(b, n):
        return b is None or (b.dtype == x.dtype and tuple(b.shape) == (n,))

    return (_FUSED_GELU_MLP and not any(isinstance(t, _DTensor) for t in (x, w1, w2)) and not WeightGradStore.route
            and w1.dim() == 2 and w2.dim() == 2 and w1.dtype == x.dtype == w2.dtype
            and x.shape[-1] == w1.shape[0] and w1.shape[1] == w2.shape[0] and G.enabled(x)
            and _bias_ok(b1, w1.shape[1]) and _bias_ok(b2, w2.shape[1]) and x.is_contiguous()
            and G.supported_fwd(x.reshape(-1, w1.shape[0]), w1) and w2.shape[1] % 8 == 0
            and _pass_native("fwd", x) and _pass_native("dgrad", x))


def gelu_mlp(x, w1, b1, w2, b2, approximate=True):
    """gelu(x @ W1 + b1) @ W2 + b2 with Paddle-layout weights: the fused node when gelu_mlp_ok, the plain
    composition otherwise."""
    if gelu_mlp_ok(x, w1, b1, w2, b2):
        return _GeluMLPFn.apply(x, w1, b1, w2, b2, bool(approximate))
    t = linear(x, w1, b1)
    return linear(torch.nn.functional.gelu(t, approximate="tanh" if approximate else "none"), w2, b2)


# The gate|up forward: "fused" = the GEMM's SwiGLU epilogue writes gu AND a (one kernel); "split" = the plain GEMM
# writes gu and the memory-bound SwiGLU kernel reads it back for a (measured in profiles/r5_swiglu_fwd.md)
_SWIGLU_FWD = _os.environ.get("PADDLE2_AMD_SWIGLU_FWD", "split")


class _SwiGLULinearFn(torch.autograd.Function):
    """a = swiglu(x @ W) for the packed gate|up projection W [K, 2H] (Llama MLP up half), one node:
    forward through W^T (fast hipBLASLt layout); backward's SwiGLU kernel also writes dY^T, so the weight
    gradient runs (X^T) @ (dY^T)^T without a separate dY transpose pass (csrc/kernels/elementwise.hip
    swiglu_bwd_t_kernel)."""

    @staticmethod
    def forward(ctx, x, w):
        K, H2 = w.shape
        x2 = x.reshape(-1, K)
        from . import gemm as G

        if _pass_native("fwd", x2) and G.supported_fwd(x2, w):
            if _SWIGLU_FWD == "split":
                gu = G.mm_fwd(x2, w)    # plain GEMM (its 16-B bf16 epilogue), then the SwiGLU pass
                a = swiglu(gu)
            else:
                a, gu = G.mm_swiglu(x2, w)  # one kernel: GEMM + SwiGLU epilogue (gu kept for the backward)
        else:
            gu = torch.matmul(x2, transpose2d(w).t())
            a = swiglu(gu)
        ctx.save_for_backward(x2, w, gu)
        ctx.xshape = x.shape
        ctx.gt = getattr(w, "_p2_gt", None)
        return a.view(*x.shape[:-1], H2 // 2)

    @staticmethod
    def backward(ctx, da):
        x2, w, gu = ctx.saved_tensors
        M, H2 = gu.shape
        da2 = da.reshape(M, H2 // 2).contiguous()
        dgu = torch.empty_like(gu)
        from . import gemm as G

        native_w = _pass_native("wgrad", x2) and G.supported_wgrad(x2, gu)
        if ctx.gt is not None or native_w:  # native / main-grad GEMM reads dgu in place: no dY^T image needed
            H, es = H2 // 2, gu.element_size()
            N.native().swiglu_bwd(_DT[gu.dtype], gu.data_ptr(), gu.data_ptr() + H * es, da2.data_ptr(),
                                  dgu.data_ptr(), dgu.data_ptr() + H * es, M, H, H2, H2, H2, H2, N.stream())
        else:
            dguT = torch.empty(H2, M, dtype=gu.dtype, device=gu.device)
            N.native().swiglu_bwd_t(gu.data_ptr(), da2.data_ptr(), dgu.data_ptr(), dguT.data_ptr(), M, H2 // 2, H2,
                                    N.stream())
        dx = None
        if ctx.needs_input_grad[0]:
            if _pass_native("dgrad", dgu) and G.supported_dgrad(dgu, w):
                dx = G.mm_dgrad(dgu, w).view(ctx.xshape)
            else:
                dx = torch.matmul(dgu, w.t()).view(ctx.xshape)
        dw = None
        if ctx.needs_input_grad[1]:
            if ctx.gt is not None:
                _main_grad_accumulate(ctx.gt, x2, dgu)
            elif native_w:
                dw = G.mm_wgrad_bf16(x2, dgu)
            else:
                dw = torch.matmul(transpose2d(x2), dguT.t())
        return dx, dw


class _SwiGLUMLPFn(torch.autograd.Function):
    """y = swiglu(x @ W_gu) @ W_down (Llama MLP, W_gu [K, 2H] packed gate | up) as ONE autograd node so the SwiGLU
    backward runs in the down projection's dgrad epilogue: d_a = dy @ W_down^T never leaves the fp32 accumulators,
    the epilogue reads gate / up from the saved pre-activations and writes d_gate / d_up (gemm kEpiDSwiGLU) — no
    d_a round trip and no separate SwiGLU-backward pass."""

    @staticmethod
    def forward(ctx, x, w_gu, w_down):
        from . import gemm as G

        K = w_gu.shape[0]
        x2 = x.reshape(-1, K)
        a, gu = G.mm_swiglu(x2, w_gu)
        y = G.mm_fwd(a, w_down)
        ctx.save_for_backward(x2, w_gu, w_down, a, gu)
        ctx.gts = (getattr(w_gu, "_p2_gt", None), getattr(w_down, "_p2_gt", None))
        ctx.xshape = x.shape
        return y.view(*x.shape[:-1], w_down.shape[1])

    @staticmethod
    def backward(ctx, dy):
        from . import gemm as G

        x2, w_gu, w_down, a, gu = ctx.saved_tensors
        gt_gu, gt_down = ctx.gts
        dy2 = dy.reshape(-1, w_down.shape[1]).contiguous()
        dgu = G.mm_dgrad_dswiglu(dy2, w_down, gu)
        if dgu is None:   # another dgrad schedule selected: GEMM, then the SwiGLU backward kernel
            da = G.mm_dgrad(dy2, w_down)
            M, H2 = gu.shape
            H, es = H2 // 2, gu.element_size()
            dgu = torch.empty_like(gu)
            N.native().swiglu_bwd(_DT[gu.dtype], gu.data_ptr(), gu.data_ptr() + H * es, da.data_ptr(),
                                  dgu.data_ptr(), dgu.data_ptr() + H * es, M, H, H2, H2, H2, H2, N.stream())
        dw_down = weight_grad(a, dy2, gt_down) if ctx.needs_input_grad[2] else None
        dx = G.mm_dgrad(dgu, w_gu).view(ctx.xshape) if ctx.needs_input_grad[0] else None
        dw_gu = weight_grad(x2, dgu, gt_gu) if ctx.needs_input_grad[1] else None
        return dx, dw_gu, dw_down


# Opt-in (PADDLE2_AMD_SWIGLU_MLP_NODE=1).  Measured in the Llama-2-7B step (profiles/r4_epilogue_fusions.md): the
# SwiGLU-backward epilogue takes the down dgrad from ~2.0 to 3.2 ms per layer (two reads and two writes per output
# element in the element-checked epilogue) against 0.65 ms for the separate pass: 27,071 vs 27,408 tokens/s.
_SWIGLU_MLP_NODE = _os.environ.get("PADDLE2_AMD_SWIGLU_MLP_NODE", "0") != "0"


def swiglu_mlp_ok(x, w_gu, w_down):
    from . import gemm as G

    K, H2 = w_gu.shape
    M = x.numel() // K if K else 0
    return (_SWIGLU_MLP_NODE and x.device.type == "cuda" and x.dtype == torch.bfloat16 and w_gu.dtype == x.dtype
            and w_down.dtype == x.dtype and N.use_native(x) and not isinstance(x, _DTensor)
            and not isinstance(w_gu, _DTensor) and not isinstance(w_down, _DTensor) and not WeightGradStore.route
            and x.shape[-1] == K and w_down.shape[0] == H2 // 2 and (H2 // 2) % 128 == 0 and M >= 4096
            and M % 8 == 0 and x.is_contiguous() and G.supported_fwd(x.reshape(-1, K), w_gu)
            and _pass_native("fwd", x) and _pass_native("dgrad", x) and _pass_native("swiglu", x)
            and G._variant("dgrad") == G.V7_SPREAD and w_down.shape[1] % 128 == 0)


def swiglu_mlp(x, w_gu, w_down):
    return _SwiGLUMLPFn.apply(x, w_gu, w_down)


def swiglu_linear(x, w):
    """swiglu(x @ W) with W [K, 2H] packed [gate | up]."""
    K, H2 = w.shape
    M = x.numel() // K
    if (x.device.type == "cuda" and x.dtype == torch.bfloat16 and w.dtype == x.dtype and N.use_native(x)
            and (H2 // 2) % 64 == 0 and M >= 4096 and M % 8 == 0 and _LINEAR_LAYOUT != "off"):
        return _SwiGLULinearFn.apply(x, w)
    return swiglu(linear(x, w))


# ============================================================================ fused masked softmax
def _softmax_mask_reference(x, mask, causal):
    xf = x.float()
    if causal:
        Sq, Sk = x.shape[-2], x.shape[-1]
        keep = torch.ones(Sq, Sk, dtype=torch.bool, device=x.device).tril()
        xf = xf.masked_fill(~keep, float("-inf"))
    else:
        xf = xf + mask.float()
    return torch.softmax(xf, -1).to(x.dtype)


class _SoftmaxMaskFn(torch.autograd.Function):
    """softmax(x + mask) / causal softmax over [B, H, Sq, Sk] scores (csrc/kernels/softmax_mask.hip)."""

    @staticmethod
    def forward(ctx, x, mask, causal):
        B, H, Sq, Sk = x.shape
        xc = x.contiguous()
        y = torch.empty_like(xc)
        mc = None
        if not causal:
            m = mask
            if m.dtype != x.dtype:
                # keep an fp32 mask's large negatives finite in a 16-bit x (fp16 would round -1e9 to -inf)
                m = m.float().clamp(min=torch.finfo(x.dtype).min)
            mc = m.to(x.dtype).expand(B, 1, Sq, Sk).contiguous()
        N.native().softmax_mask_fwd(_DT[x.dtype], int(causal), xc.data_ptr(), 0 if mc is None else mc.data_ptr(),
                                    y.data_ptr(), B * H * Sq, H, Sq, Sk, N.stream())
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        dyc = dy.contiguous()
        dx = torch.empty_like(y)
        Sk = y.shape[-1]
        N.native().softmax_mask_bwd(_DT[y.dtype], y.data_ptr(), dyc.data_ptr(), dx.data_ptr(), y.numel() // Sk, Sk,
                                    N.stream())
        return dx, None, None


def softmax_mask(x, mask=None, causal=False):
    """Fused attention-score softmax. ``x`` [B, H, Sq, Sk]; ``mask`` additive, broadcastable to [B, 1, Sq, Sk]
    (ignored when ``causal``: column c > row r is masked and gets probability exactly 0).  Sk <= 8192."""
    if x.dim() != 4:
        raise ValueError(f"softmax_mask expects [B, H, Sq, Sk] scores, got {tuple(x.shape)}")
    B, H, Sq, Sk = x.shape
    if causal and Sq != Sk:
        raise ValueError("softmax_mask_fuse_upper_triangle needs square scores (Sq == Sk)")
    if not causal and mask is None:
        raise ValueError("softmax_mask_fuse needs a mask")
    if Sk > 8192:
        raise ValueError(f"fused masked softmax supports key length <= 8192, got {Sk}")
    if not causal and (mask.dim() != 4 or mask.shape[1] != 1):
        # reference fused_softmax_mask_kernel.cu checks mask dim1 == 1 (one mask shared by all heads)
        raise ValueError(f"softmax_mask_fuse expects a [B, 1, Sq, Sk] mask, got {tuple(mask.shape)}")
    if N.use_native(x) and x.dtype in _DT:
        return _SoftmaxMaskFn.apply(x, mask, causal)
    return _softmax_mask_reference(x, mask, causal)


# ============================================================================ softmax cross entropy
class _SCEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels, ignore_index):
        V = logits.shape[-1]
        x2 = logits.reshape(-1, V).contiguous()
        lab = labels.reshape(-1).to(torch.int64).contiguous()
        Nr = x2.shape[0]
        if N.use_native(logits) and logits.dtype in _DT:
            C = N.native()
            mx = torch.empty(Nr, dtype=torch.float32, device=x2.device)
            se = torch.empty_like(mx)
            tgt = torch.empty_like(mx)
            C.ce_stats(_DT[x2.dtype], x2.data_ptr(), lab.data_ptr(), mx.data_ptr(), se.data_ptr(), tgt.data_ptr(), Nr,
                       V, 0, N.stream())
            lse = mx + torch.log(se)
            ctx.native = True
        else:
            xf = x2.float()
            lse = torch.logsumexp(xf, -1)
            safe = lab.clamp(0, V - 1)
            tgt = xf.gather(1, safe[:, None]).squeeze(1)
            ctx.native = False
        valid = lab != ignore_index
        loss = torch.where(valid, lse - tgt, torch.zeros_like(lse))
        ctx.save_for_backward(x2, lab, lse)
        ctx.ignore = ignore_index
        ctx.shape = logits.shape
        return loss.reshape(labels.shape)

    @staticmethod
    def backward(ctx, dloss):
        x2, lab, lse = ctx.saved_tensors
        Nr, V = x2.shape
        dl = dloss.reshape(-1).float().contiguous()
        if ctx.native:
            C = N.native()
            dx = torch.empty_like(x2)
            C.ce_bwd(_DT[x2.dtype], x2.data_ptr(), lab.data_ptr(), lse.data_ptr(), dl.data_ptr(), dx.data_ptr(), Nr, V,
                     0, ctx.ignore, 0, N.stream())
        else:
            p = torch.exp(x2.float() - lse[:, None])
            valid = lab != ctx.ignore
            p[torch.arange(Nr, device=x2.device)[valid], lab[valid]] -= 1.0
            dx = (p * (dl * valid)[:, None]).to(x2.dtype)
        return dx.reshape(ctx.shape), None, None


def softmax_cross_entropy(logits, labels, ignore_index=-100):
    """Per-token fp32 loss (0 at ignore_index); logits [..., V], labels [...]."""
    return _SCEFn.apply(logits, labels, ignore_index)


# ============================================================================ embedding
class _EmbFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, w, padding_idx, start):
        Vl, H = w.shape
        idc = ids.reshape(-1).to(torch.int64).contiguous()
        wc = w.contiguous()
        if N.use_native(w) and w.dtype in _DT and (H * w.element_size()) % 16 == 0:
            C = N.native()
            out = torch.empty(idc.numel(), H, dtype=w.dtype, device=w.device)
            C.embed_fwd(_DT[w.dtype], idc.data_ptr(), wc.data_ptr(), out.data_ptr(), idc.numel(), H, start, Vl,
                        N.stream())
            ctx.native = True
        else:
            local = idc - start
            ok = (local >= 0) & (local < Vl)
            out = wc[local.clamp(0, Vl - 1)] * ok[:, None].to(w.dtype)
            ctx.native = False
        ctx.save_for_backward(idc)
        ctx.meta = (Vl, H, padding_idx if padding_idx is not None else -(2 ** 62), start, w.dtype, ids.shape)
        return out.reshape(list(ids.shape) + [H])

    @staticmethod
    def backward(ctx, g):
        (idc,) = ctx.saved_tensors
        Vl, H, pad, start, wdt, ishape = ctx.meta
        gc = g.reshape(-1, H).contiguous()
        from ..framework.flags import flag

        if flag("FLAGS_embedding_deterministic"):
            # reproducible order: rows sorted by id, then a sort-based (atomics-free) accumulation
            local = idc - start
            ok = (local >= 0) & (local < Vl) & (idc != pad)
            li, gi = local[ok], gc[ok].float()
            order = torch.argsort(li, stable=True)
            dw32 = torch.zeros(Vl, H, dtype=torch.float32, device=g.device)
            prev = torch.are_deterministic_algorithms_enabled()
            torch.use_deterministic_algorithms(True, warn_only=True)
            try:
                dw32.index_put_((li[order],), gi[order], accumulate=True)
            finally:
                torch.use_deterministic_algorithms(prev, warn_only=True)
            return None, dw32.to(wdt), None, None
        if ctx.native:
            C = N.native()
            dw32 = torch.zeros(Vl, H, dtype=torch.float32, device=g.device)
            C.embed_bwd(_DT[gc.dtype], idc.data_ptr(), gc.data_ptr(), dw32.data_ptr(), idc.numel(), H, start, Vl, pad,
                        N.stream())
        else:
            dw32 = torch.zeros(Vl, H, dtype=torch.float32, device=g.device)
            local = idc - start
            ok = (local >= 0) & (local < Vl) & (idc != pad)
            dw32.index_add_(0, local[ok], gc[ok].float())
        return None, dw32.to(wdt), None, None


def embedding(ids, w, padding_idx=None, start=0):
    if isinstance(w, _DTensor) or isinstance(ids, _DTensor):
        return _dist_ops().embedding(ids, w, padding_idx, start)
    if padding_idx is not None and padding_idx < 0:
        padding_idx = padding_idx + w.shape[0]
    return _EmbFn.apply(ids, w, padding_idx, start)


# ============================================================================ flash attention
def _attn_reference(q, k, v, causal, scale):
    """fp32 math attention on [B, S, H, D] with GQA; returns (out, lse[B, H, Sq])."""
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    qf = q.float().transpose(1, 2)
    kf = k.float().transpose(1, 2)
    vf = v.float().transpose(1, 2)
    if Hk != Hq:
        rep = Hq // Hk
        kf = kf.repeat_interleave(rep, 1)
        vf = vf.repeat_interleave(rep, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        off = Sk - Sq
        i = torch.arange(Sq, device=q.device)[:, None]
        j = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill(j > i + off, float("-inf"))
    lse = torch.logsumexp(s, -1)
    p = torch.exp(s - lse[..., None])
    p = torch.nan_to_num(p, nan=0.0)
    out = torch.matmul(p, vf).transpose(1, 2)
    return out.to(q.dtype), lse


_ATTN_DT = {torch.bfloat16: 1, torch.float16: 2}  # csrc/kernels/common.h DType: kBF16, kF16


def _attn_dim(D):
    """Kernel head dim for D: 64 / 128 / 256 run as they are; any other D <= 256 is zero-padded to the next
    one (the padded columns add 0 to Q.K^T and produce 0 output / gradient columns)."""
    for c in (64, 128, 256):
        if D <= c:
            return c
    return None


def _pad_d(t, Dp):
    return t if t.shape[-1] == Dp else torch.nn.functional.pad(t, (0, Dp - t.shape[-1]))


def _bwd_block(D):
    return 128 if D > 128 else 256  # pd_flash_bwd_block: key-block width of the dQ partial slabs


def _row_view_ok(t):
    # [B, S, H, D] with unit stride on D, stride D on H, uniform row stride on S, batch = S*row
    B, S, H, D = t.shape
    st = t.stride()
    return st[3] == 1 and st[2] == D and st[0] == S * st[1]


class _FlashFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale):
        B, Sq, Hq, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        Dp = _attn_dim(D)
        native = (N.use_native(q) and q.dtype in _ATTN_DT and k.dtype == q.dtype and v.dtype == q.dtype
                  and Dp is not None and Hq % Hk == 0)
        if native:
            q_, k_, v_ = (_pad_d(t, Dp) for t in (q, k, v))
            q_, k_, v_ = (t if _row_view_ok(t) else t.contiguous() for t in (q_, k_, v_))
            out, lse = _flash_fwd_native(q_, k_, v_, causal, scale)
            ctx.save_for_backward(q_, k_, v_, out, lse)
            if Dp != D:
                out = out[..., :D]
        else:
            out, lse = _attn_reference(q, k, v, causal, scale)
            ctx.save_for_backward(q, k, v, out, lse)
        ctx.native, ctx.causal, ctx.scale, ctx.D = native, causal, scale, D
        return out, lse

    @staticmethod
    def backward(ctx, dout, dlse):
        q, k, v, out, lse = ctx.saved_tensors
        B, Sq, Hq, D = q.shape
        Sk, Hk = k.shape[1], k.shape[2]
        if ctx.native:
            do = _pad_d(dout, D).contiguous()
            dq = torch.empty(B, Sq, Hq, D, dtype=q.dtype, device=q.device)
            dk = torch.empty(B, Sk, Hk, D, dtype=q.dtype, device=q.device)
            dv = torch.empty(B, Sk, Hk, D, dtype=q.dtype, device=q.device)
            if not _row_view_ok(out):
                out = out.contiguous()
            assert out.stride(1) == do.stride(1), "out/dout row strides must match"
            _flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, ctx.scale, ctx.causal)
            if D != ctx.D:
                dq, dk, dv = dq[..., :ctx.D], dk[..., :ctx.D], dv[..., :ctx.D]
            return dq, dk, dv, None, None
        with torch.enable_grad():
            qq = q.detach().float().requires_grad_(True)
            kk = k.detach().float().requires_grad_(True)
            vv = v.detach().float().requires_grad_(True)
            o, _ = _attn_reference(qq, kk, vv, ctx.causal, ctx.scale)
            gq, gk, gv = torch.autograd.grad(o, (qq, kk, vv), dout.float())
        return gq.to(q.dtype), gk.to(k.dtype), gv.to(v.dtype), None, None


def flash_attention(q, k, v, causal=False, scale=None):
    """q [B, Sq, Hq, D], k/v [B, Sk, Hk, D] -> (out [B, Sq, Hq, D], lse [B, Hq, Sq] fp32)."""
    if isinstance(q, _DTensor) or isinstance(k, _DTensor):
        return _dist_ops().flash_attention(q, k, v, causal, scale)
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    return _FlashFn.apply(q, k, v, bool(causal), float(scale))


def _flash_fwd_native(q, k, v, causal, scale):
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    out = torch.empty(B, Sq, Hq, D, dtype=q.dtype, device=q.device)
    lse = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
    N.native().flash_fwd(_ATTN_DT[q.dtype], q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), lse.data_ptr(), B, Sq, Sk, Hq,
                         Hk, D, q.stride(1), k.stride(1), v.stride(1), out.stride(1), float(scale), int(causal),
                         N.stream())
    return out, lse


def dq_atomic():
    """Dense flash backward accumulates dQ with fp32 atomics into one slab unless PADDLE2_AMD_FA_DQ_ATOMIC=0
    (FLAGS_cudnn_deterministic sets it): the workspace is sized by this rule, the kernel reads the same env."""
    e = _os.environ.get("PADDLE2_AMD_FA_DQ_ATOMIC")
    return True if e is None else int(e) != 0


def _flash_bwd_native(q, k, v, out, do, lse, dq, dk, dv, scale, causal, rope=None):
    """dq/dk/dv may be token-strided views (e.g. slices of a dQKV buffer).  ``rope`` = (cos, sin) fp32 [>= S, 128]
    tables: q / k were rotate-half RoPE'd by their producer, and dq / dk come out as the gradients of the
    PRE-rotation q / k (RoPE^T folded into the dK epilogue and the dQ reduce; dense, D = 128)."""
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    bnk = _bwd_block(D)
    nkb = (Sk + bnk - 1) // bnk
    # split dQ (opt-in PADDLE2_AMD_FA_DQ_SPLIT=1; dense, D = 128; flash_attn.hip dq_gemm_kernel): the backward
    # stores dS into a compact bf16 buffer and a second kernel computes dQ = scale * dS . K — deterministic, no fp32
    # dQ slab, no atomics (slower than the fused atomic default at the Llama shape: profiles/r6_flash_dq_split.md)
    ds_n = N.native().flash_ds_elems(B, Sq, Sk, Hq, D, int(bool(causal)))
    if ds_n > 0:
        ds = torch.empty(ds_n, dtype=q.dtype, device=q.device)
        dq32 = torch.empty(0, dtype=torch.float32, device=q.device)
    else:
        ds = None
        # per-key-block dQ partials, or one atomically accumulated slab (same rule as fa_dq_atomic in flash_attn.hip)
        slabs = 1 if dq_atomic() else nkb
        dq32 = torch.empty(slabs * B * Sq * Hq * D, dtype=torch.float32, device=q.device)
    delta = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
    if rope is not None:
        cos, sin = rope
        assert D == 128 and cos.dtype == torch.float32 and cos.is_contiguous() and sin.is_contiguous() and \
            cos.shape[-1] == 128 and cos.shape[0] >= max(Sq, Sk), "RoPE^T fold: fp32 [S, 128] tables, D = 128"
        N.native().flash_bwd_set_rope(cos.data_ptr(), sin.data_ptr())
    if ds is not None:
        N.native().flash_bwd_set_ds(ds.data_ptr())
    N.native().flash_bwd(_ATTN_DT[q.dtype], q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), do.data_ptr(), lse.data_ptr(),
                         delta.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(), dq32.data_ptr(), B, Sq, Sk,
                         Hq, Hk, D, q.stride(1), k.stride(1), v.stride(1), do.stride(1), dq.stride(1), dk.stride(1),
                         dv.stride(1), float(scale), int(causal), N.stream())


# ------------------------------------------------------------- raw block primitives (ring / context parallel)
def attn_block_fwd(q, k, v, causal, scale):
    """One (query block x key block) flash forward, no autograd: (out [B, Sq, Hq, D], lse [B, Hq, Sq] fp32)."""
    if _native_attn_ok(q, k):
        q, k, v = (t if _row_view_ok(t) else t.contiguous() for t in (q, k, v))
        return _flash_fwd_native(q, k, v, causal, scale)
    return _attn_reference(q, k, v, causal, scale)


def attn_block_bwd(q, k, v, out, do, lse, causal, scale):
    """Gradients of one block product given the rows' FINAL out / lse (after merging every key block):
    P = exp(S - lse) is then exactly this block's slice of the global softmax, so the per-block dQ/dK/dV
    sum to the full-attention gradients.  Native flash bwd on the MI355X, fp32 math on CPU."""
    if _native_attn_ok(q, k):
        q, k, v, out, do = (t if _row_view_ok(t) else t.contiguous() for t in (q, k, v, out, do))
        if out.stride(1) != do.stride(1):
            out, do = out.contiguous(), do.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        _flash_bwd_native(q, k, v, out, do, lse.contiguous(), dq, dk, dv, scale, causal)
        return dq, dk, dv
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    g = Hq // Hk
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    kr, vr = kf.repeat_interleave(g, 1), vf.repeat_interleave(g, 1)
    s = torch.matmul(qf, kr.transpose(-1, -2)) * scale
    if causal:
        i = torch.arange(Sq, device=q.device)[:, None]
        j = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (Sk - Sq), float("-inf"))
    p = torch.nan_to_num(torch.exp(s - lse.float()[..., None]), nan=0.0)
    dof, of = do.float().transpose(1, 2), out.float().transpose(1, 2)
    dvr = torch.matmul(p.transpose(-1, -2), dof)
    dp = torch.matmul(dof, vr.transpose(-1, -2))
    delta = (dof * of).sum(-1, keepdim=True)
    ds = p * (dp - delta)
    dq = torch.matmul(ds, kr) * scale
    dkr = torch.matmul(ds.transpose(-1, -2), qf) * scale
    dk = dkr.view(B, Hk, g, Sk, D).sum(2)
    dv = dvr.view(B, Hk, g, Sk, D).sum(2)
    return (dq.transpose(1, 2).to(q.dtype), dk.transpose(1, 2).to(k.dtype), dv.transpose(1, 2).to(v.dtype))


# ------------------------------------------------------------- varlen (cu_seqlens) and FlashMask variants
# Same MFMA kernels, MODE-templated (csrc/kernels/flash_attn.hip kVarlen / kMask): varlen locates each
# sequence's rows through cu_seqlens (reference flash_attn_kernel.cu FlashAttnUnpaddedKernel); FlashMask
# (reference flash_attn_kernel.cu:445-494) masks per-key row intervals and skips fully masked tiles.
_MODE_DENSE, _MODE_VARLEN, _MODE_MASK = 0, 1, 2
_BIG_ROW = 1 << 30


def flashmask_intervals(startend_row_indices, causal):
    """[B, Hm, Sk, n] LTS/LTE/UTS/UTE -> [B, Hm, Sk, 4] int32 (a1, b1, a2, b2): rows in [a1, b1) U [a2, b2)
    are masked for that key column."""
    idx = startend_row_indices.to(torch.int32)
    n = idx.shape[-1]
    z = torch.zeros_like(idx[..., 0])
    big = torch.full_like(z, _BIG_ROW)
    if causal and n == 1:
        parts = (idx[..., 0], big, z, z)
    elif causal and n == 2:
        parts = (idx[..., 0], idx[..., 1], z, z)
    elif not causal and n == 2:
        parts = (idx[..., 0], big, z, idx[..., 1])
    elif not causal and n == 4:
        parts = (idx[..., 0], idx[..., 1], idx[..., 2], idx[..., 3])
    else:
        raise ValueError(f"startend_row_indices last dim {n} invalid for causal={causal}")
    return torch.stack(parts, -1).contiguous()


def _fm_tiles(fm, tile):
    """Per-tile [min a1, max a1, min b1, max b1, min a2, max a2, min b2, max b2] over `tile` keys
    -> [B*Hm, ntiles, 8]."""
    B, Hm, Sk, _ = fm.shape
    nt = (Sk + tile - 1) // tile
    pad = nt * tile - Sk
    if pad:
        fm = torch.cat([fm, fm[:, :, -1:].expand(B, Hm, pad, 4)], 2)  # edge-replicate: min/max unchanged
    f = fm.view(B * Hm, nt, tile, 4)
    mn, mx = f.amin(2), f.amax(2)
    return torch.stack([mn[..., 0], mx[..., 0], mn[..., 1], mx[..., 1], mn[..., 2], mx[..., 2], mn[..., 3],
                        mx[..., 3]], -1)


def _fm_classify(summ, rows, row_tile, Sq):
    """Class of every (row tile x key tile): 0 unmasked, 1 partial, 2 fully masked -> [B*Hm, n_row_tiles, nt]."""
    r0 = torch.arange(0, Sq, row_tile, device=summ.device, dtype=torch.int32)[None, :, None]
    r1 = (r0 + row_tile).clamp(max=Sq)
    s = summ[:, None]  # [BH, 1, nt, 8]
    full = ((s[..., 1] <= r0) & (s[..., 2] >= r1)) | ((s[..., 5] <= r0) & (s[..., 6] >= r1))
    unm = ((s[..., 0] >= r1) | (s[..., 3] <= r0)) & ((s[..., 4] >= r1) | (s[..., 7] <= r0))
    return torch.where(full, 2, torch.where(unm, 0, 1)).to(torch.int32)


_FM_PLAN_CACHE = {}


def flashmask_plan(fm, Sq):
    """Host plans for the kMask kernels.

    fwd: [B*Hm, ceil(Sq/128), 2 + ceil(Sk/64)] = (first, end) non-fully-masked key tile + class per 64-key tile;
    bwd: [B*Hm, ceil(Sq/32), ceil(Sk/256)] class per (32-row q tile, 256-key block)."""
    c64 = _fm_classify(_fm_tiles(fm, 64), None, 128, Sq)
    nt = c64.shape[-1]
    active = c64 != 2
    idx = torch.arange(nt, device=fm.device, dtype=torch.int32)
    any_a = active.any(-1)
    first = torch.where(any_a, torch.where(active, idx, nt).amin(-1), nt)
    end = torch.where(any_a, torch.where(active, idx + 1, 0).amax(-1), nt)
    fwd = torch.cat([first[..., None], end[..., None], c64], -1).to(torch.int32).contiguous()
    bwd = _fm_classify(_fm_tiles(fm, 256), None, 32, Sq).contiguous()
    return fwd, bwd


def _flashmask_prepare(startend_row_indices, causal, B, Sq, device):
    """Normalised intervals + plans, cached per mask tensor (every layer of a step shares one mask)."""
    key = (id(startend_row_indices), startend_row_indices._version, bool(causal), B, Sq, str(device))
    hit = _FM_PLAN_CACHE.get(key)
    if hit is not None and hit[0] is startend_row_indices:
        return hit[1]
    fm = flashmask_intervals(startend_row_indices.to(device), causal)
    if fm.shape[0] != B:
        fm = fm.expand(B, *fm.shape[1:]).contiguous()
    out = (fm,) + flashmask_plan(fm, Sq)
    if len(_FM_PLAN_CACHE) > 8:
        _FM_PLAN_CACHE.clear()
    _FM_PLAN_CACHE[key] = (startend_row_indices, out)
    return out


def _attn_reference_masked(q, k, v, causal, scale, fm):
    """fp32 reference with FlashMask intervals fm [B, Hm, Sk, 4]; returns (out, lse[B, H, Sq])."""
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if Hk != Hq:
        kf, vf = kf.repeat_interleave(Hq // Hk, 1), vf.repeat_interleave(Hq // Hk, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    r = torch.arange(Sq, device=q.device)[:, None]
    f = fm.to(q.device).long()[:, :, None]  # [B, Hm, 1, Sk, 4]
    masked = ((r >= f[..., 0]) & (r < f[..., 1])) | ((r >= f[..., 2]) & (r < f[..., 3]))
    if causal:
        masked = masked | (torch.arange(Sk, device=q.device)[None, :] > r + (Sk - Sq))
    s = s.masked_fill(masked, float("-inf"))
    lse = torch.logsumexp(s, -1)
    p = torch.nan_to_num(torch.exp(s - lse[..., None]), nan=0.0)
    return torch.matmul(p, vf).transpose(1, 2).to(q.dtype), lse


def _native_attn_ok(q, k, dims=(64, 128, 256)):
    return (q.device.type == "cuda" and N.use_native(q) and q.dtype in _ATTN_DT and k.dtype == q.dtype
            and q.shape[-1] in dims and q.shape[-2] % k.shape[-2] == 0)


class _FlashExtFn(torch.autograd.Function):
    """mode 0: dense [B, S, H, D]; mode 1: q/k/v packed [total, H, D] + cu_q/cu_k; mode 2: dense + FlashMask
    intervals.  ``drop`` = None or (seed32, p): in-kernel attention dropout (modes 0/1) whose keep mask is a
    counter hash of (seed, batch*head, query, key), regenerated by the backward instead of stored."""

    @staticmethod
    def forward(ctx, q, k, v, causal, scale, mode, aux, drop):
        q, k, v = q.contiguous(), k.contiguous(), v.contiguous()
        Hq, D = q.shape[-2], q.shape[-1]
        Hk = k.shape[-2]
        dargs = (0, 0, 0.0) if drop is None else (1, int(drop[0]) & 0xFFFFFFFF, float(drop[1]))
        if mode == _MODE_DENSE:
            B, Sq, _, _ = q.shape
            Sk = k.shape[1]
            lse = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
            ptrs = (0, 0, 0, 0, 0, 0, 1)
            aux = ()
        elif mode == _MODE_VARLEN:
            cu_q, cu_k, max_q, max_k = aux
            B, Sq, Sk, total_q = cu_q.numel() - 1, max_q, max_k, q.shape[0]
            lse = torch.empty(Hq, total_q, dtype=torch.float32, device=q.device)
            ptrs = (cu_q.data_ptr(), cu_k.data_ptr(), total_q, 0, 0, 0, 1)
        else:
            fm, t64, t256 = aux
            B, Sq, _, _ = q.shape
            Sk = k.shape[1]
            lse = torch.empty(B, Hq, Sq, dtype=torch.float32, device=q.device)
            ptrs = (0, 0, 0, fm.data_ptr(), t64.data_ptr(), t256.data_ptr(), fm.shape[1])
        out = torch.empty_like(q)
        N.native().flash_fwd_ext(_ATTN_DT[q.dtype], q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), lse.data_ptr(), B, Sq,
                                 Sk, Hq, Hk, D, q.stride(-3), k.stride(-3), v.stride(-3), out.stride(-3), float(scale),
                                 int(causal), mode, *ptrs, *dargs, N.stream())
        ctx.save_for_backward(q, k, v, out, lse, *aux[:2] if mode == _MODE_VARLEN else aux)
        ctx.meta = (causal, scale, mode, B, Sq, Sk, ptrs, dargs)
        return out, lse

    @staticmethod
    def backward(ctx, dout, dlse):
        q, k, v, out, lse = ctx.saved_tensors[:5]
        causal, scale, mode, B, Sq, Sk, ptrs, dargs = ctx.meta
        Hq, D = q.shape[-2], q.shape[-1]
        Hk = k.shape[-2]
        do = dout.contiguous()
        dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
        nrows = q.shape[0] if mode == _MODE_VARLEN else B * Sq
        bnk = _bwd_block(D)
        nkb = (Sk + bnk - 1) // bnk
        slabs = 1 if (mode == _MODE_DENSE and dq_atomic()) else nkb  # the kernel's fa_dq_atomic rule
        dq32 = torch.empty(slabs * nrows * Hq * D, dtype=torch.float32, device=q.device)
        delta = torch.empty_like(lse)
        N.native().flash_bwd_ext(_ATTN_DT[q.dtype], q.data_ptr(), k.data_ptr(), v.data_ptr(), out.data_ptr(), do.data_ptr(),
                                 lse.data_ptr(), delta.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr(),
                                 dq32.data_ptr(), B, Sq, Sk, Hq, Hk, D, q.stride(-3), k.stride(-3), v.stride(-3),
                                 do.stride(-3), dq.stride(-3), dk.stride(-3), dv.stride(-3), float(scale), int(causal),
                                 mode, *ptrs, *dargs, N.stream())
        return dq, dk, dv, None, None, None, None, None


def flash_attention_varlen(q, k, v, cu_seqlens_q, cu_seqlens_k, max_seqlen_q, max_seqlen_k, causal=False,
                           scale=None, dropout=0.0, seed32=None):
    """Packed variable-length attention: q [total_q, Hq, D], k/v [total_k, Hk, D], cu_seqlens [B+1].

    Returns (out [total_q, Hq, D], lse [Hq, total_q]).  Causal masks are bottom-right aligned per sequence.
    ``dropout`` > 0 masks P with the counter hash over (sequence * Hq + head, row, key) positions.
    """
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if dropout > 0.0 and seed32 is None:
        seed32 = attn_dropout_seed()
    if _native_attn_ok(q, k):
        cu_q = cu_seqlens_q.to(device=q.device, dtype=torch.int32).contiguous()
        cu_k = cu_seqlens_k.to(device=q.device, dtype=torch.int32).contiguous()
        drop = (seed32, float(dropout)) if dropout > 0.0 else None
        return _FlashExtFn.apply(q, k, v, bool(causal), float(scale), _MODE_VARLEN,
                                 (cu_q, cu_k, int(max_seqlen_q), int(max_seqlen_k)), drop)
    cq, ck = cu_seqlens_q.tolist(), cu_seqlens_k.tolist()
    outs, lses = [], []
    Hq = q.shape[1]
    for i in range(len(cq) - 1):
        qi, ki, vi = (q[cq[i]:cq[i + 1]].unsqueeze(0), k[ck[i]:ck[i + 1]].unsqueeze(0),
                      v[ck[i]:ck[i + 1]].unsqueeze(0))
        if dropout > 0.0:
            # the kernel's batch*head index is sequence * Hq + head: shift the seed-free bh counter per sequence
            ar = lambda n: torch.arange(n, dtype=torch.int64, device=q.device)  # noqa: E731
            keep = attn_dropout_keep(seed32, (i * Hq + ar(Hq)).view(1, Hq, 1, 1), ar(qi.shape[1]).view(1, 1, -1, 1),
                                     ar(ki.shape[1]).view(1, 1, 1, -1), dropout)
            o, l = _attn_reference_dropout(qi, ki, vi, causal, scale, keep, dropout)
        else:
            o, l = flash_attention(qi, ki, vi, causal, scale)
        outs.append(o.squeeze(0))
        lses.append(l.squeeze(0))
    return torch.cat(outs, 0), torch.cat(lses, -1)


def flash_attention_mask(q, k, v, startend_row_indices, causal=False, scale=None):
    """FlashMask attention on [B, S, H, D] with per-key row-interval masks ([B, Hm, Sk, n], Hm in {1, Hq})."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if _native_attn_ok(q, k, (64, 128)) and startend_row_indices.shape[1] in (1, q.shape[2]):
        aux = _flashmask_prepare(startend_row_indices, causal, q.shape[0], q.shape[1], q.device)
        return _FlashExtFn.apply(q, k, v, bool(causal), float(scale), _MODE_MASK, aux, None)
    fm = flashmask_intervals(startend_row_indices.to(q.device), causal)
    return _FlashMaskRefFn.apply(q, k, v, causal, scale, fm)


class _FlashMaskRefFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, fm):
        ctx.save_for_backward(q, k, v, fm)
        ctx.meta = (causal, scale)
        return _attn_reference_masked(q, k, v, causal, scale, fm)

    @staticmethod
    def backward(ctx, dout, dlse):
        q, k, v, fm = ctx.saved_tensors
        causal, scale = ctx.meta
        with torch.enable_grad():
            qq, kk, vv = (t.detach().float().requires_grad_(True) for t in (q, k, v))
            o, _ = _attn_reference_masked(qq, kk, vv, causal, scale, fm)
            gq, gk, gv = torch.autograd.grad(o, (qq, kk, vv), dout.float())
        return gq.to(q.dtype), gk.to(k.dtype), gv.to(v.dtype), None, None, None


# ------------------------------------------------------------- attention dropout (in-kernel, counter-based mask)
# Reference: flash_attn_kernel.cu draws the dropout mask from Philox(seed, offset) inside the kernel and
# regenerates it in the backward.  Ours keeps that contract (same (seed, offset) => same mask, no stored
# bitmask) with a 32-bit counter hash evaluated per (batch*head, query, key) element in registers
# (csrc/kernels/flash_attn.hip drop_keep); the mask functions below reproduce it bit-exactly on the host.
_M32 = 0xFFFFFFFF


def _mul32(x, c):
    """(x * c) mod 2^32 for int64 tensors x in [0, 2^32) without int64 overflow."""
    return (x * (c & 0xFFFF) + (((x * (c >> 16)) & 0xFFFF) << 16)) & _M32


def attn_dropout_threshold(p):
    """The kernel's keep threshold: float32(p) * 2^32 in float32, clamped below 2^32, truncated."""
    t = torch.tensor(float(p), dtype=torch.float32) * torch.tensor(4294967296.0, dtype=torch.float32)
    return int(min(float(t), 4294967040.0))


def attn_dropout_keep(seed32, bh, q, k, p):
    """Keep mask of drop_keep() for broadcastable int64 index tensors bh / q / k (all >= 0)."""
    x = (int(seed32) & _M32) ^ _mul32(bh, 0x27D4EB2D)
    x = (x + _mul32(q, 0x9E3779B1)) & _M32
    x = x ^ (x >> 15)
    x = _mul32(x, 0x85EBCA77)
    x = (x + _mul32(k, 0xC2B2AE3D)) & _M32
    x = x ^ (x >> 13)
    x = _mul32(x, 0x27D4EB2F)
    x = x ^ (x >> 16)
    return x >= attn_dropout_threshold(p)


def attn_dropout_mask(seed32, B, H, Sq, Sk, p, device="cpu"):
    """[B, H, Sq, Sk] bool keep mask of the dense kernel (batch*head index b * H + h)."""
    ar = lambda n: torch.arange(n, dtype=torch.int64, device=device)  # noqa: E731
    return attn_dropout_keep(seed32, ar(B * H).view(B, H, 1, 1), ar(Sq).view(1, 1, Sq, 1), ar(Sk).view(1, 1, 1, Sk), p)


def attn_dropout_seed(fixed_seed_offset=None):
    """32-bit kernel seed from a Philox (seed, offset) pair: ``fixed_seed_offset`` when given, else the current
    device generator's (seed, offset) -- so RNG-tracker states (TP local/global seeds) decorrelate the mask --
    which is advanced like a torch dropout call; the global paddle (seed, offset) counter on CPU."""
    if fixed_seed_offset is not None:
        fso = fixed_seed_offset
        fso = fso._t if hasattr(fso, "_t") else fso
        seed, off = (int(v) for v in (fso.tolist() if isinstance(fso, torch.Tensor) else fso))
    else:
        seed = off = None
        if torch.cuda.is_available():
            try:
                g = torch.cuda.default_generators[torch.cuda.current_device()]
                seed, off = g.initial_seed(), g.get_offset()
                g.set_offset(off + 4)
            except (AttributeError, RuntimeError):
                seed = None
        if seed is None:
            from ..framework.random import next_philox

            seed, off = next_philox(4)
    m64 = (1 << 64) - 1
    x = (seed * 0x9E3779B97F4A7C15 + off * 0xD1B54A32D192ED03 + 0x632BE59BD9B4E019) & m64
    x ^= x >> 31
    x = (x * 0xBF58476D1CE4E5B9) & m64
    x ^= x >> 27
    return x & _M32


def _attn_reference_dropout(q, k, v, causal, scale, keep, p):
    """fp32 attention with the dropout keep mask [B, Hq, Sq, Sk] applied to P (not to the row sums)."""
    B, Sq, Hq, D = q.shape
    Sk, Hk = k.shape[1], k.shape[2]
    qf, kf, vf = q.float().transpose(1, 2), k.float().transpose(1, 2), v.float().transpose(1, 2)
    if Hk != Hq:
        kf, vf = kf.repeat_interleave(Hq // Hk, 1), vf.repeat_interleave(Hq // Hk, 1)
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if causal:
        i = torch.arange(Sq, device=q.device)[:, None]
        j = torch.arange(Sk, device=q.device)[None, :]
        s = s.masked_fill(j > i + (Sk - Sq), float("-inf"))
    lse = torch.logsumexp(s, -1)
    pr = torch.nan_to_num(torch.exp(s - lse[..., None]), nan=0.0)
    pr = pr * keep.to(pr.device) / (1.0 - p)
    return torch.matmul(pr, vf).transpose(1, 2).to(q.dtype), lse


class _FlashDropRefFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, causal, scale, p, seed32):
        keep = attn_dropout_mask(seed32, q.shape[0], q.shape[2], q.shape[1], k.shape[1], p, q.device)
        ctx.save_for_backward(q, k, v, keep)
        ctx.meta = (causal, scale, p)
        return _attn_reference_dropout(q, k, v, causal, scale, keep, p)

    @staticmethod
    def backward(ctx, dout, dlse):
        q, k, v, keep = ctx.saved_tensors
        causal, scale, p = ctx.meta
        with torch.enable_grad():
            qq, kk, vv = (t.detach().float().requires_grad_(True) for t in (q, k, v))
            o, _ = _attn_reference_dropout(qq, kk, vv, causal, scale, keep, p)
            gq, gk, gv = torch.autograd.grad(o, (qq, kk, vv), dout.float())
        return gq.to(q.dtype), gk.to(k.dtype), gv.to(v.dtype), None, None, None, None


def flash_attention_dropout(q, k, v, p, causal=False, scale=None, seed32=None):
    """Attention with dropout on the softmax probabilities (upscale_in_train): q [B, Sq, Hq, D], k/v [B, Sk, Hk, D]
    -> (out, lse).  The MI355X path runs the DROP variant of the flash kernels (mask regenerated in the backward);
    elsewhere an fp32 reference with the bit-identical mask."""
    if scale is None:
        scale = 1.0 / math.sqrt(q.shape[-1])
    if seed32 is None:
        seed32 = attn_dropout_seed()
    if not 0.0 < p < 1.0:
        raise ValueError(f"dropout probability must be in (0, 1), got {p}")
    if _native_attn_ok(q, k):
        return _FlashExtFn.apply(q, k, v, bool(causal), float(scale), _MODE_DENSE, None, (seed32, float(p)))
    return _FlashDropRefFn.apply(q, k, v, bool(causal), float(scale), float(p), int(seed32))


class _QKVRopeAttnFn(torch.autograd.Function):
    """Fused QKV split -> RoPE(q, k) -> causal flash attention, one autograd node.

    Forward reads q/k/v straight out of the fused projection output ``qkv`` [B, S, Hq+2Hk, D]
    (token-strided views, no split copies); backward writes dV, RoPE^T(dQ), RoPE^T(dK) straight
    into a single dQKV buffer — no zero-fill + slice-add of per-view gradients.
    """

    @staticmethod
    def forward(ctx, qkv, nh, nkv, cos, sin, pos, causal, scale):
        B, S, _, D = qkv.shape
        q_in = qkv[:, :, :nh]
        k_in = qkv[:, :, nh:nh + nkv]
        v = qkv[:, :, nh + nkv:]
        q = _rope_apply(q_in, cos, sin, pos, 0, False, False)
        k = _rope_apply(k_in, cos, sin, pos, 0, False, False)
        out, lse = _flash_fwd_native(q, k, v, causal, scale)
        ctx.save_for_backward(q, k, qkv, out, lse, cos, sin, pos)
        ctx.meta = (nh, nkv, causal, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, qkv, out, lse, cos, sin, pos = ctx.saved_tensors
        nh, nkv, causal, scale = ctx.meta
        v = qkv[:, :, nh + nkv:]
        dqkv = torch.empty_like(qkv)
        if pos is None and q.shape[-1] == 128 and _ROPE_BWD_IN_FLASH:
            # RoPE^T inside the flash backward: dQ / dK land in dQKV already un-rotated (no RoPE passes)
            _flash_bwd_native(q, k, v, out, dout.contiguous(), lse, dqkv[:, :, :nh], dqkv[:, :, nh:nh + nkv],
                              dqkv[:, :, nh + nkv:], scale, causal, rope=(cos, sin))
            return dqkv, None, None, None, None, None, None, None
        dq = torch.empty_like(q)
        dk = torch.empty_like(k)
        _flash_bwd_native(q, k, v, out, dout.contiguous(), lse, dq, dk, dqkv[:, :, nh + nkv:], scale, causal)
        _rope_apply(dq, cos, sin, pos, 0, False, True, out=dqkv[:, :, :nh])
        _rope_apply(dk, cos, sin, pos, 0, False, True, out=dqkv[:, :, nh:nh + nkv])
        return dqkv, None, None, None, None, None, None, None


# PADDLE2_AMD_ROPE_BWD_IN_FLASH=0: RoPE^T as separate passes after the flash backward (A/B switch)
_ROPE_BWD_IN_FLASH = _os.environ.get("PADDLE2_AMD_ROPE_BWD_IN_FLASH", "1") != "0"


class _QKVProjRopeAttnFn(torch.autograd.Function):
    """x -> qkv = RoPE_{q,k}(x @ W) -> causal flash attention as ONE autograd node (Llama's fused QKV path).

    Forward: the rotation runs in the QKV GEMM epilogue (gemm7.hip kEpiRope) and the attention reads the rotated
    qkv in place.  Backward: the flash backward writes dV and the gradients of the PRE-rotation q / k straight into
    one dQKV buffer (RoPE^T folded into its dK epilogue and dQ reduce), which feeds the projection's dgrad / wgrad
    directly — no RoPE kernel and no rotated copies in either direction."""

    @staticmethod
    def forward(ctx, x, w, cos, sin, nh, nkv, seq, scale):
        from . import gemm as G

        K = w.shape[0]
        x2 = x.reshape(-1, K)
        y = G.mm_fwd_rope(x2, w, cos, sin, (nh + nkv) * 128, seq)
        if y is None:
            y = G.mm_fwd(x2, w)
            y4 = y.view(-1, seq, w.shape[1] // 128, 128)
            y4[:, :, :nh + nkv].copy_(_rope_apply(y4[:, :, :nh + nkv], cos, sin, None, 0, False, False))
        qkv = y.view(-1, seq, nh + 2 * nkv, 128)
        out, lse = _flash_fwd_native(qkv[:, :, :nh], qkv[:, :, nh:nh + nkv], qkv[:, :, nh + nkv:], True, scale)
        ctx.save_for_backward(x2, w, cos, sin, qkv, out, lse)
        ctx.meta = (x.shape, nh, nkv, scale)
        ctx.gt = getattr(w, "_p2_gt", None)
        return out

    @staticmethod
    def backward(ctx, dout):
        from . import gemm as G

        x2, w, cos, sin, qkv, out, lse = ctx.saved_tensors
        xshape, nh, nkv, scale = ctx.meta
        dqkv = torch.empty_like(qkv)
        _flash_bwd_native(qkv[:, :, :nh], qkv[:, :, nh:nh + nkv], qkv[:, :, nh + nkv:], out, dout.contiguous(), lse,
                          dqkv[:, :, :nh], dqkv[:, :, nh:nh + nkv], dqkv[:, :, nh + nkv:], scale, True,
                          rope=(cos, sin))
        d2 = dqkv.view(-1, w.shape[1])
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = G.mm_dgrad(d2, w).view(xshape)
        if ctx.needs_input_grad[1]:
            dw = weight_grad(x2, d2, ctx.gt)
        return dx, dw, None, None, None, None, None, None


def qkv_proj_rope_attention(x, w, cos, sin, nh, nkv, seq, scale=None):
    """Fused QKV projection + RoPE + causal attention (see _QKVProjRopeAttnFn); x [B, S, K] -> [B, S, nh, 128].
    Callers check qkv_rope_linear_ok first; cos / sin are fp32 [seq, 128]."""
    if scale is None:
        scale = 1.0 / math.sqrt(128)
    return _QKVProjRopeAttnFn.apply(x, w, cos, sin, nh, nkv, seq, float(scale))


class _QKVRopeLinearFn(torch.autograd.Function):
    """qkv = RoPE_{q,k}(x @ W) for the fused QKV projection (W [K, (Hq+2Hk) * 128]): the rotation of the q / k heads
    runs in the GEMM epilogue on the fp32 accumulators (gemm7.hip kEpiRope), so neither a RoPE kernel nor rotated
    q / k copies exist in the forward; the attention then reads the rotated qkv in place (_QKVAttnFn).  Backward:
    RoPE^T on the q / k columns of the incoming gradient, then the projection's dgrad / wgrad."""

    @staticmethod
    def forward(ctx, x, w, cos, sin, nq_heads, seq):
        from . import gemm as G

        K = w.shape[0]
        x2 = x.reshape(-1, K)
        rope_cols = nq_heads * 128
        y = G.mm_fwd_rope(x2, w, cos, sin, rope_cols, seq)
        if y is None:   # another GEMM schedule selected: GEMM, then RoPE on the q / k heads
            y = G.mm_fwd(x2, w)
            y4 = y.view(-1, seq, w.shape[1] // 128, 128)
            y4[:, :, :nq_heads].copy_(_rope_apply(y4[:, :, :nq_heads], cos, sin, None, 0, False, False))
        ctx.save_for_backward(x2, w, cos, sin)
        ctx.meta = (x.shape, nq_heads, seq)
        ctx.gt = getattr(w, "_p2_gt", None)
        return y.view(*x.shape[:-1], w.shape[1])

    @staticmethod
    def backward(ctx, dy):
        from . import gemm as G

        x2, w, cos, sin = ctx.saved_tensors
        xshape, nq, seq = ctx.meta
        Nn = w.shape[1]
        dy4 = dy.reshape(-1, seq, Nn // 128, 128)
        dpre = torch.empty(dy4.shape, dtype=dy.dtype, device=dy.device)
        _rope_apply(dy4[:, :, :nq], cos, sin, None, 0, False, True, out=dpre[:, :, :nq])
        dpre[:, :, nq:].copy_(dy4[:, :, nq:])
        d2 = dpre.view(-1, Nn)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = G.mm_dgrad(d2, w).view(xshape)
        if ctx.needs_input_grad[1]:
            dw = weight_grad(x2, d2, ctx.gt)
        return dx, dw, None, None, None, None


def qkv_rope_linear_ok(x, w, bias, head_dim, pos):
    from . import gemm as G

    return (head_dim == 128 and bias is None and pos is None and not isinstance(x, _DTensor)
            and not isinstance(w, _DTensor) and not WeightGradStore.route and w.dim() == 2
            and w.dtype == x.dtype and x.shape[-1] == w.shape[0] and G.enabled(x) and x.is_contiguous()
            and G.supported_fwd(x.reshape(-1, w.shape[0]), w) and w.shape[1] % 128 == 0
            and _pass_native("fwd", x) and _pass_native("dgrad", x) and _ROPE_IN_GEMM)


# RoPE in the QKV GEMM epilogue: opt-in.  Measured in the Llama-2-7B step (profiles/r4_rope_fusion.md) the rotating
# epilogue costs the QKV GEMM 0.73 ms per layer (1.45 -> 1.10 PF/s) against 0.2 ms for the separate RoPE pass:
# 27,221 vs 27,521 tokens/s.  The backward's RoPE^T stays folded into the flash backward either way.
_ROPE_IN_GEMM = _os.environ.get("PADDLE2_AMD_ROPE_IN_GEMM", "0") != "0"


class _QKVAttnFn(torch.autograd.Function):
    """Fused QKV split -> flash attention (no rotary; GPT): q/k/v are token-strided views of ``qkv``
    [B, S, Hq+2Hk, D] and the backward writes dQ / dK / dV straight into one dQKV buffer (the per-view slice
    backward was 3 zero-fills + 3 strided copies / adds per layer: 13 ms of the GPT-3 13B step)."""

    @staticmethod
    def forward(ctx, qkv, nh, nkv, causal, scale):
        q, k, v = qkv[:, :, :nh], qkv[:, :, nh:nh + nkv], qkv[:, :, nh + nkv:]
        out, lse = _flash_fwd_native(q, k, v, causal, scale)
        ctx.save_for_backward(qkv, out, lse)
        ctx.meta = (nh, nkv, causal, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        qkv, out, lse = ctx.saved_tensors
        nh, nkv, causal, scale = ctx.meta
        dqkv = torch.empty_like(qkv)
        _flash_bwd_native(qkv[:, :, :nh], qkv[:, :, nh:nh + nkv], qkv[:, :, nh + nkv:], out, dout.contiguous(), lse,
                          dqkv[:, :, :nh], dqkv[:, :, nh:nh + nkv], dqkv[:, :, nh + nkv:], scale, causal)
        return dqkv, None, None, None, None


def qkv_attention(qkv, num_heads, num_kv_heads, causal=True, scale=None):
    """qkv [B, S, Hq+2Hk, D] (fused projection output) -> attention output [B, S, Hq, D], no rotary."""
    D = qkv.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    if (qkv.device.type == "cuda" and N.use_native(qkv) and qkv.dtype in _ATTN_DT and D in (64, 128, 256)
            and num_heads % num_kv_heads == 0 and qkv.stride(-1) == 1 and qkv.stride(-2) == D
            and qkv.stride(0) == qkv.shape[1] * qkv.stride(1)):
        return _QKVAttnFn.apply(qkv, num_heads, num_kv_heads, bool(causal), float(scale))
    o, _ = flash_attention(qkv[:, :, :num_heads], qkv[:, :, num_heads:num_heads + num_kv_heads],
                           qkv[:, :, num_heads + num_kv_heads:], causal, scale)
    return o


def qkv_rope_attention(qkv, num_heads, num_kv_heads, cos, sin, position_ids=None, causal=True, scale=None):
    """qkv [B, S, Hq+2Hk, D] (fused projection output) -> attention output [B, S, Hq, D]."""
    D = qkv.shape[-1]
    if scale is None:
        scale = 1.0 / math.sqrt(D)
    native = (qkv.device.type == "cuda" and N.use_native(qkv) and qkv.dtype in _ATTN_DT and qkv.dtype in _DT
              and D in (64, 128, 256)
              and num_heads % num_kv_heads == 0)
    cos = cos.reshape(-1, D).float().contiguous()
    sin = sin.reshape(-1, D).float().contiguous()
    pos = None if position_ids is None else position_ids.to(torch.int64).contiguous()
    if native:
        return _QKVRopeAttnFn.apply(qkv, num_heads, num_kv_heads, cos, sin, pos, bool(causal), float(scale))
    q = rope(qkv[:, :, :num_heads], cos, sin, pos, 0)
    k = rope(qkv[:, :, num_heads:num_heads + num_kv_heads], cos, sin, pos, 0)
    o, _ = flash_attention(q, k, qkv[:, :, num_heads + num_kv_heads:], causal, scale)
    return o


# Static-graph capture: each native-kernel entry point is recorded as ONE op when called on symbolic
# tensors (paddle2_amd.static.graph), so executed Programs use the same HIP kernels as dygraph.
from ..static.graph import graph_op as _graph_op  # noqa: E402

rms_norm = _graph_op(rms_norm)
layer_norm = _graph_op(layer_norm)
swiglu = _graph_op(swiglu)
rope = _graph_op(rope)
softmax_cross_entropy = _graph_op(softmax_cross_entropy)
embedding = _graph_op(embedding)
flash_attention = _graph_op(flash_attention)
qkv_rope_attention = _graph_op(qkv_rope_attention)


# ============================================================================ BatchNorm (+add +ReLU), channels-last
class _BNActFn(torch.autograd.Function):
    """Training-mode BN over the last (channel) dim of a contiguous [..., C] tensor, with the
    residual add and ReLU fused (csrc/kernels/batch_norm.hip)."""

    @staticmethod
    def forward(ctx, x, weight, bias, z, running_mean, running_var, momentum, eps, relu):
        C_ = N.native()
        Cn = x.shape[-1]
        M = x.numel() // Cn
        dt = _DT[x.dtype]
        y = torch.empty_like(x)
        ws = torch.empty(C_.bn_workspace(dt, M, Cn) + 3 * Cn, dtype=torch.float32, device=x.device)
        mean = torch.empty(Cn, dtype=torch.float32, device=x.device)
        invstd = torch.empty_like(mean)
        w32 = weight.float().contiguous() if weight is not None else None
        b32 = bias.float().contiguous() if bias is not None else None
        C_.bn_fwd_train(dt, x.data_ptr(), N.ptr(z), y.data_ptr(), M, Cn, running_mean.data_ptr(),
                        running_var.data_ptr(), N.ptr(w32), N.ptr(b32), float(momentum), float(eps),
                        mean.data_ptr(), invstd.data_ptr(), ws.data_ptr(), int(relu), 1, N.stream())
        ctx.save_for_backward(x, y if relu else None, mean, invstd, w32)
        ctx.relu, ctx.has_z = relu, z is not None
        ctx.wdt = weight.dtype if weight is not None else None
        ctx.bdt = bias.dtype if bias is not None else None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, mean, invstd, w32 = ctx.saved_tensors
        C_ = N.native()
        Cn = x.shape[-1]
        M = x.numel() // Cn
        dt = _DT[x.dtype]
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        dz = torch.empty_like(x) if (ctx.has_z and ctx.relu) else None
        dg = torch.empty(Cn, dtype=torch.float32, device=x.device)
        db = torch.empty_like(dg)
        ws = torch.empty(C_.bn_workspace(dt, M, Cn) + 3 * Cn, dtype=torch.float32, device=x.device)
        C_.bn_bwd(dt, dy.data_ptr(), x.data_ptr(), N.ptr(y), mean.data_ptr(), invstd.data_ptr(), N.ptr(w32),
                  dx.data_ptr(), N.ptr(dz), dg.data_ptr(), db.data_ptr(), M, Cn, ws.data_ptr(), int(ctx.relu),
                  N.stream())
        if ctx.has_z and not ctx.relu:
            dz = dy
        return (dx, dg.to(ctx.wdt) if ctx.wdt is not None else None, db.to(ctx.bdt) if ctx.bdt is not None else None,
                dz, None, None, None, None, None)


def _bn_act_reference(x, running_mean, running_var, weight, bias, training, momentum, eps, relu, residual):
    t = x.movedim(-1, 1)
    y = F.batch_norm(t, running_mean, running_var, weight, bias, training, 1.0 - momentum, eps).movedim(1, -1)
    if residual is not None:
        y = y + residual
    return torch.relu(y) if relu else y


def batch_norm_act(x, running_mean, running_var, weight=None, bias=None, training=True, momentum=0.9, eps=1e-5,
                   act=None, residual=None):
    """y = act(BN(x) [+ residual]) for a channels-last [..., C] tensor (paddle momentum convention:
    running = momentum * running + (1 - momentum) * batch).  On the MI355X this is the fused HIP
    kernel whenever x is channels-last contiguous with fp32 running stats; otherwise the composite
    PyTorch reference (F.batch_norm + add + relu)."""
    if act not in (None, "relu"):
        raise ValueError(f"fused batch norm supports act in (None, 'relu'), got {act!r}")
    relu = act == "relu"
    Cn = x.shape[-1]
    ok = (x.device.type == "cuda" and N.use_native(x) and x.dtype in _DT and x.is_contiguous()
          and Cn % (4 if x.dtype == torch.float32 else 8) == 0
          and running_mean.dtype == torch.float32 and running_var.dtype == torch.float32
          and running_mean.is_contiguous() and running_var.is_contiguous()
          and (residual is None or (residual.shape == x.shape and residual.dtype == x.dtype)))
    if ok and N.use_native(x):
        if residual is not None:
            residual = residual.contiguous()
        if training:
            return _BNActFn.apply(x, weight, bias, residual, running_mean, running_var, momentum, eps, relu)
        if not (torch.is_grad_enabled() and (x.requires_grad or (weight is not None and weight.requires_grad))):
            inv = torch.rsqrt(running_var + eps)
            scale = inv * (weight.float() if weight is not None else 1.0)
            shift = (bias.float() if bias is not None else 0.0) - running_mean * scale
            scale = scale.contiguous() if torch.is_tensor(scale) else torch.full_like(running_mean, scale)
            shift = shift.contiguous()
            y = torch.empty_like(x)
            N.native().bn_apply(_DT[x.dtype], x.data_ptr(), N.ptr(residual), y.data_ptr(), x.numel() // Cn, Cn,
                                scale.data_ptr(), shift.data_ptr(), int(relu), N.stream())
            return y
    return _bn_act_reference(x, running_mean, running_var, weight, bias, training, momentum, eps, relu, residual)
