"""FP8 (OCP e4m3fn / e5m2) linear layers with delayed scaling on MI355X.

Reference: the reference's fp8 GEMM entry ``fp8_fp8_half_gemm_fused`` (python/paddle/tensor/
linalg.py:329 -> phi/kernels/fusion/gpu/fp8_gemm) with per-tensor scales; SURVEY §7.2 item 8
("fp8 e4m3/e5m2 GEMM with per-tensor scales plus an amax history recipe").

Recipe (HYBRID format): forward operands x, W in e4m3fn; the output gradient in e5m2.  Each
tensor role keeps an amax history on the device; the scale used for a cast is derived from the
history BEFORE the cast (delayed scaling), and the cast kernel (csrc/kernels/fp8.hip) records the
tensor's amax in the same pass, so quantization is one fused read of the bf16 tensor — plus the
transposed copy the column-major B operand needs.  The GEMMs run on the hand-written K=128 fp8 MFMA kernel
(csrc/kernels/gemm8.hip, both operands K-major, the inverse scales as device dequant factors, bf16 out);
shapes outside its domain (K % 256) go to hipBLASLt through ``torch._scaled_mm``.
A CPU emulation (quantize -> dequantize -> fp32 matmul) keeps the recipe testable without a GPU.
"""
from __future__ import annotations

import os

import torch

from ..static.graph import graph_op as _graph_op
from . import _native as N

E4M3 = torch.float8_e4m3fn
E5M2 = torch.float8_e5m2
_MAX = {E4M3: 448.0, E5M2: 57344.0}
AMAX_SLOTS = 64   # csrc/kernels/fp8.hip kAmaxSlots


class FP8TensorMeta:
    """Device-resident delayed-scaling state of one tensor role."""

    def __init__(self, fmt=E4M3, history_len=16, margin=0, device=None):
        dev = device or torch.device("cpu")
        self.fmt = fmt
        self.history = torch.zeros(history_len, dtype=torch.float32, device=dev)
        # AMAX_SLOTS floats: the native cast kernels spread their per-workgroup atomicMax over the slots
        # (csrc/kernels/fp8.hip kAmaxSlots); update() folds them
        self.amax = torch.zeros(AMAX_SLOTS, dtype=torch.float32, device=dev)
        self.scale = torch.ones(1, dtype=torch.float32, device=dev)
        self.inv_scale = torch.ones(1, dtype=torch.float32, device=dev)
        self.margin = margin
        self.initialized = False

    def init_from(self, x):
        """First use: no history yet, so scale from the tensor itself (just-in-time) instead of 1.0 —
        otherwise the first steps' tiny gradients underflow e5m2 and the early updates are lost."""
        amax = x.detach().abs().amax().float().reshape(1)
        s = torch.where(amax > 0, _MAX[self.fmt] / amax / 2 ** self.margin, torch.ones_like(amax))
        self.scale.copy_(s)
        self.inv_scale.copy_(1.0 / s)
        self.initialized = True

    # Host-visible reads of a role whose update is still queued (defer_update) launch the queue first.
    def _settled(name):
        key = "_" + name

        def get(self):
            if id(self) in _PENDING_IDS:
                flush_updates()
            return self.__dict__[key]

        def put(self, v):
            self.__dict__[key] = v
        return property(get, put)

    history = _settled("history")
    amax = _settled("amax")
    scale = _settled("scale")
    inv_scale = _settled("inv_scale")
    del _settled

    def to(self, device):
        for k in ("history", "amax", "scale", "inv_scale"):
            setattr(self, k, getattr(self, k).to(device))
        return self

    def update(self, snap=None):
        """Roll the history, recompute scale = fp8_max / max(history) / 2^margin, reset amax.  ``snap``: a 1-float
        tensor that receives the inverse scale in force BEFORE the update (what this step's cast used)."""
        update_metas([(self, snap)])

    def _native_role(self, snap):
        return (self.history.data_ptr(), self.history.numel(), self.amax.data_ptr(), self.scale.data_ptr(),
                self.inv_scale.data_ptr(), N.ptr(snap), _MAX[self.fmt], float(2 ** self.margin))

    def _update_ref(self, snap=None):
        if snap is not None:
            snap.copy_(self.inv_scale.reshape(snap.shape))
        self.history.copy_(torch.roll(self.history, 1))
        self.history[0] = self.amax.max()
        m = self.history.max()
        if float(m) > 0 and torch.isfinite(m):
            self.scale.fill_(_MAX[self.fmt] / float(m) / 2 ** self.margin)
        self.inv_scale.copy_(1.0 / self.scale)
        self.amax.zero_()


_CODE = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2}


_MAX_ROLES = 16   # csrc/kernels/fp8.hip kMaxMetas
# GPU role updates deferred by defer_update(): launched in batches of _MAX_ROLES, or as soon as one of the pending
# roles is cast again (its next cast must see the rolled scale) — 480 per-role updates of the GPT-3 13B fp8 step
# become ~30 launches.  Stream order keeps every update after the casts that recorded its amax.
DEFER_UPDATES = os.environ.get("PADDLE2_AMD_FP8_DEFER", "1") != "0"
_PENDING = []
_PENDING_IDS = set()


def update_metas(pairs):
    """[(meta, snap or None)]: every role's delayed-scaling update, now — on the GPU in as few launches as possible
    (up to 16 roles each), each snap receiving that role's pre-update inverse scale."""
    gpu = [p for p in pairs if p[0].amax.device.type == "cuda" and N.use_native(p[0].amax)]
    for i in range(0, len(gpu), _MAX_ROLES):
        N.native().fp8_update_scale([m._native_role(s) for m, s in gpu[i:i + _MAX_ROLES]], N.stream())
    for m, s in pairs:
        if not (m.amax.device.type == "cuda" and N.use_native(m.amax)):
            m._update_ref(s)


def defer_update(pairs):
    """Queue the updates of GPU roles (CPU roles update at once); the snaps are written when the batch launches,
    which is before anything reads them (the backward of the same linear runs after later casts or a flush)."""
    if not DEFER_UPDATES or (pairs[0][0].amax.is_cuda and torch.cuda.is_current_stream_capturing()):
        # (a HIP-graph capture must contain its own updates: a queue flushed after the capture ends would run once,
        # eagerly, and never on replay; a queue left by eager steps raises here instead of entering the graph)
        flush_updates()
        update_metas(pairs)
        return
    now = []
    for m, s in pairs:
        if m.amax.device.type == "cuda" and N.use_native(m.amax) and id(m) not in _PENDING_IDS:
            _PENDING.append((m, s))
            _PENDING_IDS.add(id(m))
        else:
            now.append((m, s))
    if now:
        flush_updates()
        update_metas(now)
    if len(_PENDING) >= _MAX_ROLES:
        flush_updates()


def flush_updates():
    """Launch every queued role update (call before reading a pending role's scale / history on the host)."""
    if _PENDING:
        _check_not_capturing()
        batch = list(_PENDING)
        _PENDING.clear()
        _PENDING_IDS.clear()
        update_metas(batch)


def _check_not_capturing():
    """Updates queued by EAGER steps must never be flushed into a HIP-graph capture: the graph would replay that
    stale update (one extra history roll per replay) and write pre-update inverse scales into snap tensors that
    live outside the graph's pool.  Every capture entry of the framework calls before_capture() first; a capture
    started elsewhere with updates still queued is an error, not a silent corruption."""
    if _PENDING and torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
        raise RuntimeError("fp8: delayed-scaling updates from eager steps are still queued at HIP-graph capture; "
                           "call paddle2_amd.ops.fp8.before_capture() (or flush_updates()) before capturing")


def before_capture():
    """Settle the eager update queue before a HIP-graph capture begins (executor, device.CUDAGraph, serving decode):
    inside a capture every update is then recorded by the cast that needs it, once per replay."""
    flush_updates()


def _dt_code(t):
    return _CODE[t.dtype]


def cast(x2, meta: FP8TensorMeta, transpose=False, keep_rowmajor=True, colsum=False):
    """x2 [R, C] -> (q [R, C] or None, qT [C, R] or None) in meta.fmt, recording amax into meta.  ``colsum``: also
    return the unscaled fp32 column sums of every 64-row block ([ceil(R/64), C], summed in the same pass over x2 —
    the fp8 linear's bias gradient), or None where the kernel path has no such output."""
    R, C = x2.shape
    if _PENDING and x2.is_cuda:
        _check_not_capturing()
    if id(meta) in _PENDING_IDS:
        flush_updates()   # this role's previous update must land before its scale is used again
    if not meta.initialized:
        meta.init_from(x2)
    if x2.device.type == "cuda" and N.use_native(x2):
        x2 = x2.contiguous()
        q = torch.empty(R, C, dtype=torch.uint8, device=x2.device) if (keep_rowmajor or not transpose) else None
        qT = torch.empty(C, R, dtype=torch.uint8, device=x2.device) if transpose else None
        part = torch.empty((R + 63) // 64, C, dtype=torch.float32, device=x2.device) if colsum else None
        done = N.native().fp8_cast(_dt_code(x2), int(meta.fmt == E5M2), x2.data_ptr(), N.ptr(q), N.ptr(qT), R, C,
                                   meta.scale.data_ptr(), meta.amax.data_ptr(), N.stream(), N.ptr(part))
        if not done:   # no fused column sums on this path: plain cast
            part = None
            N.native().fp8_cast(_dt_code(x2), int(meta.fmt == E5M2), x2.data_ptr(), N.ptr(q), N.ptr(qT), R, C,
                                meta.scale.data_ptr(), meta.amax.data_ptr(), N.stream())
        out = (None if q is None else q.view(meta.fmt)), (None if qT is None else qT.view(meta.fmt))
        return (*out, part) if colsum else out
    xf = x2.float()
    meta.amax[:1].copy_(torch.maximum(meta.amax[:1], xf.abs().max().reshape(1)))
    q = (xf * meta.scale).clamp(-_MAX[meta.fmt], _MAX[meta.fmt]).to(meta.fmt)
    out = (q if (keep_rowmajor or not transpose) else None), (q.t().contiguous() if transpose else None)
    return (*out, None) if colsum else out


# "auto" (default): per (formats, M, N, K) the faster of the native kernel and hipBLASLt, timed on device events the
# first time the shape is seen (the native kernel has no split-K: at M = 4096 its 256 x 256 tiles leave a partial
# last wave that hipBLASLt's stream-K does not — profiles/r4_secondary_configs.md); "native": the hand-written
# K=128 fp8 MFMA GEMM (csrc/kernels/gemm8.hip) for every shape in its domain; "blas": hipBLASLt (torch._scaled_mm)
GEMM = os.environ.get("PADDLE2_AMD_FP8_GEMM", "auto")
_ROUTE = {}
_CUS = {}
_FMT = {E4M3: 0, E5M2: 1}
# (A format, B format, output) pairs the kernel is instantiated for: forward e4m3 x e4m3, dgrad e5m2 x e4m3,
# wgrad e4m3 x e5m2 (bf16 or fp32 dW)
_NATIVE_CASES = {(0, 0, torch.bfloat16), (1, 0, torch.bfloat16), (0, 1, torch.bfloat16), (0, 1, torch.float32)}


def _cus(dev):
    c = _CUS.get(dev.index)
    if c is None:
        c = _CUS[dev.index] = torch.cuda.get_device_properties(dev).multi_processor_count
    return c


# tile-group height of the native fp8 GEMM's tile order (rows of 256 x 256 tiles walked together; 4 by default)
GROUP_M = int(os.environ.get("PADDLE2_AMD_FP8_GROUP_M", "4"))

# tail split-K (gemm_tn.h: a last partial wave of <= CUs / 2 tiles as K-slices + an fp32 fix-up) on the bf16 GEMM's
# per-stream workspace; "0" disables
TAILK = os.environ.get("PADDLE2_AMD_FP8_TAILK", "1") != "0"


def _ws(t):
    if not TAILK:
        return 0, 0
    from . import gemm as G

    return G._workspace(t) if G.SPLITK else (0, 0)


def mm_native(a, bT, inv_a, inv_b, out_dtype, bias=None, out=None, beta=0.0):
    """C[M, N] = (a[M, K] . bT[N, K]^T) * inv_a * inv_b (+ bias) on the native fp8 GEMM (both operands K-major
    fp8, dequant factors as device scalars).  ``out``: write into this [M, N] tensor (fp32 output: C = product +
    beta * C, e.g. a sharding unit's fp32 main-grad slot).  None when the problem is outside the kernel's domain."""
    fa, fb = _FMT.get(a.dtype), _FMT.get(bT.dtype)
    if (fa, fb, out_dtype) not in _NATIVE_CASES or a.stride(1) != 1 or bT.stride(1) != 1:
        return None
    if bias is not None and (out_dtype != torch.bfloat16 or bias.dtype != torch.bfloat16 or not bias.is_contiguous()):
        return None
    M, K = a.shape
    Nn = bT.shape[0]
    if out is not None and (out.dtype != out_dtype or tuple(out.shape) != (M, Nn) or out.stride(1) != 1):
        return None
    c = torch.empty(M, Nn, dtype=out_dtype, device=a.device) if out is None else out
    rc = N.native().gemm_f8(fa, fb, 0 if out_dtype == torch.bfloat16 else 1, a.data_ptr(), a.stride(0),
                            bT.data_ptr(), bT.stride(0), c.data_ptr(), c.stride(0), N.ptr(bias),
                            inv_a.data_ptr(), inv_b.data_ptr(), M, Nn, K, float(beta), GROUP_M, _cus(a.device),
                            *_ws(a), N.stream())
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"native fp8 GEMM failed: {rc}")
    return c


def _native_faster(nat, lib, iters=10):
    """Time both GEMM routes once on device events (after one untimed call each); False when the native kernel
    does not cover the problem."""
    from ..incubate.autotune import _bench

    if nat() is None:
        return False
    return _bench(nat, iters) <= _bench(lib, iters)


def _mm(a, b_colmajor, inv_a, inv_b, out_dtype, bias=None):
    """(a * inv_a) @ (b * inv_b) with a row-major [M, K] fp8 and b a column-major [K, N] fp8 view."""
    if a.device.type == "cuda":
        if GEMM in ("native", "auto") and N.use_native(a):
            ia = inv_a.float().reshape(1).contiguous()
            ib = inv_b.float().reshape(1).contiguous()
            nat = lambda: mm_native(a, b_colmajor.t(), ia, ib, out_dtype, bias)  # noqa: E731
            use = True
            if GEMM == "auto":
                key = (a.dtype, b_colmajor.dtype, out_dtype, a.shape[0], b_colmajor.shape[1], a.shape[1], bias is None)
                use = _ROUTE.get(key)
                if use is None and torch.cuda.is_current_stream_capturing():
                    use = True                     # no timing inside a graph capture
                elif use is None:
                    use = _ROUTE[key] = _native_faster(nat, lambda: torch._scaled_mm(
                        a, b_colmajor, scale_a=inv_a, scale_b=inv_b, bias=bias, out_dtype=out_dtype))
            if use:
                c = nat()
                if c is not None:
                    return c
        return torch._scaled_mm(a, b_colmajor, scale_a=inv_a, scale_b=inv_b, bias=bias, out_dtype=out_dtype)
    y = (a.float() * inv_a) @ (b_colmajor.float() * inv_b)
    if bias is not None:
        y = y + bias.float()
    return y.to(out_dtype)


# The weight gradient of an fp8 linear whose weight has an fp32 main-grad slot (a sharding unit's ``_p2_gt``, as the
# bf16 linear): the native fp8 GEMM writes the fp32 product straight into the slot (C = dW + beta * C) instead of a
# bf16 dW that autograd hands to the unit's hook for a bf16 -> fp32 conversion pass (on by default: GPT-3 13B fp8
# step 14,686 vs 14,542 tok/s, profiles/r5_gpt13b_fp8_step.md).  "0" keeps the bf16 dW.
WGRAD_MAIN = os.environ.get("PADDLE2_AMD_FP8_WGRAD_MAIN", "1") != "0"


def _wgrad_into_main(gt, xqT, gqT, inv_x, inv_g):
    """dW^T layout note: W is [K, N]; dW = x^T dY = (xqT [K, M]) . (gqT [N, M])^T -> [K, N] written into the
    unit's fp32 slot.  True when done (the slot is then marked written)."""
    owner, idx = gt
    view, beta = owner.grad_target(idx)
    if view.dtype != torch.float32 or not view.is_contiguous() or not N.use_native(xqT):
        return False
    ia = inv_x.float().reshape(1).contiguous()
    ib = inv_g.float().reshape(1).contiguous()
    if mm_native(xqT, gqT, ia, ib, torch.float32, out=view, beta=float(beta)) is None:
        return False
    owner.param_grad_done(idx)
    return True


class _FP8LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, bias, mx, mw, mg):
        K = x.shape[-1]
        N_ = w.shape[1]
        x2 = x.reshape(-1, K)
        xq, xqT = cast(x2, mx, transpose=True)                   # x [M, K] and x^T [K, M] (for dW)
        wq, wqT = cast(w, mw, transpose=True)                    # W [K, N] (for dX) and W^T [N, K] (fwd B)
        out_dtype = x.dtype if x.dtype in (torch.bfloat16, torch.float16) else torch.float32
        y = _mm(xq, wqT.t(), mx.inv_scale, mw.inv_scale, out_dtype,
                None if bias is None else bias.to(out_dtype))
        # dequant factors of THIS step's casts, snapshotted by the (single) update launch that rolls both scales
        snap = torch.empty(2, dtype=torch.float32, device=mx.inv_scale.device)
        defer_update([(mx, snap[0:1]), (mw, snap[1:2])])
        ctx.save_for_backward(xqT, wq, snap[0:1], snap[1:2])
        ctx.meta = (mg, x.shape, bias is not None, out_dtype, w.dtype, mx, mw)
        ctx.gt = getattr(w, "_p2_gt", None) if WGRAD_MAIN and w.is_cuda else None
        ctx.bt = bias
        return y.reshape(*x.shape[:-1], N_)

    @staticmethod
    def backward(ctx, dy):
        xqT, wq, inv_x, inv_w = ctx.saved_tensors
        mg, xshape, has_b, out_dtype, wdt, mx, mw = ctx.meta
        if id(mx) in _PENDING_IDS or id(mw) in _PENDING_IDS:
            flush_updates()   # the snaps read below are written by that queued launch
        N_ = dy.shape[-1]
        dy2 = dy.reshape(-1, N_)
        # dY [M, N], dY^T [N, M] and, with a bias, dY's column sums per 64-row block from the same pass
        if has_b:
            gq, gqT, dpart = cast(dy2, mg, transpose=True, colsum=True)
        else:
            (gq, gqT), dpart = cast(dy2, mg, transpose=True), None
        dx = _mm(gq, wq.t(), mg.inv_scale, inv_w, out_dtype)     # [M, N] @ [N, K]
        if ctx.gt is not None and ctx.needs_input_grad[1] and _wgrad_into_main(ctx.gt, xqT, gqT, inv_x, mg.inv_scale):
            dw = None
        else:
            dw = _mm(xqT, gqT.t(), inv_x, mg.inv_scale,
                     wdt if wdt in (torch.bfloat16, torch.float16) else torch.float32).to(wdt)
        db = None
        if has_b and dpart is not None and wdt in _CODE:
            # the cast's per-block column sums folded in a fixed order (no second read of dY) — into the bias's
            # fp32 main-grad slot when it has one
            from .torch_ops import BIAS_MAIN, main_slot

            slot = main_slot(ctx.bt) if BIAS_MAIN and ctx.needs_input_grad[2] else None
            if slot is not None:
                view, beta, owner, idx = slot
                N.native().colsum(_CODE[torch.float32], dpart.data_ptr(), view.data_ptr(), dpart.shape[0], N_,
                                  N.stream(), acc=int(beta != 0))
                owner.param_grad_done(idx)
            else:
                db = torch.empty(N_, dtype=wdt, device=dy2.device)
                N.native().colsum(_CODE[wdt], dpart.data_ptr(), db.data_ptr(), dpart.shape[0], N_, N.stream())
        elif has_b:
            # the native two-pass column sum (torch_ops.bias_grad): ATen's bf16 dim-0 reduce took 24.5 ms / 160
            # calls of the GPT-3 13B fp8 step (profiles/r4_gpt13b_fp8_step_kernels.txt)
            from .torch_ops import bias_grad

            db = (bias_grad(dy2.contiguous(), out_dtype=wdt) if dy2.is_cuda and dy2.dtype in (torch.bfloat16, torch.float16)
                  else dy2.sum(0, dtype=torch.float32).to(wdt))
        defer_update([(mg, None)])
        return dx.reshape(xshape), dw, db, None, None, None


@_graph_op
def fp8_linear(x, w, bias, mx, mw, mg):
    """y = x @ w + bias through e4m3 GEMMs (fwd) and e5m2-gradient GEMMs (bwd); w is [in, out]."""
    return _FP8LinearFn.apply(x, w, bias, mx, mw, mg)


def fp8_gemm(x, y, transpose_x=False, transpose_y=False, bias=None, scale=1.0, output_dtype="bfloat16"):
    """Plain fp8 x fp8 -> half GEMM (the reference's fp8_fp8_half_gemm_fused): x, y already fp8."""
    a = x.t() if transpose_x else x
    b = y.t() if transpose_y else y
    od = torch.bfloat16 if output_dtype in ("bfloat16", torch.bfloat16) else torch.float16
    one = torch.ones(1, dtype=torch.float32, device=a.device)
    sc = torch.full((1,), float(scale), dtype=torch.float32, device=a.device)
    a = a.contiguous()
    bcm = b.t().contiguous().t()  # column-major B
    return _mm(a, bcm, sc, one, od, bias)
