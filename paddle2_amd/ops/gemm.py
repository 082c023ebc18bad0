"""Python entry points of the hand-written gfx950 MFMA GEMM (csrc/kernels/gemm.hip).

The three GEMMs of a Paddle-layout Linear (W is [in, out]) map onto one kernel template with no
transpose pass (reference: paddle/phi/kernels/impl/matmul_kernel_impl.h:108 MatMulFunction and
matmul_grad; fusion/gpu/fused_linear_param_grad_add_kernel.cu:282):

  ``mm_fwd(x, w)``          y  = x @ W            A K-major, B N-major      (+bias epilogue)
  ``mm_dgrad(dy, w)``       dx = dy @ W^T         A K-major, B K-major
  ``mm_wgrad(x, dy, out)``  out = x^T @ dy (+ beta*out), fp32 main-grad epilogue; A M-major, B N-major
  ``mm_swiglu(x, w)``       gu = x @ W (packed [gate | up]), a = silu(gate) * up, in one kernel

Every function takes 2-D bf16 tensors with unit stride on the last dim.  ``supported(...)`` tells
whether the kernel accepts a problem (K % 8 == 0, 16-B aligned rows); callers fall back to
hipBLASLt (torch.matmul) otherwise.  On a GPU without the extension `_native.native()` raises.
"""
from __future__ import annotations

import os

import torch

from . import _native as N

LAYOUT_AK, LAYOUT_BK = 1, 2
EPI_BF16, EPI_F32, EPI_SWIGLU, EPI_GELU, EPI_DGELU, EPI_ROPE, EPI_DSWIGLU = 0, 1, 2, 3, 4, 5, 6
GROUP_M = int(os.environ.get("PADDLE2_AMD_GEMM_GROUP_M", "8"))
_GROUP_FORCED = "PADDLE2_AMD_GEMM_GROUP_M" in os.environ
# kernel schedule (csrc/kernels/gemm.hip): 0 = v2 (8 waves, 2 per SIMD, 128x64 wave tiles), 4 = v4 (4 waves,
# 128x128 wave tiles on AGPR accumulators, spread LDS-DMA, 8/16-B epilogue stores), 6 = v6 (v4 persistent: one
# workgroup per CU, the DMA pipeline running across tile boundaries).  Per pass, from the measured table in
# profiles/r3_gemm_v4.md: forward / dgrad (bf16 out, K = 4096..32000) v6, wgrad into the fp32 main grad v4 (its
# long token reduction leaves persistence little to win, and v6's fp32 read-modify-write epilogue spills),
# the SwiGLU-epilogue forward v4.  PADDLE2_AMD_GEMM_VARIANT forces one schedule for every pass.
# 7..10 = v7 (gemm7.hip, SCHED 0..3): the TN schedule with both operands K-major — dgrad in place, the forward and
# the SwiGLU forward on W^T (one transpose of the weight per forward); problems outside its domain (K % 128,
# >= 2 GiB operands) run v6.
# 64 + cfg = v7 with SCHED cfg (gemm7.hip); V7_SPREAD = SCHED 384: the spread three-barrier K-tile schedule
# (LDS-DMA pieces spread over 100 MFMAs, every fragment read >= 8 MFMAs before use, 3 barriers) + 16-B epilogue
# stores (v_permlane16_swap pairing) — profiles/r4_gemm_spread.md: the forward / dgrad / SwiGLU default.
V7_SPREAD = 64 + 384
# The spread schedule on the persistent v7 kernel with MN-major operands (gemm7.hip SCHED bits 15 / 16 = A / B):
# V7_MN both — the weight gradient on X and dY as stored (fp32 main-grad or bf16 epilogue); V7_NNF B only — the
# forward on W as stored (bf16 + bias).  Tail split-K like the TN forward; outside their domain v4's spread kernel.
V7_MN = 64 + (384 | 32768 | 65536)
V7_NNF = 64 + (384 | 65536)
_FORCE = os.environ.get("PADDLE2_AMD_GEMM_VARIANT")
VARIANT = int(_FORCE) if _FORCE is not None else None
PASS_VARIANT = {"fwd": V7_SPREAD, "dgrad": V7_SPREAD, "wgrad": V7_MN, "wgrad_acc": 5, "wgrad_bf16": V7_MN,
                "swiglu": V7_SPREAD, "rope": V7_SPREAD, "fwd_nn": V7_NNF, "fwd_nn_wide": V7_NNF, "wgrad_short": V7_MN}
for _k in list(PASS_VARIANT):   # per-pass override: PADDLE2_AMD_GEMM_VARIANT_FWD=6 (the forward on W as is, no W^T)
    _e = os.environ.get("PADDLE2_AMD_GEMM_VARIANT_" + _k.upper())
    if _e:
        PASS_VARIANT[_k] = int(_e)
# grouped tile order per pass (row tiles that sweep the column tiles together): 4 for the spread TN schedule
# (forward +2..7 %, dgrad +0..2 % over 8 at M = 32768; profiles/r4_gemm_spread.md), 8 for the wgrad kernels
# the N-major forward: 4, but 2 for long outputs wider than 16384 columns (M >= 16384: gate|up 22016 at 32768 tokens
# 4.24 -> 4.08 ms, 8 / 16 lose 10-22 %; at 4096 tokens 4 stays best); the MN-major wgrad: 8, but 4 for short token
# reductions into wide outputs (<= 8192 tokens, N >= 2 M: GPT-3 13B qkv / fc1 -4 %) — profiles/r6_gemm_mn_major.md,
# r6/gemm_groupm_r6w.jsonl, r6/gemm_groupm_r6x.jsonl
PASS_GROUP_M = {"fwd": 4, "dgrad": 4, "swiglu": 4, "wgrad": 8, "wgrad_acc": 8, "wgrad_bf16": 8, "rope": 4, "fwd_nn": 4,
                "fwd_nn_wide": 2, "wgrad_short": 4}
for _k in list(PASS_GROUP_M):   # per-pass override: PADDLE2_AMD_GEMM_GROUP_M_FWD=2, ..._DGRAD, ..._SWIGLU, ...
    _e = os.environ.get("PADDLE2_AMD_GEMM_GROUP_M_" + _k.upper())
    if _e:
        PASS_GROUP_M[_k] = int(_e)


def _variant(name):
    return VARIANT if VARIANT is not None else PASS_VARIANT[name]
# "native" (default on the MI355X) | "blas": route the Linear GEMMs through hipBLASLt instead
BACKEND = os.environ.get("PADDLE2_AMD_GEMM", "native")


def enabled(t: torch.Tensor) -> bool:
    return BACKEND == "native" and t.device.type == "cuda" and t.dtype == torch.bfloat16 and N.use_native(t)


def _ok2d(t, inner):
    return (t.dim() == 2 and t.stride(1) == 1 and t.stride(0) % 8 == 0 and t.data_ptr() % 16 == 0
            and t.shape[1] == inner)


def supported_fwd(x2, w):
    M, K = x2.shape
    return K % 8 == 0 and w.shape[0] == K and w.shape[1] % 8 == 0 and _ok2d(x2, K) and _ok2d(w, w.shape[1])


def supported_dgrad(dy2, w):
    return dy2.shape[1] % 8 == 0 and _ok2d(dy2, w.shape[1]) and _ok2d(w, w.shape[1])


def supported_wgrad(x2, dy2):
    # both operands are M/N-major here: any token count, 16-B column chunks
    return x2.shape[1] % 8 == 0 and dy2.shape[1] % 8 == 0 and _ok2d(x2, x2.shape[1]) and _ok2d(dy2, dy2.shape[1])


# tail split-K workspace (fp32 K-slice slabs of the last, partial wave's tiles: 8 XCDs x tail x slices x 256 KiB;
# 192 MiB covers a 24-tile tail in 4 slices), one per (device, stream) so GEMMs on concurrent streams never share
# slabs; "0" disables the split
SPLITK = os.environ.get("PADDLE2_AMD_GEMM_SPLITK", "1") != "0"
# the spread TN schedule's tail split-K (gemm7.hip SCHED bit 12: a last partial wave of <= CUs / 2 tiles runs as
# K-slices on every CU + an fp32 fix-up), bf16-output forward / dgrad; "0" disables
V7_TAILK = os.environ.get("PADDLE2_AMD_GEMM_V7_TAILK", "1") != "0"
_WS_BYTES = 192 << 20
_WS = {}


def _workspace(t):
    if not SPLITK:
        return 0, 0
    st = torch.cuda.current_stream(t.device)
    key = (t.device.index, st.cuda_stream)
    ws = _WS.get(key)
    if ws is None:
        ws = _WS[key] = torch.empty(_WS_BYTES, dtype=torch.uint8, device=t.device)
    return ws.data_ptr(), _WS_BYTES


def _launch(layout, epi, a, lda, b, ldb, c, ldc, c2, ldc2, bias, M, Nn, K, beta=0.0, H=0, name="fwd"):
    v = _variant(name)
    tail = ((epi in (EPI_BF16, EPI_F32) and v in (0, 4, 5, V7_MN, V7_NNF))
            or (V7_TAILK and epi == EPI_BF16 and v == V7_SPREAD))
    ws, ws_bytes = _workspace(a) if tail else (0, 0)
    gm = GROUP_M if _GROUP_FORCED else PASS_GROUP_M.get(name, GROUP_M)
    N.native().gemm(layout, epi, a.data_ptr(), lda, b.data_ptr(), ldb, c.data_ptr(), ldc, N.ptr(c2), ldc2,
                    N.ptr(bias), M, Nn, K, float(beta), H, gm, v, ws, ws_bytes, N.stream())


def _v7(name, K):
    """The pass runs the TN schedule (v7) on this reduction length."""
    v = _variant(name)
    return (7 <= v <= 10 or v >= 64) and K % 128 == 0


def _wt(w):
    """W [K, N] -> contiguous W^T [N, K] (HBM-speed HIP transpose) for the TN schedule."""
    from .torch_ops import transpose2d

    return transpose2d(w)


# The forward on W as stored (B operand N-major through transposed LDS reads) instead of the TN kernel on a per-call
# W^T: the persistent spread kernel with W N-major (V7_NNF) ties the TN route at M = 32768 (Llama-2-7B 28,036 vs
# 28,033 tok/s) and wins at M = 4096 (GPT-3 13B 11,563 -> 11,780) — no transpose pass, no transient W^T.  (v4's
# spread kernel on W, variant 5, lost 2.1 % at M = 32768: profiles/r6_gemm_mn_major.md.)  Rows at or below this take
# it; "0" keeps every forward on the TN route.
FWD_NN_MAX_M = int(os.environ.get("PADDLE2_AMD_GEMM_FWD_NN_MAX_M", str(1 << 30)))


def _fwd_nn(M):
    return (0 < M <= FWD_NN_MAX_M and VARIANT is None and PASS_VARIANT["fwd"] == V7_SPREAD
            and "PADDLE2_AMD_GEMM_VARIANT_FWD" not in os.environ)


def mm_fwd(x2, w, bias=None, out=None):
    """y[M, N] = x2[M, K] @ w[K, N] (+ bias[N]), bf16."""
    M, K = x2.shape
    Nn = w.shape[1]
    if out is None:
        out = torch.empty(M, Nn, dtype=x2.dtype, device=x2.device)
    if _fwd_nn(M):
        _launch(LAYOUT_AK, EPI_BF16, x2, x2.stride(0), w, w.stride(0), out, out.stride(0), None, 0, bias, M, Nn, K,
                name="fwd_nn_wide" if Nn > 16384 and M >= 16384 else "fwd_nn")
        return out
    if _v7("fwd", K):
        wt = _wt(w)
        _launch(LAYOUT_AK | LAYOUT_BK, EPI_BF16, x2, x2.stride(0), wt, wt.stride(0), out, out.stride(0), None, 0,
                bias, M, Nn, K)
        return out
    _launch(LAYOUT_AK, EPI_BF16, x2, x2.stride(0), w, w.stride(0), out, out.stride(0), None, 0, bias, M, Nn, K)
    return out


def mm_dgrad(dy2, w, out=None):
    """dx[M, K] = dy2[M, N] @ w[K, N]^T, bf16."""
    M, Nn = dy2.shape
    K = w.shape[0]
    if out is None:
        out = torch.empty(M, K, dtype=dy2.dtype, device=dy2.device)
    _launch(LAYOUT_AK | LAYOUT_BK, EPI_BF16, dy2, dy2.stride(0), w, w.stride(0), out, out.stride(0), None, 0, None,
            M, K, Nn, name="dgrad")
    return out


def mm_wgrad(x2, dy2, out, beta=0.0):
    """out[K, N] (fp32) = x2[M, K]^T @ dy2[M, N] + beta * out — dW accumulated in fp32, never rounded."""
    M, K = x2.shape
    Nn = dy2.shape[1]
    assert out.dtype == torch.float32 and out.shape == (K, Nn) and out.stride(1) == 1
    # the step's first write (beta 0) on the persistent MN-major kernel; accumulation (beta != 0) on v4's spread
    # kernel, whose read-modify-write epilogue beats the persistent kernel's atomic adds (profiles/r6_gemm_mn_major.md)
    name = "wgrad_acc" if beta != 0 else ("wgrad_short" if M <= 8192 and Nn >= 2 * K else "wgrad")
    _launch(0, EPI_F32, x2, x2.stride(0), dy2, dy2.stride(0), out, out.stride(0), None, 0, None, K, Nn, M, beta,
            name=name)
    return out


def mm_wgrad_bf16(x2, dy2, out=None):
    """out[K, N] (bf16) = x2^T @ dy2."""
    M, K = x2.shape
    Nn = dy2.shape[1]
    if out is None:
        out = torch.empty(K, Nn, dtype=x2.dtype, device=x2.device)
    _launch(0, EPI_BF16, x2, x2.stride(0), dy2, dy2.stride(0), out, out.stride(0), None, 0, None, K, Nn, M,
            name="wgrad_bf16")
    return out


def mm_gelu(x2, w, bias=None, approximate=True):
    """a[M, N] = gelu(x2 @ w + bias), h[M, N] = x2 @ w + bias (the pre-activation, kept for the backward) from ONE
    GEMM (GELU_AUX_BIAS epilogue, reference funcs/fused_gemm_epilogue.h:382).  -> (a, h)."""
    M, K = x2.shape
    Nn = w.shape[1]
    a = torch.empty(M, Nn, dtype=x2.dtype, device=x2.device)
    h = torch.empty(M, Nn, dtype=x2.dtype, device=x2.device)
    if _v7("fwd", K):
        wt = _wt(w)
        _launch(LAYOUT_AK | LAYOUT_BK, EPI_GELU, x2, x2.stride(0), wt, wt.stride(0), a, a.stride(0), h, h.stride(0),
                bias, M, Nn, K, 0.0, int(bool(approximate)))
        return a, h
    _launch(LAYOUT_AK, EPI_GELU, x2, x2.stride(0), w, w.stride(0), a, a.stride(0), h, h.stride(0), bias, M, Nn, K,
            0.0, int(bool(approximate)))
    return a, h


def mm_dgrad_dgelu(dy2, w, h, approximate=True):
    """dh[M, K] = (dy2[M, N] @ w[K, N]^T) * gelu'(h[M, K]): the next linear's input gradient with the GELU backward
    in its epilogue (reference funcs/fused_gemm_epilogue.h:580) — the product is never rounded before the scale."""
    M, Nn = dy2.shape
    K = w.shape[0]
    assert h.shape == (M, K) and h.stride(1) == 1 and h.dtype == dy2.dtype
    out = torch.empty(M, K, dtype=dy2.dtype, device=dy2.device)
    _launch(LAYOUT_AK | LAYOUT_BK, EPI_DGELU, dy2, dy2.stride(0), w, w.stride(0), out, out.stride(0), h, h.stride(0),
            None, M, K, Nn, 0.0, int(bool(approximate)), name="dgrad")
    return out


def mm_dgrad_dswiglu(dy2, w, gu, out=None):
    """d_gu[M, 2H] from the down projection's output gradient: d_a = dy2[M, N] @ w[H, N]^T stays in fp32 in the
    epilogue, which writes d_gate = d_a * up * silu'(gate) and d_up = d_a * silu(gate) (gu = [gate | up] the SwiGLU
    forward saved).  ``out`` may be ``gu`` itself (in place).  None unless the spread TN schedule is selected."""
    M, Nn = dy2.shape
    H = w.shape[0]
    if _variant("dgrad") != V7_SPREAD or Nn % 128 or gu.shape != (M, 2 * H) or gu.stride(1) != 1 or H % 8:
        return None
    if out is None:
        out = torch.empty_like(gu)
    _launch(LAYOUT_AK | LAYOUT_BK, EPI_DSWIGLU, dy2, dy2.stride(0), w, w.stride(0), out, out.stride(0), gu,
            gu.stride(0), None, M, H, Nn, 0.0, H, name="dgrad")
    return out


def mm_fwd_rope(x2, w, cos, sin, rope_cols, seq):
    """y[M, N] = x2 @ w with rotate-half RoPE applied in the epilogue to the 128-wide heads of columns < rope_cols
    (row r at position r % seq; fp32 cos / sin [seq, 128]) — the QKV projection with its q / k rotation fused.
    None when the spread TN schedule is not the one selected (the caller then runs GEMM + RoPE)."""
    M, K = x2.shape
    Nn = w.shape[1]
    # whole 256 x 256 tiles and seq >= 128 (the kernel's fused epilogue carries no edge-tile form)
    if _variant("rope") != V7_SPREAD or K % 128 or rope_cols % 128 or Nn % 256 or M % 256 or seq < 128:
        return None
    assert cos.dtype == sin.dtype == torch.float32 and cos.shape == sin.shape == (seq, 128)
    out = torch.empty(M, Nn, dtype=x2.dtype, device=x2.device)
    wt = _wt(w)
    N.native().gemm_set_rope(cos.data_ptr(), sin.data_ptr(), int(rope_cols), int(seq))
    _launch(LAYOUT_AK | LAYOUT_BK, EPI_ROPE, x2, x2.stride(0), wt, wt.stride(0), out, out.stride(0), None, 0, None,
            M, Nn, K, name="rope")
    return out


def mm_swiglu(x2, w):
    """gu[M, 2H] = x2 @ w (w = [gate | up] packed [K, 2H]); a[M, H] = silu(gate) * up.  -> (a, gu)."""
    M, K = x2.shape
    H = w.shape[1] // 2
    gu = torch.empty(M, 2 * H, dtype=x2.dtype, device=x2.device)
    a = torch.empty(M, H, dtype=x2.dtype, device=x2.device)
    if _v7("swiglu", K):
        wt = _wt(w)
        _launch(LAYOUT_AK | LAYOUT_BK, EPI_SWIGLU, x2, x2.stride(0), wt, wt.stride(0), a, a.stride(0), gu,
                gu.stride(0), None, M, 2 * H, K, 0.0, H, name="swiglu")
        return a, gu
    _launch(LAYOUT_AK, EPI_SWIGLU, x2, x2.stride(0), w, w.stride(0), a, a.stride(0), gu, gu.stride(0), None, M,
            2 * H, K, 0.0, H, name="swiglu")
    return a, gu


# ------------------------------------------------------------------------------------ grouped (MoE experts)
# One launch over every expert: rows are sorted by expert and goff [E + 1] (int32, on the device) delimits
# each expert's slice — no host read of the per-expert counts (reference fusion/cutlass/fused_moe_kernel.cu
# runs a CUTLASS grouped GEMM from host-known problem sizes; here the kernel resolves them itself).
def _goff_ok(goff, E):
    return goff.dtype == torch.int32 and goff.is_contiguous() and goff.numel() == E + 1


def grouped_fwd(xs, w, goff, bias=None, out=None):
    """out[goff[e]:goff[e+1]] = xs[goff[e]:goff[e+1]] @ w[e] (+ bias[e]); xs [T, K], w [E, K, N] bf16."""
    T, K = xs.shape
    E, _, Nn = w.shape
    assert _goff_ok(goff, E) and w.is_contiguous()
    if out is None:
        out = torch.empty(T, Nn, dtype=xs.dtype, device=xs.device)
    if T:
        N.native().gemm_grouped(LAYOUT_AK, EPI_BF16, xs.data_ptr(), xs.stride(0), w.data_ptr(), Nn, K * Nn,
                                out.data_ptr(), out.stride(0), 0, 0, 0, N.ptr(bias), 0 if bias is None else Nn,
                                goff.data_ptr(), E, 0, 0, Nn, K, T, 0.0, 0, GROUP_M, N.stream())
    return out


def grouped_swiglu(xs, w, goff):
    """Grouped x @ w[e] with w[e] = [gate | up] ([E, K, 2F]) and the SwiGLU epilogue -> (a [T, F], gu [T, 2F])."""
    T, K = xs.shape
    E, _, F2 = w.shape
    F = F2 // 2
    assert _goff_ok(goff, E) and w.is_contiguous()
    gu = torch.empty(T, F2, dtype=xs.dtype, device=xs.device)
    a = torch.empty(T, F, dtype=xs.dtype, device=xs.device)
    if T:
        N.native().gemm_grouped(LAYOUT_AK, EPI_SWIGLU, xs.data_ptr(), xs.stride(0), w.data_ptr(), F2, K * F2,
                                a.data_ptr(), a.stride(0), 0, gu.data_ptr(), gu.stride(0), 0, 0, goff.data_ptr(), E, 0,
                                0, F2, K, T, 0.0, F, GROUP_M, N.stream())
    return a, gu


def grouped_dgrad(dy, w, goff):
    """dx[goff[e]:goff[e+1]] = dy[...] @ w[e]^T; dy [T, N], w [E, K, N] -> dx [T, K]."""
    T, Nn = dy.shape
    E, K, _ = w.shape
    assert _goff_ok(goff, E) and w.is_contiguous()
    dx = torch.empty(T, K, dtype=dy.dtype, device=dy.device)
    if T:
        N.native().gemm_grouped(LAYOUT_AK | LAYOUT_BK, EPI_BF16, dy.data_ptr(), dy.stride(0), w.data_ptr(), Nn,
                                K * Nn, dx.data_ptr(), dx.stride(0), 0, 0, 0, 0, 0, goff.data_ptr(), E, 0, 0, K, Nn, T,
                                0.0, 0, GROUP_M, N.stream())
    return dx


def grouped_wgrad(xs, dy, goff, out, beta=0.0):
    """out[e] (+)= xs[goff[e]:goff[e+1]]^T @ dy[...]; out [E, K, N] fp32 (main grad) or bf16."""
    T, K = xs.shape
    Nn = dy.shape[1]
    E = out.shape[0]
    assert _goff_ok(goff, E) and out.is_contiguous() and out.shape[1:] == (K, Nn)
    epi = EPI_F32 if out.dtype == torch.float32 else EPI_BF16
    N.native().gemm_grouped(0, epi, xs.data_ptr(), xs.stride(0), dy.data_ptr(), dy.stride(0), 0, out.data_ptr(), Nn,
                            K * Nn, 0, 0, 0, 0, goff.data_ptr(), E, 1, K, Nn, 0, 0, float(beta), 0, GROUP_M,
                            N.stream())
    return out
