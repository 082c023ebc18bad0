"""Weight-only int8/int4 matmul dispatch (kernel: csrc/kernels/weight_only.hip).

``weight_only_matmul(x [M, K], w [N, K] int8 | [N/2, K] int4, scale [N] | [K/G, N])`` -> [M, N].
On the MI355X with bf16 activations and M <= 64 it runs the fused dequant + MFMA kernel (weights
read from HBM once, in their 1- or 0.5-byte form); larger M (prefill) dequantizes to bf16 once and
uses the hipBLASLt GEMM.  On CPU it is the fp32 reference.
"""
from __future__ import annotations

import torch

from . import _native as N


def dequantize(w, scale, weight_dtype="int8", group_size=-1, dtype=torch.float32):
    q = w
    if weight_dtype == "int4":
        u = w.view(torch.uint8).to(torch.int16)
        lo, hi = u & 0xF, (u >> 4) & 0xF
        lo = torch.where(lo > 7, lo - 16, lo)
        hi = torch.where(hi > 7, hi - 16, hi)
        q = torch.stack([lo, hi], 1).reshape(-1, w.shape[1])
    q = q.float()
    s = scale.float()
    if group_size in (-1, None) or s.dim() == 1:
        out = q * s[:, None]
    else:
        out = q * s.t().repeat_interleave(group_size, 1)[:, : q.shape[1]]
    return out.to(dtype)  # [N, K]


def _native_ok(x, w, weight_dtype, group_size):
    M, K = x.shape
    Nn = w.shape[0] * (2 if weight_dtype == "int4" else 1)
    return (x.device.type == "cuda" and N.use_native(x) and x.dtype == torch.bfloat16 and M <= 64 and K % 64 == 0
            and Nn % 64 == 0 and group_size in (-1, 64, 128) and w.is_contiguous())


def weight_only_matmul(x, w, scale, weight_dtype="int8", group_size=-1, bias=None):
    x = x.contiguous()
    M, K = x.shape
    if _native_ok(x, w, weight_dtype, group_size) and N.use_native(x):
        C = N.native()
        Nn = w.shape[0] * (2 if weight_dtype == "int4" else 1)
        g = -1 if group_size in (-1, None) else int(group_size)
        S = C.wo_splits(M, Nn, K, g)
        ws = torch.empty(C.wo_workspace(M, Nn, S), dtype=torch.float32, device=x.device)
        out = torch.empty(M, Nn, dtype=x.dtype, device=x.device)
        sc = scale.float().contiguous()
        if bias is not None:
            bias = bias.to(torch.bfloat16).contiguous()
        C.wo_gemm(int(weight_dtype == "int4"), x.data_ptr(), w.data_ptr(), sc.data_ptr() if g < 0 else 0,
                  sc.data_ptr() if g > 0 else 0, max(g, 0), N.ptr(bias), out.data_ptr(), ws.data_ptr(), M, Nn, K,
                  S, N.stream())
        return out
    wd = dequantize(w, scale, weight_dtype, group_size, x.dtype if x.device.type == "cuda" else torch.float32)
    y = x.to(wd.dtype) @ wd.t()
    if bias is not None:
        y = y + bias.to(y.dtype)
    return y.to(x.dtype)


# ---------------------------------------------------------------------------------------------- bf16 decode GEMM
# "native": the split-K MFMA stream kernel (csrc/kernels/weight_only.hip dec_gemm_kernel) for decode-sized token
# counts on the cached [N, K] weights; "blas": hipBLASLt through torch.matmul
import os as _os  # noqa: E402

DECODE_GEMM = _os.environ.get("PADDLE2_AMD_DECODE_GEMM", "auto")   # auto | native | blas
DEC64_WAVES = int(_os.environ.get("PADDLE2_AMD_DEC64_WAVES", "8"))  # waves per workgroup of the M > 16 kernel
DEC64_RT = int(_os.environ.get("PADDLE2_AMD_DEC64_RT", "0"))        # its channel tiles per workgroup (0 = auto)
# M > 16 kernel: "r" = dec64_kernel (X prefetched in registers), "s" = dec64s_kernel (X through an LDS ring, waves
# split the channels; cfg "dw,rt,S" with 0 = auto), "auto" = r for M <= 32, s above (measured per M:
# profiles/r5_decode_serving.md)
DEC64_IMPL = _os.environ.get("PADDLE2_AMD_DEC64_IMPL", "auto")
DEC64S_CFG = tuple(int(v) for v in _os.environ.get("PADDLE2_AMD_DEC64S_CFG", "0,0,0").split(","))


def decode_ok(x, wt):
    """The native stream kernel is taken where it measured faster than hipBLASLt's skinny GEMM
    (profiles/r4_decode_gemm.md): M <= 16 with N <= 8192 (the o / down projections: 2.6-4.0 vs 1.9-3.4 TB/s).
    16 < M <= 64 has the whole-K stream kernels (dec64_kernel up to M = 32, the LDS-X dec64s_kernel above), which
    beat the library only on the square 4096 x 4096 projection (profiles/r5_decode_serving.md: 2.2 vs 1.8 TB/s at
    M <= 32, 1.86-1.89 vs 1.83-1.84 above; 2.5-3.7 vs 4.0-4.3 TB/s on the wide ones), so auto routes only that
    shape to them.
    PADDLE2_AMD_DECODE_GEMM=native forces the native kernels for every M <= 64, =blas the library."""
    M, K = x.shape
    Nn = wt.shape[0]
    ok = (x.device.type == "cuda" and x.dtype == torch.bfloat16 and wt.dtype == torch.bfloat16 and 1 <= M <= 64
          and K % 64 == 0 and wt.shape[1] == K and wt.is_contiguous() and N.use_native(x))
    if not ok:
        return False
    if DECODE_GEMM == "blas":
        return False
    if M > 16:   # the whole-K MFMA stream kernel (dec64_kernel): the b17-64 serving step
        return Nn % 16 == 0 and (DECODE_GEMM == "native" or (Nn <= 4096 and K <= 4096))
    # the split-K kernel (64-row blocks): every width up to 8 rows — in the HIP-graph decode step it beats hipBLASLt
    # on the wide qkv / gate|up projections too (b1-b8 3.8-6.6 % faster per step, profiles/r5_decode_serving.md) —
    # and N <= 8192 for 9-16 rows (b16: the library wins the wide ones by ~1.5 %)
    return Nn % 64 == 0 and (DECODE_GEMM == "native" or M <= 8 or Nn <= 8192)


def decode_glu_ok(gu, wt):
    """The SwiGLU-staged split-K decode GEMM covers the M <= 16 rows whose plain decode GEMM runs native."""
    M, K2 = gu.shape
    K, Nn = K2 // 2, wt.shape[0]
    return (gu.device.type == "cuda" and gu.dtype == torch.bfloat16 and wt.dtype == torch.bfloat16 and K2 % 2 == 0
            and 1 <= M <= 16 and K % 64 == 0 and wt.shape[1] == K and wt.is_contiguous() and N.use_native(gu)
            and DECODE_GEMM != "blas" and Nn % 64 == 0 and (DECODE_GEMM == "native" or Nn <= 8192))


def decode_glu_matmul(gu, wt):
    """y[M, N] = (silu(gate) * up) @ wt[N, K]^T for the gate|up output gu = [gate | up] [M, 2K], M <= 16: the SwiGLU
    is applied while the split-K kernel stages X in LDS (csrc/kernels/weight_only.hip dec_gemm_kernel<GLU>)."""
    M, K2 = gu.shape
    K = K2 // 2
    Nn = wt.shape[0]
    gu = gu.contiguous()
    C = N.native()
    S = C.dec_splits(M, Nn, K)
    ws = torch.empty(S * M * Nn, dtype=torch.float32, device=gu.device)
    out = torch.empty(M, Nn, dtype=gu.dtype, device=gu.device)
    C.dec_gemm(gu.data_ptr(), wt.data_ptr(), 0, out.data_ptr(), ws.data_ptr(), M, Nn, K, S, N.stream(), 1,
               _dec_counters(gu.device, Nn))
    return out


# The split-K decode GEMM reduces its partials in the last-arriving workgroup of each column block (no reduce launch);
# its arrival counters: one zeroed int32 buffer per (device, stream), re-armed by the kernel itself.
DEC_FUSED_REDUCE = _os.environ.get("PADDLE2_AMD_DEC_FUSED_REDUCE", "0") != "0"
_DEC_CNT = {}
_DEC_CNT_LEN = 4096   # column blocks: N / 64 <= 4096 (N <= 262,144)


def _dec_counters(dev, Nn):
    if not DEC_FUSED_REDUCE or Nn // 64 > _DEC_CNT_LEN:
        return 0
    key = (dev, N.stream())
    buf = _DEC_CNT.get(key)
    if buf is None:
        buf = _DEC_CNT[key] = torch.zeros(_DEC_CNT_LEN, dtype=torch.int32, device=dev)
    return buf.data_ptr()


# Opt-in ("1"): decode rows (M <= 16) on the split-K kernel leave their S fp32 partials to the consumer — the o / down
# projections' outputs feed a residual-add + RMSNorm that sums them itself (torch_ops.rms_norm_partials,
# csrc/kernels/norm.hip PART), so the per-projection reduce launch disappears.  Bit-identical, but slower in the
# graphed decode step (b1 4.46 vs 4.39 ms, b16 6.28 vs 6.22; profiles/r6_decode_partials.md): the norm sums the 16
# partials of a row on ONE workgroup, where the reduce launch spreads them over several.
PARTIALS = _os.environ.get("PADDLE2_AMD_DEC_PARTIALS", "0") == "1"


class DecodePartials:
    """The unreduced output of a split-K decode GEMM: ``ws`` [S, M, N] fp32, summed in split order by its consumer
    (bit-identical to the reduce launch's bf16 output); ``materialize()`` runs that reduce for any other consumer."""

    __slots__ = ("ws", "S", "M", "N", "shape", "dtype")

    def __init__(self, ws, S, M, Nn, shape, dtype):
        self.ws, self.S, self.M, self.N, self.shape, self.dtype = ws, S, M, Nn, shape, dtype

    def materialize(self):
        out = torch.empty(self.M, self.N, dtype=self.dtype, device=self.ws.device)
        N.native().dec_reduce(self.ws.data_ptr(), self.S, self.M, self.N, 0, out.data_ptr(), N.stream())
        return out.view(self.shape)


def _partials_ok(M):
    return PARTIALS and not DEC_FUSED_REDUCE and 1 <= M <= 16


def decode_matmul_partials(x, wt, shape):
    """x[M, K] @ wt[N, K]^T as DecodePartials (``shape``: the view of the materialised output), or None when these
    rows do not run the split-K kernel."""
    x = x.contiguous()
    M, K = x.shape
    if not (_partials_ok(M) and decode_ok(x, wt)):
        return None
    Nn = wt.shape[0]
    C = N.native()
    S = C.dec_splits(M, Nn, K)
    ws = torch.empty(S * M * Nn, dtype=torch.float32, device=x.device)
    C.dec_gemm(x.data_ptr(), wt.data_ptr(), 0, 0, ws.data_ptr(), M, Nn, K, S, N.stream(), 0, 0, 1)
    return DecodePartials(ws, S, M, Nn, shape, x.dtype)


def decode_glu_partials(gu, wt, shape):
    """(silu(gate) * up) @ wt^T (decode_glu_matmul) as DecodePartials, or None outside its route."""
    M, K2 = gu.shape
    if not (_partials_ok(M) and decode_glu_ok(gu, wt)):
        return None
    K = K2 // 2
    Nn = wt.shape[0]
    gu = gu.contiguous()
    C = N.native()
    S = C.dec_splits(M, Nn, K)
    ws = torch.empty(S * M * Nn, dtype=torch.float32, device=gu.device)
    C.dec_gemm(gu.data_ptr(), wt.data_ptr(), 0, 0, ws.data_ptr(), M, Nn, K, S, N.stream(), 1, 0, 1)
    return DecodePartials(ws, S, M, Nn, shape, gu.dtype)


def decode_matmul(x, wt, bias=None):
    """y[M, N] = x[M, K] @ wt[N, K]^T (+ bias) for M <= 64 on the native stream kernel (weights read once, split-K
    over the 256 CUs, fp32 partials summed in a second pass); torch.matmul otherwise."""
    x = x.contiguous()
    if not decode_ok(x, wt):
        y = torch.matmul(x, wt.t())
        return y if bias is None else y + bias
    M, K = x.shape
    Nn = wt.shape[0]
    C = N.native()
    if M > 16:
        out = torch.empty(M, Nn, dtype=x.dtype, device=x.device)
        if bias is not None:
            bias = bias.to(torch.bfloat16).contiguous()
        impl = DEC64_IMPL if DEC64_IMPL != "auto" else ("r" if M <= 32 else "s")
        if impl == "s" and Nn % 64 == 0:
            dw, rt, S = DEC64S_CFG
            n_ws = C.dec64s_workspace(M, Nn, K, dw, rt, S)
            ws = torch.empty(max(n_ws, 1), dtype=torch.float32, device=x.device)
            C.dec64s_gemm(x.data_ptr(), wt.data_ptr(), N.ptr(bias), out.data_ptr(), ws.data_ptr(), M, Nn, K, dw, rt,
                          S, N.stream())
            return out
        C.dec64_gemm(x.data_ptr(), wt.data_ptr(), N.ptr(bias), out.data_ptr(), M, Nn, K, DEC64_WAVES, DEC64_RT,
                     N.stream())
        return out
    S = C.dec_splits(M, Nn, K)
    ws = torch.empty(S * M * Nn, dtype=torch.float32, device=x.device)
    out = torch.empty(M, Nn, dtype=x.dtype, device=x.device)
    if bias is not None:
        bias = bias.to(torch.bfloat16).contiguous()
    C.dec_gemm(x.data_ptr(), wt.data_ptr(), N.ptr(bias), out.data_ptr(), ws.data_ptr(), M, Nn, K, S, N.stream(), 0,
               _dec_counters(x.device, Nn))
    return out
