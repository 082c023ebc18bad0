"""Attention-bias descriptors for memory_efficient_attention (reference python/paddle/incubate/nn/attn_bias.py):
they describe a mask structurally so the kernel can pick a fused path (causal / block-diagonal varlen) instead
of materialising an [Sq, Sk] bias."""
from __future__ import annotations

import torch


class AttentionBias:
    def materialize(self, shape, dtype=torch.float32, device="cpu"):
        raise NotImplementedError


class LowerTriangularMask(AttentionBias):
    """Causal: key j is visible to query i iff j <= i."""

    def materialize(self, shape, dtype=torch.float32, device="cpu"):
        sq, sk = shape[-2], shape[-1]
        m = torch.ones(sq, sk, dtype=torch.bool, device=device).tril(sk - sq)
        return torch.zeros(shape, dtype=dtype, device=device).masked_fill(~m, float("-inf"))

    def add_bias(self, bias):
        return LowerTriangularMaskWithTensorBias(bias)


class LowerTriangularMaskWithTensorBias(LowerTriangularMask):
    def __init__(self, bias):
        self._bias = bias

    def materialize(self, shape, dtype=torch.float32, device="cpu"):
        b = self._bias._t if hasattr(self._bias, "_t") else self._bias
        return super().materialize(shape, dtype, device) + b.to(dtype)


class _SeqLenInfo:
    def __init__(self, seqlens):
        self.seqlens = [int(s) for s in seqlens]
        self.seqstart = [0]
        for s in self.seqlens:
            self.seqstart.append(self.seqstart[-1] + s)
        self.max_seqlen = max(self.seqlens) if self.seqlens else 0

    @classmethod
    def from_seqlens(cls, seqlens):
        return cls(seqlens)


class BlockDiagonalMask(AttentionBias):
    """Several sequences packed along the token axis ([1, total, H, D]); each attends only within itself."""

    _causal = False

    def __init__(self, q_seqinfo, k_seqinfo):
        self.q_seqinfo, self.k_seqinfo = q_seqinfo, k_seqinfo

    @classmethod
    def from_seqlens(cls, q_seqlen, kv_seqlen=None):
        q = _SeqLenInfo(q_seqlen)
        k = q if kv_seqlen is None else _SeqLenInfo(kv_seqlen)
        return cls(q, k)

    def make_causal(self):
        return BlockDiagonalCausalMask(self.q_seqinfo, self.k_seqinfo)

    def materialize(self, shape, dtype=torch.float32, device="cpu"):
        out = torch.full(shape[-2:], float("-inf"), dtype=dtype, device=device)
        for i in range(len(self.q_seqinfo.seqlens)):
            q0, q1 = self.q_seqinfo.seqstart[i], self.q_seqinfo.seqstart[i + 1]
            k0, k1 = self.k_seqinfo.seqstart[i], self.k_seqinfo.seqstart[i + 1]
            blk = torch.zeros(q1 - q0, k1 - k0, dtype=dtype, device=device)
            if self._causal:
                blk = LowerTriangularMask().materialize(blk.shape, dtype, device)
            out[q0:q1, k0:k1] = blk
        return out.expand(shape)


class BlockDiagonalCausalMask(BlockDiagonalMask):
    _causal = True
