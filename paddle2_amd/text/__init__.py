"""paddle.text (reference: python/paddle/text/viterbi_decode.py:31 viterbi_decode, :103 ViterbiDecoder;
text/datasets/*.py).

``viterbi_decode`` is a batched max-product DP on the device of the emissions: per time step one
broadcast add + max/argmax over the previous tag, then a gather-based backtrace.  With
``include_bos_eos_tag`` the last tag is BOS (its transition ROW scores the first tag) and the
second-to-last is EOS (``transitions[-2, tag]`` scores the final tag), matching the reference op.
"""
from __future__ import annotations

import torch

from ..framework.tensor import Tensor
from ..nn.layer.layers import Layer
from .datasets import Conll05st, Imdb, Imikolov, Movielens, UCIHousing, WMT14, WMT16  # noqa: F401

_w = Tensor._wrap


def _t(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x)


def viterbi_decode(potentials, transition_params, lengths, include_bos_eos_tag=True, name=None):
    """-> (scores [B], paths [B, max(lengths)] int64; positions past a sequence's length are 0)."""
    pot, trans = _t(potentials), _t(transition_params).to(_t(potentials).dtype)
    L = _t(lengths).to(pot.device).long()
    B, _, N = pot.shape
    T = int(L.max().item()) if L.numel() else 0
    if T == 0:
        return _w(torch.zeros(B, dtype=pot.dtype)), _w(torch.zeros(B, 0, dtype=torch.int64))
    alpha = pot[:, 0] + (trans[-1][None, :] if include_bos_eos_tag else 0)
    hist = []
    for t in range(1, T):
        best, arg = (alpha[:, :, None] + trans[None]).max(dim=1)
        active = (t < L)[:, None]
        alpha = torch.where(active, best + pot[:, t], alpha)
        hist.append(arg)
    if include_bos_eos_tag:
        alpha = alpha + trans[-2][None, :]
    scores, last = alpha.max(dim=1)
    path = torch.zeros(B, T, dtype=torch.int64, device=pot.device)
    cur = last.clone()
    for t in range(T - 1, -1, -1):
        inside = t <= L - 1
        cur = torch.where(t == L - 1, last, cur)
        path[:, t] = torch.where(inside, cur, torch.zeros_like(cur))
        if t > 0:
            prev = hist[t - 1].gather(1, cur[:, None])[:, 0]
            cur = torch.where(inside, prev, cur)
    return _w(scores), _w(path)


class ViterbiDecoder(Layer):
    def __init__(self, transitions, include_bos_eos_tag=True, name=None):
        super().__init__()
        self.transitions = transitions
        self.include_bos_eos_tag = include_bos_eos_tag

    def forward(self, potentials, lengths):
        return viterbi_decode(potentials, self.transitions, lengths, self.include_bos_eos_tag)


__all__ = ["viterbi_decode", "ViterbiDecoder", "Conll05st", "Imdb", "Imikolov", "Movielens", "UCIHousing", "WMT14",
           "WMT16"]
