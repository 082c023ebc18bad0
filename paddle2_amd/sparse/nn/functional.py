"""paddle.sparse.nn.functional: sparse convolution / pooling on COO point-cloud tensors, activations,
row softmax and sparse-mask attention (reference: python/paddle/sparse/nn/functional/{conv,pooling,activation,
transformer}.py; phi/kernels/sparse/gpu/conv_kernel.cu gather-GEMM-scatter, pool_kernel.cu,
fused_attention_kernel.cu).

Sparse convolution (x: COO ``[N, *spatial, C_in]`` with indices ``[1 + nd, nnz]``, weight
``[*kernel, C_in, C_out]``):
  1. rulebook — for every (input nonzero, kernel offset) pair the output site it feeds, found with sorted
     linear keys + ``searchsorted`` (no hash table): regular conv creates every reachable output site, the
     submanifold variant keeps only sites that are active in the input;
  2. the pairs are sorted by kernel offset so each offset's rows form one contiguous slice; the gathered
     input rows go through ONE grouped GEMM over all offsets (ops/moe.grouped_linear — on the MI355X the
     native MFMA GEMM in grouped mode, device-side offsets, no per-offset launches);
  3. the products are scatter-added (``index_add``) into the output rows.
Autograd flows through gather / grouped GEMM / index_add (the grouped GEMM has its own dgrad / wgrad).
"""
from __future__ import annotations

import itertools
import math

import torch

from ...framework.tensor import Tensor
from ..creation import _is_csr, _u, real_entries, to_coo_torch
from ..ops import _rebuild, _vals, relu as _relu

_w = Tensor._wrap


def _tuple(v, n):
    return tuple(v) if isinstance(v, (list, tuple)) else (v,) * n


def _keys(coords, dims):
    """Row-major linear key of integer coordinates [P, 1 + nd] over dims (batch first)."""
    k = torch.zeros(coords.shape[0], dtype=torch.int64, device=coords.device)
    for d, s in enumerate(dims):
        k = k * s + coords[:, d]
    return k


def _rulebook(idx, in_sp, ks, stride, pad, dil, subm):
    """-> (in_row [P], out_row [P], kernel offset [P] (sorted), out coords [n_out, 1 + nd], out spatial)."""
    nd = len(in_sp)
    dev = idx.device
    if subm:
        out_sp = list(in_sp)
    else:
        out_sp = [(in_sp[d] + 2 * pad[d] - dil[d] * (ks[d] - 1) - 1) // stride[d] + 1 for d in range(nd)]
    offs = torch.tensor(list(itertools.product(*[range(k) for k in ks])), dtype=torch.int64, device=dev)  # [K, nd]
    coords = idx.t()                       # [nnz, 1 + nd]
    sp = coords[:, 1:]
    num = sp[:, None, :] + torch.tensor(pad, device=dev) - offs[None] * torch.tensor(dil, device=dev)  # [nnz,K,nd]
    st = torch.tensor(stride, device=dev)
    o = torch.div(num, st, rounding_mode="floor")
    valid = (num % st == 0).all(-1) & (o >= 0).all(-1) & (o < torch.tensor(out_sp, device=dev)).all(-1)
    in_row, kk = valid.nonzero(as_tuple=True)
    oc = torch.cat([coords[in_row, :1], o[in_row, kk]], 1)
    dims = [int(idx[0].max()) + 1 if idx.shape[1] else 1] + out_sp
    okey = _keys(oc, dims)
    if subm:
        ikey = _keys(coords, dims)  # coalesced COO: keys already sorted
        pos = torch.searchsorted(ikey, okey)
        hit = (pos < ikey.numel()) & (ikey[pos.clamp_max(max(ikey.numel() - 1, 0))] == okey)
        in_row, kk, out_row = in_row[hit], kk[hit], pos[hit]
        out_coords = coords
    else:
        ukeys, out_row = torch.unique(okey, return_inverse=True)
        out_coords = torch.zeros(ukeys.numel(), 1 + nd, dtype=torch.int64, device=dev)
        rem = ukeys
        for d in range(nd, -1, -1):
            out_coords[:, d] = rem % dims[d]
            rem = rem // dims[d]
    order = torch.argsort(kk, stable=True)
    return in_row[order], out_row[order], kk[order], out_coords, out_sp


def _conv(x, weight, bias, stride, padding, dilation, groups, subm, nd, data_format):
    if groups != 1:
        raise NotImplementedError("sparse conv: groups > 1")
    t = to_coo_torch(_u(x))
    w = _u(weight)
    ks = tuple(w.shape[:nd])
    stride, dil = _tuple(stride, nd), _tuple(dilation, nd)
    pad = _tuple(padding, nd)
    if subm:
        stride = (1,) * nd
        pad = tuple(dil[d] * (ks[d] // 2) for d in range(nd))
    idx, vals = t.indices(), t.values()
    in_row, out_row, kk, out_coords, out_sp = _rulebook(idx, list(t.shape[1:1 + nd]), ks, stride, pad, dil, subm)
    K = math.prod(ks)
    cin, cout = w.shape[-2], w.shape[-1]
    wk = w.reshape(K, cin, cout)
    goff = torch.zeros(K + 1, dtype=torch.int32, device=vals.device)
    goff[1:] = torch.bincount(kk, minlength=K).cumsum(0).to(torch.int32)
    from ...ops import moe as MOE

    xs = vals.index_select(0, in_row)
    ys = MOE.grouped_linear(xs, wk.to(xs.dtype), goff)
    n_out = out_coords.shape[0]
    out = torch.zeros(n_out, cout, dtype=torch.float32, device=vals.device).index_add(0, out_row, ys.float())
    out = out.to(vals.dtype)
    if bias is not None:
        out = out + _u(bias).to(out.dtype)
    shape = [t.shape[0]] + list(out_sp) + [cout]
    return _w(torch.sparse_coo_tensor(out_coords.t(), out, size=shape, is_coalesced=True))


def conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, False, 3, data_format)


def subm_conv3d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NDHWC", key=None,
                name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, True, 3, data_format)


def conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NHWC", name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, False, 2, data_format)


def subm_conv2d(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, data_format="NHWC", key=None,
                name=None):
    return _conv(x, weight, bias, stride, padding, dilation, groups, True, 2, data_format)


# implicit-GEMM variants of the reference: same math, same rulebook + grouped GEMM here
subm_conv3d_igemm = subm_conv3d
subm_conv2d_igemm = subm_conv2d


def max_pool3d(x, kernel_size, stride=None, padding=0, ceil_mode=False, data_format="NDHWC", name=None):
    """Max over each window's ACTIVE inputs (reference pool_kernel: absent sites do not count as zeros)."""
    t = to_coo_torch(_u(x))
    ks = _tuple(kernel_size, 3)
    st = _tuple(stride if stride is not None else kernel_size, 3)
    pad = _tuple(padding, 3)
    idx, vals = t.indices(), t.values()
    in_row, out_row, _, out_coords, out_sp = _rulebook(idx, list(t.shape[1:4]), ks, st, pad, (1, 1, 1), False)
    C = vals.shape[1]
    out = torch.full((out_coords.shape[0], C), float("-inf"), dtype=vals.dtype, device=vals.device)
    out = out.scatter_reduce(0, out_row[:, None].expand(-1, C), vals.index_select(0, in_row), "amax")
    shape = [t.shape[0]] + list(out_sp) + [C]
    return _w(torch.sparse_coo_tensor(out_coords.t(), out, size=shape, is_coalesced=True))


# ------------------------------------------------------------------------------------------ activations
def relu(x, name=None):
    return _relu(x)


def relu6(x, name=None):
    t = _u(x)
    return _w(_rebuild(t, torch.clamp(_vals(t), 0, 6)))


def leaky_relu(x, negative_slope=0.01, name=None):
    t = _u(x)
    return _w(_rebuild(t, torch.nn.functional.leaky_relu(_vals(t), negative_slope)))


def _row_ids(t):
    """Segment id per stored value: rows of a CSR matrix (batched: b*M + row); COO: every index but the last."""
    if _is_csr(t):
        crow = t.crow_indices()
        if t.dim() == 2:
            return torch.repeat_interleave(torch.arange(t.shape[0], device=crow.device), crow[1:] - crow[:-1])
        B, M = t.shape[0], t.shape[1]
        counts = (crow[:, 1:] - crow[:, :-1]).reshape(-1)
        return torch.repeat_interleave(torch.arange(B * M, device=crow.device), counts)
    c = to_coo_torch(t)
    idx = c.indices()[:-1]
    dims = list(c.shape[:c.sparse_dim() - 1])
    k = torch.zeros(idx.shape[1], dtype=torch.int64, device=idx.device)
    for d, s in enumerate(dims):
        k = k * s + idx[d]
    return k


def _segment_softmax(v, seg, nseg):
    vf = v.float()
    mx = torch.full((nseg,), float("-inf"), device=v.device).scatter_reduce(0, seg, vf, "amax")
    e = torch.exp(vf - mx[seg])
    den = torch.zeros(nseg, device=v.device).index_add(0, seg, e)
    return (e / den[seg]).to(v.dtype)


def softmax(x, axis=-1, name=None):
    """Softmax over the stored values of each row (last axis), absent entries excluded (reference
    sparse softmax_kernel)."""
    if axis not in (-1, _u(x).dim() - 1):
        raise ValueError("sparse softmax: only the last axis")
    t = _u(x)
    v = _vals(t).reshape(-1)
    real = real_entries(t)
    if real is not None:
        v = v.masked_fill(~real.reshape(-1), float("-inf"))
    seg = _row_ids(t)
    nseg = int(math.prod(t.shape[:-1]))
    return _w(_rebuild(t, torch.nan_to_num(_segment_softmax(v, seg, nseg), nan=0.0)))


def attention(query, key, value, sparse_mask, key_padding_mask=None, attn_mask=None, name=None):
    """Sparse-pattern attention (reference sparse/nn/functional/transformer.py): q/k/v [B, H, S, D] dense,
    sparse_mask CSR [B*H, S, S]: scores only at the mask's nonzeros (SDDMM), row softmax over them, then
    SpMM with V.  key_padding_mask [B, S] / attn_mask [S, S] are additive-0/-inf style 0-1 masks as in the
    reference (0 = masked)."""
    q, k, v = _u(query), _u(key), _u(value)
    B, H, S, D = q.shape
    mt = _u(sparse_mask)
    m = to_coo_torch(mt)
    bh, i, j = m.indices()
    real = real_entries(mt)
    qf, kf, vf = q.reshape(B * H, S, D), k.reshape(B * H, S, D), v.reshape(B * H, S, D)
    sc = (qf[bh, i].float() * kf[bh, j].float()).sum(-1) / math.sqrt(D)
    keep = torch.ones_like(sc, dtype=torch.bool) if real is None else real.reshape(-1).clone()
    if key_padding_mask is not None:
        keep &= _u(key_padding_mask).reshape(B, S)[bh // H, j] != 0
    if attn_mask is not None:
        keep &= _u(attn_mask).reshape(S, S)[i, j] != 0
    sc = sc.masked_fill(~keep, float("-inf"))
    seg = bh * S + i
    p = torch.nan_to_num(_segment_softmax(sc, seg, B * H * S), nan=0.0)
    out = torch.zeros(B * H * S, D, dtype=torch.float32, device=q.device)
    out = out.index_add(0, seg, p[:, None] * vf[bh, j].float())
    return _w(out.reshape(B, H, S, D).to(q.dtype))
