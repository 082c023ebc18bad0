"""paddle.geometric — graph-learning message passing, segment reductions, neighbour sampling and
re-indexing (reference: python/paddle/geometric/message_passing/send_recv.py:55 send_u_recv,
:210 send_ue_recv, :413 send_uv; math.py:29-209 segment_{sum,mean,min,max};
sampling/neighbors.py:68 sample_neighbors, :256 weighted_sample_neighbors; reindex.py:34
reindex_graph, :153 reindex_heter_graph).

Reductions are one gather + one ``scatter_reduce`` (device atomics) on the tensor's device, so
they are differentiable through torch autograd; rows that receive no message are 0, as in the
reference.
"""
from __future__ import annotations

import numpy as np
import torch

from ..framework.tensor import Tensor

_w = Tensor._wrap
_RED = {"sum": "sum", "mean": "mean", "max": "amax", "min": "amin"}


def _t(x):
    return x._t if isinstance(x, Tensor) else torch.as_tensor(x)


def _out_rows(x_rows, dst, out_size):
    if out_size is None:
        return x_rows
    n = int(out_size.item() if isinstance(out_size, Tensor) else (out_size.item() if torch.is_tensor(out_size)
                                                                  else out_size))
    if n <= 0:
        return x_rows
    return n


def _reduce(msg, dst, rows, reduce_op):
    if reduce_op not in _RED:
        raise ValueError(f"reduce_op must be one of {list(_RED)}, got {reduce_op!r}")
    idx = dst.long().view(-1, *([1] * (msg.dim() - 1))).expand_as(msg)
    out = torch.zeros((rows,) + tuple(msg.shape[1:]), dtype=msg.dtype, device=msg.device)
    return out.scatter_reduce(0, idx, msg, _RED[reduce_op], include_self=False)


def _message(a, b, op):
    if op == "add":
        return a + b
    if op == "sub":
        return a - b
    if op == "mul":
        return a * b
    if op == "div":
        return a / b
    raise ValueError(f"message_op must be add/sub/mul/div, got {op!r}")


def send_u_recv(x, src_index, dst_index, reduce_op="sum", out_size=None, name=None):
    xt, src, dst = _t(x), _t(src_index).long(), _t(dst_index).long()
    msg = xt.index_select(0, src)
    return _w(_reduce(msg, dst, _out_rows(xt.shape[0], dst, out_size), reduce_op))


def send_ue_recv(x, y, src_index, dst_index, message_op="add", reduce_op="sum", out_size=None, name=None):
    xt, yt, src, dst = _t(x), _t(y), _t(src_index).long(), _t(dst_index).long()
    msg = _message(xt.index_select(0, src), yt, message_op)
    return _w(_reduce(msg, dst, _out_rows(xt.shape[0], dst, out_size), reduce_op))


def send_uv(x, y, src_index, dst_index, message_op="add", name=None):
    xt, yt = _t(x), _t(y)
    return _w(_message(xt.index_select(0, _t(src_index).long()), yt.index_select(0, _t(dst_index).long()),
                       message_op))


def _segment(data, segment_ids, op):
    d, ids = _t(data), _t(segment_ids).long()
    rows = int(ids.max().item()) + 1 if ids.numel() else 0
    return _w(_reduce(d, ids, rows, op))


def segment_sum(data, segment_ids, name=None):
    return _segment(data, segment_ids, "sum")


def segment_mean(data, segment_ids, name=None):
    return _segment(data, segment_ids, "mean")


def segment_max(data, segment_ids, name=None):
    return _segment(data, segment_ids, "max")


def segment_min(data, segment_ids, name=None):
    return _segment(data, segment_ids, "min")


# ----------------------------------------------------------------------------- sampling (host graph ops)
def _sample(row, colptr, input_nodes, sample_size, eids, return_eids, weights=None, seed=None):
    r = _t(row).cpu().numpy()
    cp = _t(colptr).cpu().numpy()
    nodes = _t(input_nodes).cpu().numpy()
    e = _t(eids).cpu().numpy() if eids is not None else None
    w = _t(weights).cpu().numpy().astype(np.float64) if weights is not None else None
    rng = np.random.default_rng(seed)
    outs, cnts, oe = [], [], []
    for n in nodes:
        lo, hi = int(cp[n]), int(cp[n + 1])
        deg = hi - lo
        if sample_size < 0 or deg <= sample_size:
            pick = np.arange(lo, hi)
        elif w is None:
            pick = lo + rng.choice(deg, sample_size, replace=False)
        else:
            p = w[lo:hi]
            p = p / p.sum() if p.sum() > 0 else None
            pick = lo + rng.choice(deg, sample_size, replace=False, p=p)
        outs.append(r[pick])
        cnts.append(len(pick))
        if return_eids:
            oe.append(e[pick])
    dev = _t(row).device
    cat = lambda xs, dt: torch.as_tensor(np.concatenate(xs) if xs else np.zeros(0), dtype=dt, device=dev)  # noqa
    res = [_w(cat(outs, _t(row).dtype)), _w(torch.as_tensor(cnts, dtype=torch.int32, device=dev))]
    if return_eids:
        res.append(_w(cat(oe, _t(eids).dtype)))
    return tuple(res)


def sample_neighbors(row, colptr, input_nodes, sample_size=-1, eids=None, return_eids=False, perm_buffer=None,
                     name=None):
    """Uniform neighbour sampling on a CSC graph -> (out_neighbors, out_count[, out_eids])."""
    if return_eids and eids is None:
        raise ValueError("eids must be given when return_eids=True")
    return _sample(row, colptr, input_nodes, sample_size, eids, return_eids)


def weighted_sample_neighbors(row, colptr, edge_weight, input_nodes, sample_size=-1, eids=None, return_eids=False,
                              name=None):
    if return_eids and eids is None:
        raise ValueError("eids must be given when return_eids=True")
    return _sample(row, colptr, input_nodes, sample_size, eids, return_eids, weights=edge_weight)


def _reindex(x, neighbor_lists, count_lists):
    xs = _t(x).cpu().numpy()
    mapping = {int(v): i for i, v in enumerate(xs)}
    order = list(xs)
    srcs, dsts = [], []
    for nb, ct in zip(neighbor_lists, count_lists):
        nb = _t(nb).cpu().numpy()
        ct = _t(ct).cpu().numpy()
        for v in nb:
            v = int(v)
            if v not in mapping:
                mapping[v] = len(order)
                order.append(v)
        srcs.append(np.array([mapping[int(v)] for v in nb], dtype=np.int64))
        dsts.append(np.repeat(np.arange(len(xs), dtype=np.int64), ct))
    dev, dt = _t(x).device, _t(x).dtype
    return (_w(torch.as_tensor(np.concatenate(srcs), dtype=dt, device=dev)),
            _w(torch.as_tensor(np.concatenate(dsts), dtype=dt, device=dev)),
            _w(torch.as_tensor(np.array(order, dtype=np.int64), dtype=dt, device=dev)))


def reindex_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    """-> (reindex_src, reindex_dst, out_nodes): input nodes first, then new neighbours in
    first-appearance order."""
    return _reindex(x, [neighbors], [count])


def reindex_heter_graph(x, neighbors, count, value_buffer=None, index_buffer=None, name=None):
    return _reindex(x, list(neighbors), list(count))


__all__ = ["send_u_recv", "send_ue_recv", "send_uv", "segment_sum", "segment_mean", "segment_min", "segment_max",
           "sample_neighbors", "weighted_sample_neighbors", "reindex_graph", "reindex_heter_graph"]
