"""Context parallelism over the ``sep`` axis: Ulysses all-to-all attention and zigzag ring flash attention.

The reference has a ``sep`` mesh axis (fleet/base/topology.py:240-263, SegmentParallel
meta_parallel/segment_parallel.py:26-40) but leaves the attention-time sequence exchange to user code
(test/collective/fleet/hybrid_parallel_sep_model.py:143-145 splits/concats on the sep group) and has no
ring attention.  Both exchanges are first-class here:

* ``ulysses_attention`` — head<->sequence all-to-all (one ``all_to_all_single`` per tensor over the sep
  group, i.e. one RCCL grouped p2p launch over xGMI), full-sequence flash attention on ``H/sep`` heads,
  all-to-all back.  Needs ``num_heads % sep == 0``; KV heads are replicated up to ``sep`` when GQA
  leaves fewer.
* ``ring_flash_attention`` — each rank keeps its queries and the K/V blocks travel the ring.  Sequences
  are sharded **zigzag** (rank r holds chunks r and 2P-1-r) so every causal step does the same
  c x 2c work on every rank.  The next K/V block is in flight (batched isend/irecv) while the current
  block runs on the MFMA flash kernel; partial results merge with the log-sum-exp.  Backward re-runs
  the same schedule with the final out / lse (flash bwd kernel), dQ accumulates locally and the dK/dV
  partial of each block travels with it, received while the next contribution is computed.

On 288 GB MI355X HBM the per-rank sequence can be long before CP is needed at all; CP degrees map
onto xGMI peers (ring = one link per hop, Ulysses a2a = all 7 links).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ....framework.tensor import Tensor
from ....ops import torch_ops as T
from ...rccl_pg import batch_isend_irecv as _batch_p2p

__all__ = ["ulysses_attention", "ring_flash_attention", "zigzag_shard", "zigzag_unshard", "context_positions",
           "shard_sequence", "SEP_MODES"]

SEP_MODES = ("ulysses", "ring")


def _raw(x):
    return x._t if isinstance(x, Tensor) else x


def _pg_info(group):
    """(torch process group, world, rank-in-group, global ranks) of a paddle Group (None = default)."""
    from ...collective import _get_default_group

    g = group if group is not None else _get_default_group()
    return g.pg, g.nranks, g.rank, list(g.ranks)


# ----------------------------------------------------------------------------------------- sharding helpers
def zigzag_shard(x, world, rank, dim=1):
    """Rank's zigzag shard of a full sequence: chunks (rank, 2*world-1-rank) of 2*world equal chunks."""
    ch = _raw(x).chunk(2 * world, dim)
    out = torch.cat([ch[rank], ch[2 * world - 1 - rank]], dim)
    return Tensor._wrap(out) if isinstance(x, Tensor) else out


def zigzag_unshard(parts, dim=1):
    """Inverse of zigzag_shard given every rank's shard (list ordered by rank)."""
    w = len(parts)
    halves = [p.chunk(2, dim) for p in (_raw(t) for t in parts)]
    order = [halves[i][0] for i in range(w)] + [halves[w - 1 - i][1] for i in range(w)]
    return torch.cat(order, dim)


def context_positions(seq_local, world, rank, mode, device=None):
    """Global token positions of this rank's local sequence (for RoPE)."""
    if mode == "ring":
        c = seq_local // 2
        return torch.cat([torch.arange(rank * c, (rank + 1) * c, device=device),
                          torch.arange((2 * world - 1 - rank) * c, (2 * world - rank) * c, device=device)])
    return torch.arange(rank * seq_local, (rank + 1) * seq_local, device=device)


def shard_sequence(x, world, rank, mode, dim=1):
    """Contiguous (ulysses) or zigzag (ring) shard of a [B, S, ...] batch."""
    if mode == "ring":
        return zigzag_shard(x, world, rank, dim)
    t = _raw(x).chunk(world, dim)[rank]
    return Tensor._wrap(t) if isinstance(x, Tensor) else t


# ----------------------------------------------------------------------------------------------- Ulysses
def _a2a(x, pg, world, scatter_dim, gather_dim):
    """Split x along scatter_dim into `world` pieces, piece j -> rank j; concat received along gather_dim."""
    parts = [p.contiguous() for p in x.chunk(world, scatter_dim)]
    send = torch.stack(parts)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send, group=pg)
    return torch.cat(list(recv.unbind(0)), gather_dim)


class _SeqAllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, pg, world, scatter_dim, gather_dim):
        ctx.meta = (pg, world, scatter_dim, gather_dim)
        return _a2a(x, pg, world, scatter_dim, gather_dim)

    @staticmethod
    def backward(ctx, g):
        pg, world, sd, gd = ctx.meta
        return _a2a(g.contiguous(), pg, world, gd, sd), None, None, None, None


def ulysses_attention(query, key, value, group=None, causal=True, scale=None):
    """q [B, S/P, Hq, D], k/v [B, S/P, Hk, D] (contiguous sequence shards) -> out [B, S/P, Hq, D]."""
    q, k, v = _raw(query), _raw(key), _raw(value)
    pg, world, _, _ = _pg_info(group)
    if world == 1:
        o, _ = T.flash_attention(q, k, v, causal, scale)
        return Tensor._wrap(o) if isinstance(query, Tensor) else o
    hq, hk = q.shape[2], k.shape[2]
    if hq % world:
        raise ValueError(f"ulysses: num_heads {hq} not divisible by sep degree {world}")
    if hk % world:  # GQA with fewer KV heads than ranks: replicate KV heads so every rank gets whole groups
        rep = world // hk if world % hk == 0 else None
        if rep is None:
            raise ValueError(f"ulysses: kv heads {hk} incompatible with sep degree {world}")
        k, v = k.repeat_interleave(rep, 2), v.repeat_interleave(rep, 2)
    qh = _SeqAllToAll.apply(q, pg, world, 2, 1)  # [B, S, Hq/P, D]
    kh = _SeqAllToAll.apply(k, pg, world, 2, 1)
    vh = _SeqAllToAll.apply(v, pg, world, 2, 1)
    o, _ = T.flash_attention(qh, kh, vh, causal, scale)
    out = _SeqAllToAll.apply(o, pg, world, 1, 2)  # back to [B, S/P, Hq, D]
    return Tensor._wrap(out) if isinstance(query, Tensor) else out


# ----------------------------------------------------------------------------------- ring (zigzag) attention
class _Ring:
    """Batched isend/irecv to the next / from the previous rank of the sep ring."""

    def __init__(self, pg, world, rank, ranks):
        self.pg = pg
        self.nxt = ranks[(rank + 1) % world]
        self.prv = ranks[(rank - 1) % world]

    def exchange(self, send, tag):
        recv = torch.empty_like(send)
        ops = [dist.P2POp(dist.isend, send, self.nxt, self.pg, tag),
               dist.P2POp(dist.irecv, recv, self.prv, self.pg, tag)]
        return recv, _batch_p2p(ops)


def _wait(works):
    for w in works:
        w.wait()


def _merge(out, lse, o_b, l_b, rows=None):
    """Online-softmax merge of a block result (o_b [B, r, H, D], l_b [B, H, r]) into fp32 accumulators."""
    if rows is None:
        o_acc, l_acc = out, lse
    else:
        o_acc, l_acc = out[:, rows], lse[:, :, rows]
    l_b = l_b.float()
    l_new = torch.logaddexp(l_acc, l_b)
    w_old = torch.exp(l_acc - l_new).transpose(1, 2).unsqueeze(-1)
    w_new = torch.exp(l_b - l_new).transpose(1, 2).unsqueeze(-1)
    o_acc.copy_(o_acc * w_old + o_b.float() * w_new)
    l_acc.copy_(l_new)


def _step_kind(i, rank, world):
    """0: diagonal (causal over both local chunks), 1: all queries vs the first kv chunk, 2: second query chunk
    vs both kv chunks (zigzag load balance: every kind is c x 2c work)."""
    if i == 0:
        return 0
    src = (rank - i) % world
    return 1 if src < rank else 2


class _RingFlashAttn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, pg, world, rank, ranks, causal, scale):
        ring = _Ring(pg, world, rank, ranks)
        B, S, Hq, D = q.shape
        c = S // 2
        out = torch.zeros(B, S, Hq, D, dtype=torch.float32, device=q.device)
        lse = torch.full((B, Hq, S), float("-inf"), dtype=torch.float32, device=q.device)
        kv = torch.stack([k, v])
        for i in range(world):
            works = None
            if i + 1 < world:
                nxt_kv, works = ring.exchange(kv, tag=1)  # next block in flight during this block's kernel
            kk, vv = kv[0], kv[1]
            if not causal:
                o_b, l_b = T.attn_block_fwd(q, kk, vv, False, scale)
                _merge(out, lse, o_b, l_b)
            else:
                kind = _step_kind(i, rank, world)
                if kind == 0:
                    o_b, l_b = T.attn_block_fwd(q, kk, vv, True, scale)
                    _merge(out, lse, o_b, l_b)
                elif kind == 1:
                    o_b, l_b = T.attn_block_fwd(q, kk[:, :c], vv[:, :c], False, scale)
                    _merge(out, lse, o_b, l_b)
                else:
                    o_b, l_b = T.attn_block_fwd(q[:, c:], kk, vv, False, scale)
                    _merge(out, lse, o_b, l_b, slice(c, S))
            if works is not None:
                _wait(works)
                kv = nxt_kv
        out = out.to(q.dtype)
        ctx.save_for_backward(q, k, v, out, lse)
        ctx.meta = (pg, world, rank, ranks, causal, scale)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, lse = ctx.saved_tensors
        pg, world, rank, ranks, causal, scale = ctx.meta
        ring = _Ring(pg, world, rank, ranks)
        B, S, Hq, D = q.shape
        c = S // 2
        do = dout.contiguous()
        dq = torch.zeros(B, S, Hq, D, dtype=torch.float32, device=q.device)
        kv = torch.stack([k, v])
        part_in = None  # dK/dV partial of the current block, accumulated by the ranks it visited before
        for i in range(world):
            kv_works = None
            if i + 1 < world:
                nxt_kv, kv_works = ring.exchange(kv, tag=2)
            kk, vv = kv[0], kv[1]
            contrib = torch.zeros(2, *kk.shape, dtype=torch.float32, device=q.device)
            kind = _step_kind(i, rank, world) if causal else 3
            if kind in (0, 3):
                gq, gk, gv = T.attn_block_bwd(q, kk, vv, out, do, lse, kind == 0, scale)
                dq += gq.float()
                contrib[0] += gk.float()
                contrib[1] += gv.float()
            elif kind == 1:
                gq, gk, gv = T.attn_block_bwd(q, kk[:, :c], vv[:, :c], out, do, lse, False, scale)
                dq += gq.float()
                contrib[0, :, :c] += gk.float()
                contrib[1, :, :c] += gv.float()
            else:
                gq, gk, gv = T.attn_block_bwd(q[:, c:], kk, vv, out[:, c:], do[:, c:], lse[:, :, c:].contiguous(),
                                              False, scale)
                dq[:, c:] += gq.float()
                contrib[0] += gk.float()
                contrib[1] += gv.float()
            if part_in is not None:
                _wait(part_in[1])
                contrib += part_in[0]
            # hand this block's partial to the next rank (it processes the block next step); the last
            # hand-off delivers every block's complete dK/dV to its owner
            part_in = ring.exchange(contrib, tag=3)
            if kv_works is not None:
                _wait(kv_works)
                kv = nxt_kv
        _wait(part_in[1])
        dkv = part_in[0]
        return dq.to(q.dtype), dkv[0].to(k.dtype), dkv[1].to(v.dtype), None, None, None, None, None, None


def ring_flash_attention(query, key, value, group=None, causal=True, scale=None):
    """q [B, S/P, Hq, D], k/v [B, S/P, Hk, D] zigzag sequence shards (see zigzag_shard) -> out like q."""
    q, k, v = _raw(query), _raw(key), _raw(value)
    if scale is None:
        scale = q.shape[-1] ** -0.5
    pg, world, rank, ranks = _pg_info(group)
    if world == 1:
        o, _ = T.flash_attention(q, k, v, causal, scale)
    else:
        if q.shape[1] % 2:
            raise ValueError("ring_flash_attention: local sequence must hold two equal zigzag chunks")
        o = _RingFlashAttn.apply(q, k, v, pg, world, rank, ranks, bool(causal), float(scale))
    return Tensor._wrap(o) if isinstance(query, Tensor) else o
