"""Pipeline parallelism: 1F1B, FThenB, interleaved (VPP) and zero-bubble (ZB-H1) schedules.

Reference: fleet/meta_parallel/pipeline_parallel.py — ``PipelineParallel`` :255 (1F1B
``forward_backward_pipeline`` :575-763, ``train_batch`` :820, ``eval_batch``),
``PipelineParallelWithInterleave`` :1174 (VPP), ``PipelineParallelWithInterleaveFthenB`` :2256;
p2p in pp_utils/p2p_communication.py (``send_forward_recv_backward`` etc., meta handshake).

Design (not a translation of the reference's hand-unrolled loops): every rank derives the SAME
global schedule by simulating all stages on a logical clock.  Each stage has an ordered unit
list — ``F(chunk, mb)`` / ``B(chunk, mb)`` in 1F1B, FThenB or Megatron-interleaved order — and
executes at most one unit per tick once the unit's producer finished on an earlier tick.  Every
cross-stage hand-off (activation forward, input-grad backward) is assigned to the tick its
producer ran, and at the end of each tick a rank posts ONE ``batch_isend_irecv`` group holding
exactly its sends and the matching receives.  Because both ends of every transfer derive it from
the same simulation and post it in the same tick's group, the schedule is deadlock-free by
construction for any ordering (1F1B, FThenB, VPP with wrap-around ``S-1 -> 0`` hand-offs), and
RCCL runs each group's transfers concurrently over the xGMI peer links.

Zero bubble (ZB-H1, Qi et al. 2023; reference passes/pipeline_scheduler_pass/pipeline_zero_bubble.py): the
backward splits into B (input gradient — what the previous stage waits for) and W (weight gradients, no
cross-stage consumer).  B units run with ops.torch_ops.WeightGradStore deferring every Linear's weight GEMM;
each stage delays its W units by (S - 1 - s) steady steps so they fill the cool-down bubble that 1F1B leaves
idle on the later stages.  Shapes/dtypes cross each
stage boundary once (a small meta handshake on first use), then buffers are allocated directly.

Overlap: a tick's group is posted and NOT waited — receives are waited only when the unit that
consumes them runs (a stream dependency on RCCL, so compute of the next units overlaps the transfer),
sends when the schedule drains.  With tensor parallelism the activations / input grads crossing a stage
boundary are replicated over the mp group, so each mp rank sends only its 1/mp slice and the receiver
all-gathers the slices over mp (the reference's partial_send / partial_recv / partial_allgather,
pp_utils/p2p_communication.py:256-283): the xGMI pipe traffic drops by mp x.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ....framework.tensor import Tensor
from ...collective import ReduceOp
from ...rccl_pg import batch_isend_irecv as _batch_p2p
from ..utils.hybrid_parallel_util import broadcast_dp_parameters, broadcast_mp_parameters, \
    broadcast_sep_parameters, broadcast_sharding_parameters
from ....ops.torch_ops import WeightGradStore
from .meta_parallel_base import MetaParallelBase

_wrap = Tensor._wrap

_DTYPES = [torch.float32, torch.bfloat16, torch.float16, torch.int64, torch.int32, torch.bool, torch.float64,
           torch.uint8]
_META_LEN = 128


# ============================================================================ schedule
def unit_orders(S, s, M, V, schedule="1F1B"):
    """Ordered unit list for stage ``s``: [("F"|"B", chunk, mb)]."""
    total = M * V

    def fwd(k):
        grp, within = divmod(k, S * V)
        chunk, lane = divmod(within, S)
        return chunk, grp * S + lane

    def bwd(k):
        c, mb = fwd(k)
        return V - 1 - c, mb

    if schedule == "ZBH1":
        assert V == 1, "ZB-H1 is a single-chunk schedule"
        warm = min(S - s - 1, M)
        lag = S - s - 1   # W of micro-batch i runs after B of micro-batch i + lag
        out = [("F", 0, k) for k in range(warm)]
        nw = 0
        for i in range(M - warm):
            out.append(("F", 0, warm + i))
            out.append(("B", 0, i))
            if i >= lag:
                out.append(("W", 0, nw))
                nw += 1
        for i in range(M - warm, M):
            out.append(("B", 0, i))
            if nw <= i:
                out.append(("W", 0, nw))
                nw += 1
        out += [("W", 0, k) for k in range(nw, M)]
        return out
    if schedule == "FThenB" or schedule == "F":
        out = [("F",) + fwd(k) for k in range(total)]
        if schedule == "FThenB":
            out += [("B",) + bwd(k) for k in range(total)]
        return out
    if V == 1:
        warm = min(S - s - 1, M)
    else:
        warm = min((S - s - 1) * 2 + (V - 1) * S, total)
    out = [("F",) + fwd(k) for k in range(warm)]
    for i in range(total - warm):
        out.append(("F",) + fwd(warm + i))
        out.append(("B",) + bwd(i))
    out += [("B",) + bwd(k) for k in range(total - warm, total)]
    return out


def simulate(S, M, V, schedule="1F1B"):
    """Run the logical-clock simulation.  Returns (ticks, comms):
    ticks[r]  = list of (tick, unit)  executed by stage r;
    comms[r]  = {tick: [("send"|"recv", peer_stage, key)]}, key = (kind, vstage, mb)."""
    if V > 1 and schedule != "F":
        assert M % S == 0, "interleaved pipeline needs accumulate_steps % pp_degree == 0"
    last = S * V - 1
    orders = [unit_orders(S, r, M, V, schedule) for r in range(S)]
    ptr = [0] * S
    done = {}
    ticks = [[] for _ in range(S)]
    comms = [dict() for _ in range(S)]
    t = 0
    total = sum(len(o) for o in orders)
    finished = 0
    while finished < total:
        progressed = False
        for r in range(S):
            if ptr[r] >= len(orders[r]):
                continue
            kind, c, mb = orders[r][ptr[r]]
            vs = c * S + r
            if kind == "F":
                ready = vs == 0 or done.get(("F", vs - 1, mb), t) < t
            elif kind == "W":
                ready = done.get(("B", vs, mb), t) < t
            else:
                ready = done.get(("F", vs, mb), t) < t and (vs == last or done.get(("B", vs + 1, mb), t) < t)
            if not ready:
                continue
            done[(kind, vs, mb)] = t
            ticks[r].append((t, (kind, c, mb)))
            ptr[r] += 1
            finished += 1
            progressed = True
            if kind == "F" and vs < last:
                dst = (vs + 1) % S
                if dst != r:
                    comms[r].setdefault(t, []).append(("send", dst, (kind, vs, mb)))
                    comms[dst].setdefault(t, []).append(("recv", r, (kind, vs, mb)))
            if kind == "B" and vs > 0:
                dst = (vs - 1) % S
                if dst != r:
                    comms[r].setdefault(t, []).append(("send", dst, (kind, vs, mb)))
                    comms[dst].setdefault(t, []).append(("recv", r, (kind, vs, mb)))
        t += 1
        if not progressed and t > 4 * (total + S * V) + 16:
            raise RuntimeError("pipeline schedule simulation made no progress")
    return ticks, comms


# ============================================================================ helpers
def _split_mb(x, M):
    if x is None:
        return [None] * M
    if isinstance(x, Tensor):
        return [_wrap(t) for t in x._t.chunk(M, dim=0)]
    if isinstance(x, torch.Tensor):
        return [_wrap(t) for t in x.chunk(M, dim=0)]
    if isinstance(x, (tuple, list)):
        parts = [_split_mb(e, M) for e in x]
        return [tuple(p[i] for p in parts) for i in range(M)]
    return [x] * M


def _flat(out):
    """Stage output -> tuple of torch tensors."""
    if isinstance(out, Tensor):
        return (out._t,)
    if isinstance(out, (tuple, list)):
        return tuple(o._t if isinstance(o, Tensor) else o for o in out)
    raise TypeError(f"pipeline stage output must be Tensor(s), got {type(out)}")


def _unflat(ts):
    w = tuple(_wrap(t) for t in ts)
    return w[0] if len(w) == 1 else w


def _is_float(t):
    return t.is_floating_point()


class _GroupWait:
    """Waits a batch's works exactly once (gloo send/recv works block on a second wait)."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        self.works = []


class PipelineParallel(MetaParallelBase):
    _schedule = "1F1B"

    def __init__(self, layers, hcg, strategy):
        super().__init__(layers, hcg, strategy)
        pc = dict(strategy.pipeline_configs) if strategy is not None else {}
        self.accumulate_steps = int(pc.get("accumulate_steps", 1))
        self.micro_batch_size = int(pc.get("micro_batch_size", 1))
        # pp_configs.delay_scale_loss: backward the raw micro-batch losses; the optimizer scales the reduced
        # gradients by 1/accumulate_steps once (HybridParallelOptimizer)
        ppc = strategy.hybrid_configs["pp_configs"] if strategy is not None else {}
        self._delay_scale_loss = bool(ppc.get("delay_scale_loss", False))
        self.num_stages = hcg.get_pipe_parallel_world_size()
        self.stage_id = hcg.get_stage_id()
        self.pp_group = hcg.get_pipe_parallel_group()
        self._pp_ranks = self.pp_group.ranks
        self._V = layers.get_num_virtual_stages() if hasattr(layers, "get_num_virtual_stages") else 1
        self._meta_cache = {}
        self._sim_cache = {}
        self._send_works = []   # this schedule's posted groups, drained when it ends
        self._send_keep = []    # send buffers kept alive until then
        self._device = None
        self._shared_groups = self._make_shared_groups()
        self._sync_shared_weights()
        self.total_loss = None

    # ----------------------------------------------------------------- init sync
    def _prepare_for_model(self):
        hcg = self._hcg
        if hcg.get_model_parallel_world_size() > 1:
            broadcast_mp_parameters(self._layers, hcg)
        if hcg.get_sharding_parallel_world_size() > 1:
            broadcast_sharding_parameters(self._layers, hcg)
        if hcg.get_data_parallel_world_size() > 1:
            broadcast_dp_parameters(self._layers, hcg)
        if hcg.get_sep_parallel_world_size() > 1:
            broadcast_sep_parameters(self._layers, hcg)

    def _make_shared_groups(self):
        from ... import collective as C

        groups = {}
        if not hasattr(self._layers, "_shared_owners"):
            return groups
        topo = self._hcg.topology()
        for key in sorted(self._layers._shared_owners):
            stages = sorted(self._layers._shared_owners[key])
            if len(stages) < 2:
                continue
            for pipe_ranks in topo.get_comm_list("pipe"):
                ranks = [pipe_ranks[s] for s in stages]
                g = C.new_group(ranks)
                if self._hcg.global_rank in ranks:
                    groups[key] = g
        return groups

    def _sync_shared_weights(self):
        for key, p, stages in self._layers.shared_params() if hasattr(self._layers, "shared_params") else []:
            g = self._shared_groups.get(key)
            if g is not None and g.nranks > 1:
                with torch.no_grad():
                    dist.broadcast(p._t.data, src=g.ranks[0], group=g.pg)

    def _allreduce_shared_weight_gradients(self):
        for key, p, stages in self._layers.shared_params() if hasattr(self._layers, "shared_params") else []:
            g = self._shared_groups.get(key)
            if g is None or g.nranks < 2:
                continue
            grad = getattr(p, "main_grad", None)
            grad = grad._t if isinstance(grad, Tensor) else (grad if grad is not None else p._t.grad)
            if grad is None:
                grad = torch.zeros_like(p._t)
                p._t.grad = grad
            dist.all_reduce(grad, group=g.pg)

    # ----------------------------------------------------------------- p2p
    def _peer(self, stage):
        return self._pp_ranks[stage]

    def _encode_meta(self, ts):
        m = torch.zeros(_META_LEN, dtype=torch.int64)
        m[0] = len(ts)
        i = 1
        for t in ts:
            m[i] = _DTYPES.index(t.dtype)
            m[i + 1] = int(t.requires_grad)
            m[i + 2] = t.dim()
            m[i + 3:i + 3 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
            i += 3 + t.dim()
        assert i <= _META_LEN
        return m.to(self._device) if self._comm_on_device() else m

    @staticmethod
    def _decode_meta(m):
        m = m.cpu().tolist()
        out, i = [], 1
        for _ in range(int(m[0])):
            dt, rg, nd = _DTYPES[m[i]], bool(m[i + 1]), m[i + 2]
            out.append((dt, rg, tuple(m[i + 3:i + 3 + nd])))
            i += 3 + nd
        return out

    def _comm_on_device(self):
        return self.pp_group.backend == "nccl"

    def _exchange(self, ops, wait=True, tick=0):
        """ops: list of (is_send, tensor, peer_stage) -> one batched group; returns its works (waited here
        when ``wait``).  Each tensor of a transfer gets its own tag (tick-salted index among the ops with
        that peer and direction) so transports that match by (peer, tag) rather than by issue order (gloo)
        pair them correctly even with several ticks' groups in flight."""
        if not ops:
            return []
        seen = {}
        p2p = []
        for s, t, st in ops:
            k = (s, st)
            tag = seen.get(k, 0)
            seen[k] = tag + 1
            p2p.append(dist.P2POp(dist.isend if s else dist.irecv, t, self._peer(st), group=self.pp_group.pg,
                                  tag=(tick % 4096) * 64 + tag))
        works = _batch_p2p(p2p)
        if wait:
            for w in works:
                w.wait()
            return []
        return works

    # ----------------------------------------------------------------- partial send / recv over mp
    def _partial_mp(self):
        """mp group when boundary tensors are replicated over it (TP without sequence parallel)."""
        if not hasattr(self, "_pmp"):
            pc = dict(self._strategy.pipeline_configs) if self._strategy is not None else {}
            cfg = getattr(self._layers, "config", None) or getattr(self._layers, "_config", None)
            sp = bool(getattr(cfg, "sequence_parallel", False))
            g = self._hcg.get_model_parallel_group()
            on = pc.get("enable_partial_send_recv", True) and not sp and g.nranks > 1
            self._pmp = g if on else None
        return self._pmp

    def _slice_of(self, t):
        g = self._partial_mp()
        if g is None or t.numel() % g.nranks:
            return None
        n = t.numel() // g.nranks
        return t.reshape(-1)[g.rank * n:(g.rank + 1) * n]

    def _gather_partial(self, full):
        g = self._partial_mp()
        n = full.numel() // g.nranks
        flat = full.reshape(-1)
        mine = flat[g.rank * n:(g.rank + 1) * n].clone()
        dist.all_gather_into_tensor(flat, mine, group=g.pg)

    # ----------------------------------------------------------------- engine
    def _run_schedule(self, data, scaler=None, forward_only=False, compute_loss=True):
        S, V, M = self.num_stages, self._V, self.accumulate_steps
        sched = "F" if forward_only else self._schedule
        key = (S, M, V, sched)
        if key not in self._sim_cache:
            self._sim_cache[key] = simulate(S, M, V, sched)
        ticks, comms = self._sim_cache[key]
        me = self.stage_id
        my_ticks = dict(ticks[me])
        my_comms = comms[me]
        last_tick = max(list(my_ticks) + list(my_comms) + [0])
        inputs, labels = (data[0], data[1]) if isinstance(data, (tuple, list)) and len(data) == 2 else (data, None)
        in_mb, lab_mb = _split_mb(inputs, M), _split_mb(labels, M)
        from ....framework.place import current_torch_device

        self._device = current_torch_device()
        last_vs = S * V - 1
        zb = sched == "ZBH1"
        w_queues = {}
        act_in, act_out, losses, outputs = {}, {}, [], []
        pending_send, recv_buf = {}, {}
        loss_fn = getattr(self._layers, "_loss_fn", None)
        for t in range(last_tick + 1):
            u = my_ticks.get(t)
            if u is not None:
                kind, c, mb = u
                vs = c * S + me
                if kind == "F":
                    if vs == 0:
                        x = in_mb[mb]
                        xin = None
                    else:
                        ts = self._take(recv_buf, ("F", vs - 1, mb))
                        xin = tuple(tt.requires_grad_(rg and _is_float(tt)) for tt, rg in ts)
                        x = _unflat(xin)
                    ctx = torch.enable_grad() if not forward_only else torch.no_grad()
                    WeightGradStore.route = zb
                    try:
                        with ctx:
                            y = self._layers(x, chunk_id=c) if V > 1 else self._layers(x)
                    finally:
                        WeightGradStore.route = False
                    with ctx:
                        if vs == last_vs:
                            if loss_fn is not None and compute_loss and lab_mb[mb] is not None:
                                loss = loss_fn(y, lab_mb[mb])
                                loss_t = loss._t if isinstance(loss, Tensor) else loss
                                losses.append(loss_t.detach().float())
                                if not forward_only:
                                    act_out[(vs, mb)] = (loss_t if self._delay_scale_loss else loss_t / M,)
                            else:
                                outputs.append(y)
                                if not forward_only:
                                    act_out[(vs, mb)] = _flat(y)
                        else:
                            yt = _flat(y)
                            if not forward_only:
                                act_out[(vs, mb)] = yt
                            pending_send[("F", vs, mb)] = yt
                    if not forward_only:
                        act_in[(vs, mb)] = xin
                elif kind == "W":  # zero bubble: the deferred weight-gradient GEMMs of (vs, mb)
                    WeightGradStore.run(w_queues.pop((vs, mb), []))
                else:  # backward (ZB-H1: input gradients only, weight GEMMs queued for the W unit)
                    outs = act_out.pop((vs, mb))
                    WeightGradStore.defer = zb
                    try:
                        if vs == last_vs:
                            if scaler is not None and hasattr(scaler, "scale"):
                                l = scaler.scale(_wrap(outs[0]))._t
                            else:
                                l = outs[0]
                            torch.autograd.backward(l)
                        else:
                            grads = self._take(recv_buf, ("B", vs + 1, mb))
                            pairs = [(o, g) for o, g in zip(outs, grads)
                                     if isinstance(o, torch.Tensor) and o.requires_grad and g is not None]
                            if pairs:
                                torch.autograd.backward([o for o, _ in pairs], [g for _, g in pairs])
                    finally:
                        WeightGradStore.defer = False
                    if zb:
                        w_queues[(vs, mb)] = WeightGradStore.take()
                    xin = act_in.pop((vs, mb))
                    if vs > 0 and xin is not None:
                        pending_send[("B", vs, mb)] = tuple(
                            (tt.grad if tt.grad is not None else torch.zeros_like(tt)) if tt.requires_grad else None
                            for tt in xin)
            # ---- communication for this tick (posted, not waited: see _take / the drain below)
            cl = my_comms.get(t)
            if cl:
                self._tick_exchange(cl, pending_send, recv_buf, t)
        for w in self._send_works:
            w.wait()
        self._send_works = []
        self._send_keep = []
        return losses, outputs

    def _take(self, recv_buf, key):
        """Consume a received boundary: wait for its transfer (and all-gather partial slices over mp)."""
        bufs, token, partial = recv_buf.pop(key)
        token.wait()
        for b in partial:
            self._gather_partial(b)
        return bufs

    def _tick_exchange(self, cl, pending_send, recv_buf, tick=0):
        meta_ops, meta_recv = [], []
        for op, peer, key in cl:
            kind, vs, mb = key
            bkey = vs  # boundary vs -> vs+1 (forward) carries the same shapes for every micro-batch
            if kind == "F" and bkey not in self._meta_cache:
                if op == "send":
                    meta = self._encode_meta(pending_send[key])
                    meta_ops.append((True, meta, peer))
                    self._meta_cache[bkey] = [(t.dtype, t.requires_grad, tuple(t.shape)) for t in pending_send[key]]
                else:
                    buf = torch.zeros(_META_LEN, dtype=torch.int64,
                                      device=self._device if self._comm_on_device() else "cpu")
                    meta_ops.append((False, buf, peer))
                    meta_recv.append((bkey, buf))
        if meta_ops:
            self._exchange(meta_ops)
            for bkey, buf in meta_recv:
                self._meta_cache[bkey] = self._decode_meta(buf)
        ops = []
        partial_of = {}
        for op, peer, key in cl:
            kind, vs, mb = key
            if op == "send":
                for t in pending_send[key]:
                    if t is not None:
                        src = t.detach().contiguous()
                        part = self._slice_of(src)
                        ops.append((True, src if part is None else part, peer))
                        self._send_keep.append(src)
            else:
                bmeta = self._meta_cache[vs if kind == "F" else vs - 1]
                bufs, partial = [], []
                for dt, rg, shp in bmeta:
                    if kind == "B" and not (rg and dt.is_floating_point):
                        bufs.append(None)
                        continue
                    b = torch.empty(shp, dtype=dt, device=self._device)
                    part = self._slice_of(b)
                    ops.append((False, b if part is None else part, peer))
                    if part is not None:
                        partial.append(b)
                    bufs.append(b)
                if kind == "F":
                    recv_buf[key] = [(b, rg) for b, (dt, rg, shp) in zip(bufs, bmeta)]
                else:
                    recv_buf[key] = bufs
                partial_of[key] = partial
        works = self._exchange(ops, wait=False, tick=tick)
        # works pair 1:1 with ops; each is waited exactly once (a second wait on a gloo send/recv work
        # blocks): receives when their consumer runs, sends when the schedule drains
        recv_works = [w for w, (is_send, _, _) in zip(works, ops) if not is_send]
        send_works = [w for w, (is_send, _, _) in zip(works, ops) if is_send]
        token = _GroupWait(recv_works)  # the tick's receives complete together; waited once, by any consumer
        for op, peer, key in cl:
            if op == "recv":
                recv_buf[key] = (recv_buf[key], token, partial_of[key])
        self._send_works.extend(send_works)
        for op, peer, key in cl:
            if op == "send":
                pending_send.pop(key, None)

    # ----------------------------------------------------------------- public API
    def forward_backward_pipeline(self, data, scaler=None, static_scheduler=False, return_micro_batch_loss=False):
        self._layers.train()
        losses, _ = self._run_schedule(data, scaler=scaler)
        self._allreduce_shared_weight_gradients()
        return self._broadcast_loss(losses, return_micro_batch_loss)

    def _broadcast_loss(self, losses, per_mb=False):
        M = self.accumulate_steps
        dev = self._device
        if self._hcg.is_last_stage():
            buf = torch.stack(losses).to(dev) if losses else torch.zeros(M, device=dev)
        else:
            buf = torch.zeros(M, device=dev)
        if self.num_stages > 1:
            dist.broadcast(buf, src=self._pp_ranks[-1], group=self.pp_group.pg)
        self.total_loss = buf
        return _wrap(buf.clone()) if per_mb else _wrap(buf.mean())

    def train_batch(self, data, optimizer, lr_scheduler=None, scaler=None, loss_fn_idx=0,
                    return_micro_batch_loss=False):
        assert getattr(self._layers, "_loss_fn", None) is not None, "PipelineLayer needs a loss_fn to train"
        loss = self.forward_backward_pipeline(data, scaler, return_micro_batch_loss=return_micro_batch_loss)
        if scaler is not None:
            scaler.step(optimizer)
            scaler.update()
        else:
            optimizer.step()
        optimizer.clear_grad()
        if lr_scheduler is not None:
            lr_scheduler.step()
        return loss

    def eval_batch(self, data, compute_loss=False, loss_fn_idx=0, return_host_tensor=False):
        self._layers.eval()
        with torch.no_grad():
            losses, outputs = self._run_schedule(data, forward_only=True, compute_loss=compute_loss)
        if compute_loss:
            return self._broadcast_loss(losses)
        return outputs

    def forward(self, *args, **kwargs):
        return self._layers(*args, **kwargs)


class PipelineParallelWithInterleave(PipelineParallel):
    """Virtual pipeline (VPP): each stage holds ``num_virtual_pipeline_stages`` model chunks and runs
    Megatron's interleaved 1F1B order (pipeline_parallel.py:1174)."""

    _schedule = "1F1B"


class PipelineParallelWithInterleaveFthenB(PipelineParallel):
    _schedule = "FThenB"


class PipelineParallelFThenB(PipelineParallel):
    _schedule = "FThenB"


class PipelineParallelZeroBubble(PipelineParallel):
    """ZB-H1: B/W-split backward with the W units delayed into the cool-down bubble."""

    _schedule = "ZBH1"
