"""ProcessGroupRCCL: the framework's own RCCL process group, registered as the torch.distributed backend
``"pdrccl"`` so every collective of the framework (collective.py, stage-3 sharding, pipeline p2p, the hybrid
optimizer) runs through it without per-call-site changes.

Reference: paddle/fluid/distributed/collective/process_group_nccl.cc (comm stream + calc<->comm events :840-847,
generic Collective :902, lo->hi p2p comms :1023-1028, RecordStream :966-971, coalescing :999-1037) and
paddle/phi/core/distributed/nccl_comm_context.cc:79-248 (ncclAvg / PreMulSum).

The communicators, streams, event fences and tasks are C++ (csrc/comm/rccl_group.cpp, module
``paddle2_amd._rccl``); this file maps torch's ProcessGroup API onto it:

* tensors are made contiguous (results copied back into non-contiguous outputs after the op);
* every tensor an asynchronous op touches is ``record_stream``-ed on the communicator's stream, so neither
  torch's caching allocator nor the native allocator (csrc/alloc, record-stream hook) hands its memory out
  again before the communication is done (the reference's RecordStream);
* ``Work.wait()`` makes the CURRENT stream wait on the op's end event (no host block); ``synchronize()``
  blocks the host with async-error polling and abort-on-timeout;
* AVG is ncclAvg; PreMulSum(factor) goes through ``all_reduce(..., premul=factor)`` of this class (torch's
  ReduceOp does not expose the factor to Python);
* ``batch_isend_irecv`` (module function) coalesces p2p ops into one RCCL group, which a same-stream
  send-then-recv pair needs to not deadlock.

This group is the default for GPU jobs: collective.init_parallel_env passes backend "pdrccl" to
init_process_group, then ``canary`` checks every collective kind on the real devices and, if any rank's check
fails, every rank falls back to torch's ProcessGroupNCCL on the same store.  ``PADDLE2_AMD_PG=rccl`` demands this
group (a failed check raises instead of falling back); ``PADDLE2_AMD_PG=c10d`` opts out.  The communicator
registry (comm_context.NCCLCommContext) creates this group too.
"""
from __future__ import annotations

import datetime
import os
import sys

import torch
import torch.distributed as dist

BACKEND = "pdrccl"

_DT = {torch.float32: 0, torch.float16: 1, torch.bfloat16: 2, torch.float64: 3, torch.int32: 4, torch.int64: 5,
       torch.int8: 6, torch.uint8: 7, torch.bool: 7}
for _n, _c in (("float8_e4m3fn", 8), ("float8_e5m2", 9)):
    if hasattr(torch, _n):
        _DT[getattr(torch, _n)] = _c

_OPS = {dist.ReduceOp.SUM: 0, dist.ReduceOp.PRODUCT: 1, dist.ReduceOp.MAX: 2, dist.ReduceOp.MIN: 3,
        dist.ReduceOp.AVG: 4}


def _native():
    from .. import _rccl  # noqa: PLC0415

    return _rccl


def _dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise TypeError(f"ProcessGroupRCCL: unsupported dtype {t.dtype}") from None


def _op(op):
    for k, v in _OPS.items():
        if op == k:
            return v
    raise ValueError(f"ProcessGroupRCCL: unsupported reduce op {op} (PreMulSum: use all_reduce(premul=...))")


class _Work(dist.Work):
    """An RCCL task plus the tensors it must keep alive and the copy-backs to run once it is waited on."""

    def __init__(self, task, keep=(), post=None, result=None):
        super().__init__()
        self._task = task
        self._keep = list(keep)
        self._post = post
        self._result = result
        self._done = task is None

    def wait(self, timeout=datetime.timedelta(0)):
        if not self._done:
            self._task.wait(torch.cuda.current_stream().cuda_stream)
            self._done = True
            if self._post is not None:
                self._post()   # copy-backs run on the current stream, after the communication
                self._post = None
        elif self._post is not None:
            self._post()
            self._post = None
        return True

    def is_completed(self):
        return self._task is None or self._task.is_completed()

    def is_success(self):
        return self.is_completed()

    def synchronize(self):
        if self._task is not None:
            self._task.synchronize()
        self.wait()

    def result(self):
        return self._result if self._result is not None else self._keep


class ProcessGroupRCCL(dist.ProcessGroup):
    def __init__(self, store, rank, size, timeout=None, prefix="pg"):
        super().__init__(rank, size)
        self._store = store
        self._dev = torch.cuda.current_device()
        tms = int(timeout.total_seconds() * 1000) if isinstance(timeout, datetime.timedelta) else 1800_000
        self._g = _native().RcclGroup(store, prefix, rank, size, self._dev, tms)
        self._ext = {}
        self._scratch = None
        self._prefix = prefix
        self._nops = 0
        self.last_op = None      # (sequence number, collective, tensor shapes) of the latest launch (hang reports)
        _LIVE.append(self._g)
        _GROUPS.append(self)

    # ------------------------------------------------------------------ plumbing
    def getBackendName(self):
        return BACKEND

    def _stream(self, handle):
        s = self._ext.get(handle)
        if s is None:
            s = self._ext[handle] = torch.cuda.ExternalStream(handle, device=torch.device("cuda", self._dev))
        return s

    def _calc(self):
        return torch.cuda.current_stream(self._dev).cuda_stream

    def _launch(self, fn, tensors, outs=(), use_calc=False, comm_stream=None):
        """run native ``fn(calc_stream, use_calc)`` on contiguous tensors; non-contiguous outputs are copied back
        after the op (on the stream that waits for it)."""
        self._nops += 1
        self.last_op = (self._nops, sys._getframe(1).f_code.co_name, [tuple(t.shape) for t in tensors[:4]])
        task = fn(self._calc(), use_calc)
        if task is not None:
            cs = self._stream(comm_stream if comm_stream is not None else self._g.comm_stream())
            for t in tensors:
                if t.is_cuda:
                    t.record_stream(cs)
        post = None
        if outs:
            def post():
                for dst, src in outs:
                    dst.copy_(src)
        w = _Work(task, tensors, post)
        return w

    @staticmethod
    def _c(t):
        return t if t.is_contiguous() else t.contiguous()

    # ------------------------------------------------------------------ collectives (torch ProcessGroup API)
    def allreduce(self, tensors, opts=None):
        t = tensors[0]
        op = _op(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        return self.all_reduce_native(t, op)

    def all_reduce_native(self, t, op=0, premul=None, sync_op=False, use_calc=False):
        """all_reduce with op code (0 sum, 1 prod, 2 max, 3 min, 4 avg) or ``premul`` = factor (PreMulSum)."""
        c = self._c(t)
        code = 5 if premul is not None else op
        w = self._launch(lambda s, u: self._g.all_reduce(c.data_ptr(), c.data_ptr(), c.numel(), _dt(c), code,
                                                         float(premul or 0.0), s, u),
                         [c], [(t, c)] if c is not t else (), use_calc)
        if sync_op:
            w.wait()
        return w

    def allreduce_coalesced(self, tensors, opts=None):
        op = _op(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        self._g.group_start(self._calc())
        cs = [self._c(t) for t in tensors]
        try:
            for c in cs:
                self._g.all_reduce(c.data_ptr(), c.data_ptr(), c.numel(), _dt(c), op, 0.0, self._calc(), False)
        finally:
            task = self._g.group_end()
        self._record(task, cs)
        return _Work(task, cs, self._copyback([(t, c) for t, c in zip(tensors, cs) if c is not t]))

    def broadcast(self, tensors, opts=None):
        t = tensors[0]
        root = opts.rootRank if opts is not None else 0
        c = self._c(t)
        return self._launch(lambda s, u: self._g.broadcast(c.data_ptr(), c.data_ptr(), c.numel(), _dt(c), root, s, u),
                            [c], [(t, c)] if c is not t else ())

    def reduce(self, tensors, opts=None):
        t = tensors[0]
        root = opts.rootRank if opts is not None else 0
        op = _op(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        c = self._c(t)
        return self._launch(lambda s, u: self._g.reduce(c.data_ptr(), c.data_ptr(), c.numel(), _dt(c), op, 0.0, root,
                                                        s, u), [c], [(t, c)] if c is not t else ())

    def _allgather_base(self, out, inp, opts=None):
        if out.numel() != inp.numel() * self.size():
            raise ValueError("all_gather_into_tensor: output must hold size() x input elements")
        o, i = self._c(out), self._c(inp)
        return self._launch(lambda s, u: self._g.all_gather(i.data_ptr(), o.data_ptr(), i.numel(), _dt(i), s, u),
                            [o, i], [(out, o)] if o is not out else ())

    def allgather_into_tensor_coalesced(self, outs, inps, opts=None):
        self._g.group_start(self._calc())
        pairs = [(self._c(o), self._c(i)) for o, i in zip(outs, inps)]
        try:
            for o, i in pairs:
                self._g.all_gather(i.data_ptr(), o.data_ptr(), i.numel(), _dt(i), self._calc(), False)
        finally:
            task = self._g.group_end()
        keep = [x for p in pairs for x in p]
        self._record(task, keep)
        return _Work(task, keep, self._copyback([(o0, o) for o0, (o, _) in zip(outs, pairs) if o is not o0]))

    def allgather(self, out_lists, inps, opts=None):
        outs, inp = out_lists[0], inps[0]
        flat = torch.empty((self.size(),) + tuple(inp.shape), dtype=inp.dtype, device=inp.device)
        w = self._allgather_base(flat, inp)

        def post():
            for k, o in enumerate(outs):
                o.copy_(flat[k])
        w._post = post
        return w

    def _reduce_scatter_base(self, out, inp, opts=None):
        if inp.numel() != out.numel() * self.size():
            raise ValueError("reduce_scatter_tensor: input must hold size() x output elements")
        op = _op(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        return self.reduce_scatter_native(out, inp, op)

    def reduce_scatter_native(self, out, inp, op=0, premul=None):
        o, i = self._c(out), self._c(inp)
        code = 5 if premul is not None else op
        return self._launch(lambda s, u: self._g.reduce_scatter(i.data_ptr(), o.data_ptr(), o.numel(), _dt(o), code,
                                                                float(premul or 0.0), s, u),
                            [o, i], [(out, o)] if o is not out else ())

    def reduce_scatter_tensor_coalesced(self, outs, inps, opts=None):
        op = _op(opts.reduceOp if opts is not None else dist.ReduceOp.SUM)
        self._g.group_start(self._calc())
        pairs = [(self._c(o), self._c(i)) for o, i in zip(outs, inps)]
        try:
            for o, i in pairs:
                self._g.reduce_scatter(i.data_ptr(), o.data_ptr(), o.numel(), _dt(o), op, 0.0, self._calc(), False)
        finally:
            task = self._g.group_end()
        keep = [x for p in pairs for x in p]
        self._record(task, keep)
        return _Work(task, keep, self._copyback([(o0, o) for o0, (o, _) in zip(outs, pairs) if o is not o0]))

    def reduce_scatter(self, outs, in_lists, opts=None):
        out, ins = outs[0], in_lists[0]
        flat = torch.cat([x.reshape(-1) for x in ins])
        return self._reduce_scatter_base(out, flat, opts)

    def alltoall_base(self, out, inp, out_split_sizes, in_split_sizes, opts=None):
        o, i = self._c(out), self._c(inp)
        n = self.size()
        row_o = o.numel() // max(o.shape[0], 1) if o.dim() else 1
        row_i = i.numel() // max(i.shape[0], 1) if i.dim() else 1
        if not out_split_sizes and not in_split_sizes:
            cnt = i.numel() // n
            fn = lambda s, u: self._g.all_to_all(i.data_ptr(), o.data_ptr(), cnt, _dt(i), s, u)  # noqa: E731
        else:
            ins = list(in_split_sizes) or [i.shape[0] // n] * n
            outs_ = list(out_split_sizes) or [o.shape[0] // n] * n
            sc = [x * row_i for x in ins]
            rc = [x * row_o for x in outs_]
            sd = [sum(sc[:k]) for k in range(n)]
            rd = [sum(rc[:k]) for k in range(n)]
            fn = lambda s, u: self._g.all_to_all_v(i.data_ptr(), o.data_ptr(), sc, sd, rc, rd, _dt(i), s, u)  # noqa
        return self._launch(fn, [o, i], [(out, o)] if o is not out else ())

    def alltoall(self, out_list, in_list, opts=None):
        inp = torch.cat([x.reshape(-1) for x in in_list])
        out = torch.empty(sum(x.numel() for x in out_list), dtype=inp.dtype, device=inp.device)
        sc = [x.numel() for x in in_list]
        rc = [x.numel() for x in out_list]
        sd = [sum(sc[:k]) for k in range(len(sc))]
        rd = [sum(rc[:k]) for k in range(len(rc))]
        w = self._launch(lambda s, u: self._g.all_to_all_v(inp.data_ptr(), out.data_ptr(), sc, sd, rc, rd, _dt(inp),
                                                           s, u), [out, inp])

        def post():
            for k, o in enumerate(out_list):
                o.copy_(out[rd[k]:rd[k] + rc[k]].view_as(o))
        w._post = post
        return w

    def send(self, tensors, dst, tag=0):
        t = self._c(tensors[0])
        return self._launch(lambda s, u: self._g.send(t.data_ptr(), t.numel(), _dt(t), dst, s, u), [t],
                            comm_stream=self._g.p2p_stream(dst))

    def recv(self, tensors, src, tag=0):
        t0 = tensors[0]
        t = self._c(t0)
        return self._launch(lambda s, u: self._g.recv(t.data_ptr(), t.numel(), _dt(t), src, s, u), [t],
                            [(t0, t)] if t is not t0 else (), comm_stream=self._g.p2p_stream(src))

    def barrier(self, opts=None):
        if self._scratch is None:
            self._scratch = torch.zeros(1, dtype=torch.int32, device=torch.device("cuda", self._dev))
        self._g.barrier(self._scratch.data_ptr(), self._calc())
        return _Work(None)

    def abort(self):
        self._g.abort()

    # ------------------------------------------------------------------ helpers
    def _record(self, task, tensors):
        if task is None:
            return
        cs = self._stream(self._g.comm_stream())
        for t in tensors:
            t.record_stream(cs)

    @staticmethod
    def _copyback(pairs):
        if not pairs:
            return None

        def post():
            for dst, src in pairs:
                dst.copy_(src)
        return post

    def batch_p2p(self, ops):
        """[(is_send, tensor, peer)] as ONE RCCL group; returns one Work per op (sharing the group's task)."""
        calc = self._calc()
        # create every pair communicator before opening the group (creation is not allowed inside it)
        for _, _, peer in ops:
            self._g.p2p_stream(peer)
        conts = [(s, self._c(t), t, p) for s, t, p in ops]
        self._g.group_start(calc)
        try:
            for s, c, _, p in conts:
                if s:
                    self._g.send(c.data_ptr(), c.numel(), _dt(c), p, calc, False)
                else:
                    self._g.recv(c.data_ptr(), c.numel(), _dt(c), p, calc, False)
        finally:
            task = self._g.group_end()
        for s, c, _, p in conts:
            if task is not None:
                c.record_stream(self._stream(self._g.p2p_stream(p)))
        post = self._copyback([(t, c) for s, c, t, _ in conts if not s and c is not t])
        w = _Work(task, [c for _, c, _, _ in conts], post)
        return [w] * len(ops)


_LIVE = []   # every native group: torn down at interpreter exit, before the HIP runtime's own atexit teardown
_GROUPS = []  # the Python groups, for last_ops()


def last_ops():
    """The latest collective launched on every ProcessGroupRCCL of this process: [{group, rank, size, seq, op,
    shapes}] — what a hang report prints (the reference comm_task_manager's last-started task per group)."""
    out = []
    for g in _GROUPS:
        seq, op, shapes = g.last_op if g.last_op is not None else (0, None, [])
        out.append({"group": g._prefix, "rank": g.rank(), "size": g.size(), "seq": seq, "op": op, "shapes": shapes})
    return out


def shutdown_all():
    while _LIVE:
        _LIVE.pop().shutdown()


import atexit as _atexit  # noqa: E402

_atexit.register(shutdown_all)


def _create(store, rank, size, timeout):
    return ProcessGroupRCCL(store, rank, size, timeout)


_registered = False


def register():
    """Register the "pdrccl" backend with torch.distributed (idempotent)."""
    global _registered
    if not _registered:
        dist.Backend.register_backend(BACKEND, _create, devices=["cuda"])
        _registered = True
    return BACKEND


def enabled():
    """The own process group is the default for GPU jobs; ``PADDLE2_AMD_PG=c10d`` (or torch / nccl) selects torch's
    ProcessGroupNCCL instead."""
    v = os.environ.get("PADDLE2_AMD_PG", "").lower()
    if v in ("c10d", "torch", "nccl", "0", "off"):
        return False
    return True


def requested():
    """The user asked for this group explicitly (no fallback to c10d if its start-up check fails)."""
    return os.environ.get("PADDLE2_AMD_PG", "").lower() in ("rccl", "native", BACKEND)


def _agree(store, key, rank, world, mine, timeout_s=300.0):
    """Every rank publishes ``mine`` (str) under key/<rank>; returns the list of all ranks' values."""
    import time

    store.set(f"{key}/{rank}", mine)
    out = []
    t0 = time.time()
    for r in range(world):
        while True:
            try:
                out.append(store.get(f"{key}/{r}").decode())
                break
            except Exception:
                if time.time() - t0 > timeout_s:
                    out.append("missing")
                    break
                time.sleep(0.05)
    return out


def canary(store, rank, world, timeout_ms=120_000):
    """Start-up check of the default ProcessGroupRCCL on the real devices: all-reduce (sum, avg), all-gather,
    reduce-scatter and a ring of pair-communicator send / recv (one coalesced group), each host-synchronised
    with a bounded wait (a hang aborts the communicator instead of blocking) and checked exactly.  Every rank
    publishes its verdict through the store; returns (all_ok, verdicts)."""
    status = "ok"
    try:
        pg = dist.distributed_c10d._get_default_group()
        if isinstance(pg, dist.ProcessGroup) and not isinstance(pg, ProcessGroupRCCL):
            try:
                pg = pg._get_backend(torch.device("cuda"))
            except Exception:
                pass
        if not isinstance(pg, ProcessGroupRCCL):
            raise RuntimeError(f"default group is {type(pg).__name__}, not ProcessGroupRCCL")
        old = pg._g.timeout_ms
        pg._g.timeout_ms = timeout_ms
        try:
            dev = torch.device("cuda", torch.cuda.current_device())
            tri = world * (world + 1) / 2
            t = torch.full((1024,), float(rank + 1), device=dev)
            pg.all_reduce_native(t, 0).synchronize()
            a = torch.full((256,), float(rank + 1), device=dev, dtype=torch.bfloat16)
            pg.all_reduce_native(a, 4).synchronize()
            ag = torch.empty(world * 8, device=dev)
            pg._allgather_base(ag, torch.full((8,), float(rank), device=dev)).synchronize()
            rs = torch.empty(8, device=dev)
            pg.reduce_scatter_native(rs, torch.arange(world * 8, device=dev, dtype=torch.float32)).synchronize()
            nxt, prv = (rank + 1) % world, (rank - 1) % world
            recv = torch.zeros(16, device=dev)
            works = pg.batch_p2p([(True, torch.full((16,), float(rank), device=dev), nxt), (False, recv, prv)])
            works[0].synchronize()
            torch.cuda.synchronize()
            exp_ag = torch.arange(world, device=dev, dtype=torch.float32).repeat_interleave(8)
            exp_rs = world * torch.arange(rank * 8, rank * 8 + 8, device=dev, dtype=torch.float32)
            bad = []
            if not bool((t == tri).all()):
                bad.append("all_reduce")
            if not bool((a.float() == tri / world).all()):
                bad.append("avg")
            if not torch.equal(ag, exp_ag):
                bad.append("all_gather")
            if not torch.equal(rs, exp_rs):
                bad.append("reduce_scatter")
            if not bool((recv == float(prv)).all()):
                bad.append("p2p")
            if bad:
                status = "mismatch:" + ",".join(bad)
        finally:
            pg._g.timeout_ms = old
    except Exception as e:   # noqa: BLE001 - any failure means: do not use this group
        status = f"error:{type(e).__name__}:{str(e)[:200]}"
    verdicts = _agree(store, "pdrccl_canary", rank, world, status)
    return all(v == "ok" for v in verdicts), verdicts


def batch_isend_irecv(p2p_ops):
    """torch-style P2POp list -> works; RCCL-group coalescing on a ProcessGroupRCCL, torch's path otherwise."""
    if not p2p_ops:
        return []
    pg = p2p_ops[0].group
    if pg is None:
        pg = dist.group.WORLD
    if isinstance(pg, ProcessGroupRCCL):
        ops = []
        for p in p2p_ops:
            is_send = p.op in (dist.isend, dist.send)
            peer = p.peer if getattr(p, "group_peer", None) is None else p.group_peer
            ops.append((is_send, p.tensor, dist.get_group_rank(pg, peer) if p.group is not None else peer))
        return pg.batch_p2p(ops)
    return dist.batch_isend_irecv(p2p_ops)
