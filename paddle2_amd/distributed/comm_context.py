"""Communicator registry: ``CommContextManager`` + ``NCCLCommContext`` / ``GlooCommContext``.

Reference parity: paddle/phi/core/distributed/comm_context_manager.cc:61-147 (communicators keyed by a
``unique_comm_key``; rank 0 publishes the unique id in the store, the others fetch it, then every rank inits)
and paddle/phi/core/distributed/nccl_comm_context.cc:79-248 (Broadcast / AllGather / ReduceScatter / Send /
Recv / AllReduce / Reduce / GroupStart / GroupEnd / RedOpCreatePreMulSum).

MI355X design: a context owns one c10d process group built directly on a ``PrefixStore(key, store)`` — no
default group and no world registration are needed, so a ring (TP ring, a 2-rank p2p pair, a DP bucket ring)
can be created for any rank subset from any store (torch TCPStore or this framework's native TCPStore
adapter).  On ROCm the ``nccl`` backend *is* RCCL over xGMI: ProcessGroupNCCL does exactly the reference's
unique-id exchange through the store (rank 0 ``ncclGetUniqueId`` -> store -> ``ncclCommInitRank``).  Gloo
contexts cover CPU tensors.  Collectives run on the group's own stream (RCCL) and return when enqueued;
``sync_op`` (default) waits for completion.
"""
from __future__ import annotations

import datetime
import threading

import torch
import torch.distributed as dist

__all__ = ["CommContext", "NCCLCommContext", "GlooCommContext", "CommContextManager", "PreMulSum"]

_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN, "prod": dist.ReduceOp.PRODUCT,
        "avg": dist.ReduceOp.SUM}


class _PostTask:
    """Async task of a collective whose result still needs a scale (gloo AVG / PreMulSum): wait() completes the
    collective, then applies the scale exactly once."""

    def __init__(self, work, fn):
        self._work, self._fn, self._done = work, fn, False

    def wait(self, timeout=None):
        if not self._done:
            self._work.wait()
            self._fn()
            self._done = True
        return True

    def is_completed(self):
        return self._done or self._work.is_completed()


class PreMulSum:
    """``RedOpCreatePreMulSum``: sum of ``scalar * x`` over ranks (the gradient-averaging reduction)."""

    def __init__(self, scalar):
        self.scalar = scalar


def _redop(op):
    if isinstance(op, dist.ReduceOp) or type(op).__name__ == "RedOpType":
        return op
    if isinstance(op, int):  # paddle.distributed.ReduceOp ints: SUM 0, MAX 1, MIN 2, PROD 3, AVG 4
        return [dist.ReduceOp.SUM, dist.ReduceOp.MAX, dist.ReduceOp.MIN, dist.ReduceOp.PRODUCT, dist.ReduceOp.SUM][op]
    return _OPS[str(op).lower()]


def _is_avg(op):
    return op == 4 or (isinstance(op, str) and op.lower() == "avg")


class CommContext:
    """One communicator (rank ``rank`` of ``size``) on its own process group."""

    backend = None

    def __init__(self, store, unique_comm_key, rank, size, timeout=datetime.timedelta(seconds=1800)):
        if not 0 <= rank < size:
            raise ValueError(f"rank {rank} out of range for a communicator of size {size}")
        self.key = str(unique_comm_key)
        self.rank, self.size = int(rank), int(size)
        self.store = dist.PrefixStore(f"{type(self).__name__}/{self.key}/", store)
        self.pg = self._make_pg(self.store, self.rank, self.size, timeout)
        self._batch = None  # pending p2p ops between group_start() and group_end()

    def _make_pg(self, store, rank, size, timeout):  # pragma: no cover - overridden
        raise NotImplementedError

    # ---------------------------------------------------------------- helpers
    @staticmethod
    def _done(work, sync_op):
        if sync_op:
            work.wait()
            return None
        return work

    def _reduce_op(self, op):
        """-> (c10d op, post scale).  RCCL: AVG is ncclAvg and PreMulSum is ncclRedOpCreatePreMulSum, both inside
        the collective (nccl_comm_context.cc:79-248); gloo has neither, so SUM plus a scale applied to the
        RESULT once the work completes (never to the caller's input)."""
        if isinstance(op, PreMulSum):
            if self.backend == "nccl" and hasattr(dist, "_make_nccl_premul_sum"):
                return dist._make_nccl_premul_sum(float(op.scalar)), None
            return dist.ReduceOp.SUM, float(op.scalar)
        if _is_avg(op):
            if self.backend == "nccl":
                return dist.ReduceOp.AVG, None
            return dist.ReduceOp.SUM, 1.0 / self.size
        return _redop(op), None

    def _post(self, work, sync_op, fn):
        """Finish ``work`` then run ``fn`` (a result scale): now if sync_op, else on the returned task's wait()."""
        if sync_op:
            work.wait()
            fn()
            return None
        return _PostTask(work, fn)

    # ---------------------------------------------------------------- collectives
    def all_reduce(self, tensor, op="sum", sync_op=True):
        from .rccl_pg import ProcessGroupRCCL

        if isinstance(self.pg, ProcessGroupRCCL) and isinstance(op, PreMulSum):
            # the framework's RCCL group takes the factor directly (ncclRedOpCreatePreMulSum)
            return self._done(self.pg.all_reduce_native(tensor, premul=float(op.scalar)), sync_op)
        rop, post = self._reduce_op(op)
        o = dist.AllreduceOptions()
        o.reduceOp = rop
        w = self.pg.allreduce([tensor], o)
        if post is not None:
            return self._post(w, sync_op, lambda: tensor.mul_(post))
        return self._done(w, sync_op)

    def broadcast(self, tensor, root, sync_op=True):
        o = dist.BroadcastOptions()
        o.rootRank, o.rootTensor = int(root), 0
        return self._done(self.pg.broadcast([tensor], o), sync_op)

    def reduce(self, tensor, root, op="sum", sync_op=True):
        rop, post = self._reduce_op(op)
        o = dist.ReduceOptions()
        o.rootRank, o.rootTensor, o.reduceOp = int(root), 0, rop
        if post is None:
            return self._done(self.pg.reduce([tensor], o), sync_op)
        # gloo post scale: reduce a copy so a non-root rank's send buffer stays untouched, scale on the root only
        buf = tensor.clone()
        w = self.pg.reduce([buf], o)

        def fin():
            if self.rank == int(root):
                tensor.copy_(buf.mul_(post))
        return self._post(w, sync_op, fin)

    def all_gather(self, out, tensor, sync_op=True):
        """``out``: a [size * n, ...] tensor (rank-major) or a list of ``size`` tensors."""
        if isinstance(out, (list, tuple)):
            return self._done(self.pg.allgather([list(out)], [tensor]), sync_op)
        parts = list(out.chunk(self.size, 0))
        if all(p.is_contiguous() for p in parts):
            return self._done(self.pg.allgather([parts], [tensor]), sync_op)
        tmp = [torch.empty_like(tensor) for _ in range(self.size)]
        self.pg.allgather([tmp], [tensor]).wait()
        torch.cat(tmp, 0, out=out)
        return None

    def reduce_scatter(self, out, tensor, op="sum", sync_op=True):
        """``out`` (n rows) = this rank's slice of the reduction of ``tensor`` ([size * n, ...])."""
        t = tensor
        rop, post = self._reduce_op(op)
        if self.backend == "nccl":
            o = dist.ReduceScatterOptions()
            o.reduceOp = rop
            w = self.pg._reduce_scatter_base(out, t, o)
            w.wait() if (sync_op or post is not None) else None
        else:  # gloo has no reduce-scatter: all-reduce a copy, keep this rank's slice
            full = t.clone() if t is tensor else t
            o = dist.AllreduceOptions()
            o.reduceOp = rop
            self.pg.allreduce([full], o).wait()
            out.copy_(full.chunk(self.size, 0)[self.rank])
            w = None
        if post is not None:
            out.mul_(post)
        return None if (sync_op or w is None) else w

    def all_to_all(self, out, tensor, sync_op=True):
        """Equal splits along dim 0."""
        if self.backend == "nccl":
            return self._done(self.pg.alltoall_base(out, tensor, [], [], dist.AllToAllOptions()), sync_op)
        ins = list(tensor.chunk(self.size, 0))
        outs = list(out.chunk(self.size, 0))
        for peer in range(self.size):  # gloo: pairwise exchange in rank order (no deadlock: lower rank sends first)
            if peer == self.rank:
                outs[peer].copy_(ins[peer])
                continue
            if self.rank < peer:
                self.pg.send([ins[peer].contiguous()], peer, 0).wait()
                buf = torch.empty_like(outs[peer])
                self.pg.recv([buf], peer, 0).wait()
            else:
                buf = torch.empty_like(outs[peer])
                self.pg.recv([buf], peer, 0).wait()
                self.pg.send([ins[peer].contiguous()], peer, 0).wait()
            outs[peer].copy_(buf)
        return None

    # ---------------------------------------------------------------- point to point
    def send(self, tensor, peer, sync_op=True):
        if self._batch is not None:
            self._batch.append(("send", tensor, int(peer)))
            return None
        return self._done(self.pg.send([tensor], int(peer), 0), sync_op)

    def recv(self, tensor, peer, sync_op=True):
        if self._batch is not None:
            self._batch.append(("recv", tensor, int(peer)))
            return None
        return self._done(self.pg.recv([tensor], int(peer), 0), sync_op)

    def group_start(self):
        """``GroupStart``: queue send/recv until ``group_end`` (issued together so pairwise exchanges cannot
        deadlock on rendezvous order)."""
        self._batch = []

    def group_end(self):
        batch, self._batch = self._batch or [], None
        if not batch:
            return
        if self.backend == "nccl":  # one RCCL group launch (ncclGroupStart/End) for the whole batch
            from .rccl_pg import ProcessGroupRCCL

            if isinstance(self.pg, ProcessGroupRCCL):
                for w in self.pg.batch_p2p([(kind == "send", t, peer) for kind, t, peer in batch]):
                    w.wait()
                return
            dev = torch.device(self._device())
            self.pg._start_coalescing(dev)
            for kind, t, peer in batch:
                (self.pg.send if kind == "send" else self.pg.recv)([t], peer, 0)
            self.pg._end_coalescing(dev).wait()
            return
        # gloo sends are asynchronous (buffered until matched): post every send, then every receive
        works = [self.pg.send([t], peer, 0) for kind, t, peer in batch if kind == "send"]
        works += [self.pg.recv([t], peer, 0) for kind, t, peer in batch if kind == "recv"]
        for w in works:
            w.wait()

    def red_op_create_pre_mul_sum(self, scalar):
        return PreMulSum(scalar)

    def barrier(self):
        t = torch.zeros(1, device=self._device())
        self.all_reduce(t)

    def _device(self):
        return "cpu"

    def get_rank(self):
        return self.rank

    def get_size(self):
        return self.size


class NCCLCommContext(CommContext):
    """RCCL communicator: the framework's own ProcessGroupRCCL (csrc/comm/rccl_group.cpp — unique id exchanged
    through the store, own comm stream and event fences), as the default process group is; PADDLE2_AMD_PG=c10d
    selects torch's ProcessGroupNCCL for both (reference comm_context_manager.cc:61-122 CreateNCCLCommContext)."""

    backend = "nccl"

    def _make_pg(self, store, rank, size, timeout):
        from . import rccl_pg

        if rccl_pg.enabled():
            return rccl_pg.ProcessGroupRCCL(store, rank, size, timeout, prefix=f"ctx/{self.key}")
        opts = dist.ProcessGroupNCCL.Options()
        opts._timeout = timeout
        return dist.ProcessGroupNCCL(store, rank, size, opts)

    def _device(self):
        return f"cuda:{torch.cuda.current_device()}"


class GlooCommContext(CommContext):
    backend = "gloo"

    def _make_pg(self, store, rank, size, timeout):
        return dist.ProcessGroupGloo(store, rank, size, timeout)


class CommContextManager:
    """Process-wide registry of communicators keyed by ``unique_comm_key`` (comm_context_manager.cc)."""

    _instance = None
    _lock = threading.Lock()

    def __init__(self):
        self._ctx = {}
        self._store = None

    @classmethod
    def get_instance(cls):
        with cls._lock:
            if cls._instance is None:
                cls._instance = cls()
            return cls._instance

    # store used when a create_* call passes none (the reference's SetStore)
    def set_store(self, store):
        self._store = store

    def get_store(self):
        return self._store

    def _create(self, kind, store, unique_comm_key, rank, size, **kw):
        key = str(unique_comm_key)
        if key in self._ctx:  # the reference returns the existing communicator (comm_context_manager.cc:70)
            return self._ctx[key]
        store = store if store is not None else self._store
        if store is None:
            raise ValueError("no store: pass one or call CommContextManager.set_store first")
        ctx = kind(store, key, rank, size, **kw)
        self._ctx[key] = ctx
        return ctx

    @staticmethod
    def create_nccl_comm_context(store, unique_comm_key, rank, size, hash_key="", **kw):
        return CommContextManager.get_instance()._create(NCCLCommContext, store, unique_comm_key, rank, size, **kw)

    @staticmethod
    def create_gloo_comm_context(store, unique_comm_key, rank, size, **kw):
        return CommContextManager.get_instance()._create(GlooCommContext, store, unique_comm_key, rank, size, **kw)

    def set(self, unique_comm_key, ctx):
        self._ctx[str(unique_comm_key)] = ctx

    def get(self, unique_comm_key):
        key = str(unique_comm_key)
        if key not in self._ctx:
            raise KeyError(f"communicator {key!r} not found; create it first")
        return self._ctx[key]

    def has(self, unique_comm_key):
        return str(unique_comm_key) in self._ctx

    def release(self, unique_comm_key=None):
        keys = list(self._ctx) if unique_comm_key is None else [str(unique_comm_key)]
        for k in keys:
            ctx = self._ctx.pop(k, None)
            if ctx is not None and hasattr(ctx.pg, "shutdown"):
                try:
                    ctx.pg.shutdown()
                except Exception:  # noqa: BLE001 - best-effort teardown
                    pass
