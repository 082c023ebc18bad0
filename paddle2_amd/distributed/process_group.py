"""ProcessGroup objects with the reference's bound method surface (reference:
paddle/fluid/pybind/distributed_py.cc:120-1438 — ``all_reduce`` / ``*_on_calc_stream`` / ``*_partial`` /
``all_to_all*`` / ``scatter*`` / ``gather`` / ``send`` / ``recv`` / ``barrier``, tasks with ``wait`` /
``is_completed`` / ``synchronize``; ``ProcessGroupNCCL.create`` / ``ProcessGroupGloo.create``).

``group.process_group`` returns one of these over the group's c10d backend (RCCL over xGMI on the GPU,
gloo on the CPU).  Ranks in ``src`` / ``dst`` are group-local, as in the reference.  A ``sync_op=True`` call
(and every ``*_on_calc_stream`` call) is ordered on the caller's current HIP stream; ``sync_op=False`` returns a
task whose ``wait()`` makes the current stream wait for it.  ``*_partial`` ops move the ``rank_id``-th of
``nranks`` equal slices (the pipeline's partial send + mp all-gather trick, p2p_communication.py:256-283).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..framework.tensor import Tensor


def _t(x):
    return x._t if isinstance(x, Tensor) else x


def _op(op, backend="nccl"):
    """paddle ReduceOp (None = SUM) -> (c10d op, divide-by-size afterwards?).  AVG on gloo = SUM then divide."""
    from .collective import ReduceOp, _top

    op = ReduceOp.SUM if op is None else op
    if not isinstance(op, int):   # already a c10d ReduceOp
        return op, False
    top = _top(op, backend)
    if top is None:
        return dist.ReduceOp.SUM, True
    return top, False


class Task:
    """ProcessGroup::Task: ``wait`` / ``is_completed`` / ``is_sync`` / ``synchronize``."""

    def __init__(self, work=None, sync=False, post=None):
        self._work, self._sync, self._post = work, sync, post
        self._done = work is None

    def wait(self, timeout=None):
        if not self._done:
            self._work.wait()
            self._done = True
            if self._post is not None:
                self._post()
                self._post = None
        return True

    def is_completed(self):
        return self._done or bool(self._work.is_completed())

    def is_sync(self):
        return self._sync

    def synchronize(self):
        self.wait()
        if torch.cuda.is_available():
            torch.cuda.current_stream().synchronize()


def _slice(t, nranks, rank_id):
    flat = t.reshape(-1)
    n = flat.numel() // nranks
    return flat[rank_id * n:(rank_id + 1) * n]


class ProcessGroup:
    """Wraps a c10d process group (registered via ``new_group`` or created standalone with ``create``)."""

    _backend_name = "gloo"

    def __init__(self, pg, name=None, gid=0):
        self._pg, self._name, self._gid = pg, name, gid

    # ---------------------------------------------------------------- identity
    def rank(self):
        return self._pg.rank()

    def size(self):
        return self._pg.size()

    get_rank = rank
    get_world_size = size

    def name(self):
        return self._name or self._backend_name.upper()

    def get_comm_name(self, rank=None):
        return f"{self.name()}_{self._gid}"

    # ---------------------------------------------------------------- plumbing
    def _run(self, work, sync_op, post=None):
        task = Task(work, sync=sync_op, post=post)
        if sync_op:
            task.wait()
        return task

    # ---------------------------------------------------------------- collectives
    def all_reduce(self, tensor, op=None, sync_op=True):
        t = _t(tensor)
        opts = dist.AllreduceOptions()
        opts.reduceOp, avg = _op(op, self._backend_name)
        n = self.size()
        return self._run(self._pg.allreduce([t], opts), sync_op, post=(lambda: t.div_(n)) if avg else None)

    def all_reduce_on_calc_stream(self, tensor, op=None):
        return self.all_reduce(tensor, op, True)

    def broadcast(self, tensor, src, sync_op=True):
        opts = dist.BroadcastOptions()
        opts.rootRank, opts.rootTensor = int(src), 0
        return self._run(self._pg.broadcast([_t(tensor)], opts), sync_op)

    def broadcast_on_calc_stream(self, tensor, src):
        return self.broadcast(tensor, src, True)

    def reduce(self, tensor, dst, op=None, sync_op=True):
        t = _t(tensor)
        opts = dist.ReduceOptions()
        opts.rootRank, opts.rootTensor = int(dst), 0
        opts.reduceOp, avg = _op(op, self._backend_name)
        n, root = self.size(), self.rank() == int(dst)
        return self._run(self._pg.reduce([t], opts), sync_op, post=(lambda: t.div_(n)) if avg and root else None)

    def reduce_on_calc_stream(self, tensor, dst, op=None):
        return self.reduce(tensor, dst, op, True)

    def all_gather(self, out_tensor_list, in_tensor, sync_op=True):
        """``out_tensor_list``: a list to fill (appended to when empty) or one concatenated output tensor."""
        if isinstance(out_tensor_list, (torch.Tensor, Tensor)):
            return self.all_gather_into_tensor(out_tensor_list, in_tensor, sync_op)
        x = _t(in_tensor)
        outs = [torch.empty_like(x) for _ in range(self.size())]
        fill = out_tensor_list

        def post():
            if fill is not None and len(fill) == 0:
                fill.extend(Tensor._wrap(o) for o in outs)
            elif fill is not None:
                for dst_, o in zip(fill, outs):
                    _t(dst_).copy_(o)

        return self._run(self._pg.allgather([outs], [x]), sync_op, post)

    def all_gather_on_calc_stream(self, out_tensor_list, in_tensor):
        return self.all_gather(out_tensor_list, in_tensor, True)

    def all_gather_into_tensor(self, out_tensor, in_tensor, sync_op=True):
        out, x = _t(out_tensor), _t(in_tensor)
        return self._run(self._pg._allgather_base(out.reshape(-1), x.contiguous().reshape(-1)), sync_op)

    def all_gather_into_tensor_on_calc_stream(self, out_tensor, in_tensor):
        return self.all_gather_into_tensor(out_tensor, in_tensor, True)

    def all_gather_partial(self, out_tensor, in_tensor, nranks, rank_id, sync_op=True):
        """Gather the ``rank_id``-th slices of ``in_tensor`` from every rank into ``out_tensor`` (flat order)."""
        x = _slice(_t(in_tensor), nranks, rank_id).contiguous()
        return self.all_gather_into_tensor(out_tensor, x, sync_op)

    def all_gather_partial_on_calc_stream(self, out_tensor, in_tensor, nranks, rank_id):
        return self.all_gather_partial(out_tensor, in_tensor, nranks, rank_id, True)

    def reduce_scatter(self, out_tensor, in_tensor_list, op=None, sync_op=True):
        return self.reduce_scatter_tensor(out_tensor, torch.cat([_t(x).reshape(-1) for x in in_tensor_list]),
                                          op, sync_op)

    def reduce_scatter_on_calc_stream(self, out_tensor, in_tensor_list, op=None):
        return self.reduce_scatter(out_tensor, in_tensor_list, op, True)

    def reduce_scatter_tensor(self, out_tensor, in_tensor, op=None, sync_op=True):
        out, x = _t(out_tensor), _t(in_tensor).contiguous()
        if self._backend_name == "gloo":   # gloo has no reduce-scatter: all-reduce a copy and keep my slice
            buf = x.reshape(-1).clone()
            opts = dist.AllreduceOptions()
            opts.reduceOp, avg = _op(op, "gloo")
            n, r, w = out.numel(), self.rank(), self.size()

            def post():
                out.reshape(-1).copy_(buf[r * n:(r + 1) * n])
                if avg:
                    out.div_(w)

            return self._run(self._pg.allreduce([buf], opts), sync_op, post=post)
        opts = dist.ReduceScatterOptions()
        opts.reduceOp, _ = _op(op, "nccl")
        return self._run(self._pg._reduce_scatter_base(out.reshape(-1), x.reshape(-1), opts), sync_op)

    def reduce_scatter_tensor_on_calc_stream(self, out_tensor, in_tensor, op=None):
        return self.reduce_scatter_tensor(out_tensor, in_tensor, op, True)

    def all_to_all(self, out_tensor_list, in_tensor_list, sync_op=True):
        ins = [_t(x).contiguous() for x in in_tensor_list]
        outs = [torch.empty_like(x) for x in ins]
        fill = out_tensor_list

        def post():
            if len(fill) == 0:
                fill.extend(Tensor._wrap(o) for o in outs)
            else:
                for dst_, o in zip(fill, outs):
                    _t(dst_).copy_(o)

        if self._backend_name == "gloo":   # gloo: list all-to-all through the flat split form
            sizes = [x.numel() for x in ins]
            flat_out = torch.empty(sum(sizes), dtype=ins[0].dtype, device=ins[0].device)
            flat_in = torch.cat([x.reshape(-1) for x in ins])

            def post_flat():
                for o, piece in zip(outs, flat_out.split(sizes)):
                    o.copy_(piece.view(o.shape))
                post()

            return self._run(self._pg.alltoall_base(flat_out, flat_in, sizes, sizes, dist.AllToAllOptions()),
                             sync_op, post_flat)
        return self._run(self._pg.alltoall(outs, ins, dist.AllToAllOptions()), sync_op, post)

    alltoall = all_to_all

    def all_to_all_on_calc_stream(self, out_tensor_list, in_tensor_list):
        return self.all_to_all(out_tensor_list, in_tensor_list, True)

    def all_to_all_single(self, out_tensor, in_tensor, out_sizes=None, in_sizes=None, sync_op=True):
        out, x = _t(out_tensor), _t(in_tensor).contiguous()
        return self._run(self._pg.alltoall_base(out, x, list(out_sizes or []), list(in_sizes or []),
                                                dist.AllToAllOptions()), sync_op)

    alltoall_single = all_to_all_single

    def all_to_all_single_on_calc_stream(self, out_tensor, in_tensor, out_sizes=None, in_sizes=None):
        return self.all_to_all_single(out_tensor, in_tensor, out_sizes, in_sizes, True)

    def all_to_all_tensor(self, out_tensor, in_tensor, sync_op=True):
        return self.all_to_all_single(out_tensor, in_tensor, None, None, sync_op)

    def all_to_all_tensor_on_calc_stream(self, out_tensor, in_tensor):
        return self.all_to_all_tensor(out_tensor, in_tensor, True)

    def scatter(self, out_tensor, in_tensor_list, src, sync_op=True):
        out = _t(out_tensor)
        opts = dist.ScatterOptions()
        opts.rootRank = int(src)
        ins = [[_t(x).contiguous() for x in in_tensor_list]] if self.rank() == int(src) else []
        return self._run(self._pg.scatter([out], ins, opts), sync_op)

    def scatter_on_calc_stream(self, out_tensor, in_tensor_list, src):
        return self.scatter(out_tensor, in_tensor_list, src, True)

    def scatter_tensor(self, out_tensor, in_tensor, src, sync_op=True):
        x = _t(in_tensor)
        parts = list(x.reshape(-1).chunk(self.size())) if self.rank() == int(src) else []
        parts = [p.reshape(_t(out_tensor).shape) for p in parts]
        return self.scatter(out_tensor, parts, src, sync_op)

    def scatter_tensor_on_calc_stream(self, out_tensor, in_tensor, src):
        return self.scatter_tensor(out_tensor, in_tensor, src, True)

    def gather(self, out_tensor_list, in_tensor, dst, sync_op=True):
        x = _t(in_tensor).contiguous()
        opts = dist.GatherOptions()
        opts.rootRank = int(dst)
        root = self.rank() == int(dst)
        outs = [torch.empty_like(x) for _ in range(self.size())] if root else []
        fill = out_tensor_list

        def post():
            if not root:
                return
            if len(fill) == 0:
                fill.extend(Tensor._wrap(o) for o in outs)
            else:
                for dst_, o in zip(fill, outs):
                    _t(dst_).copy_(o)

        return self._run(self._pg.gather([outs] if root else [], [x], opts), sync_op, post)

    # ---------------------------------------------------------------- point to point
    def send(self, tensor, dst, sync_op=True):
        return self._run(self._pg.send([_t(tensor).contiguous()], int(dst), 0), sync_op)

    def send_on_calc_stream(self, tensor, dst):
        return self.send(tensor, dst, True)

    def recv(self, tensor, src, sync_op=True):
        t = _t(tensor)
        buf = t if t.is_contiguous() else torch.empty_like(t, memory_format=torch.contiguous_format)
        post = None if buf is t else (lambda: t.copy_(buf))
        return self._run(self._pg.recv([buf], int(src), 0), sync_op, post)

    def recv_on_calc_stream(self, tensor, src):
        return self.recv(tensor, src, True)

    def send_partial(self, tensor, dst, nranks, rank_id, sync_op=True):
        return self.send(_slice(_t(tensor), nranks, rank_id).contiguous(), dst, sync_op)

    def send_partial_on_calc_stream(self, tensor, dst, nranks, rank_id):
        return self.send_partial(tensor, dst, nranks, rank_id, True)

    def recv_partial(self, tensor, src, nranks, rank_id, sync_op=True):
        view = _slice(_t(tensor), nranks, rank_id)
        return self.recv(view, src, sync_op)

    def recv_partial_on_calc_stream(self, tensor, src, nranks, rank_id):
        return self.recv_partial(tensor, src, nranks, rank_id, True)

    def barrier(self, device_id=None):
        return self._run(self._pg.barrier(dist.BarrierOptions()), True)

    # ---------------------------------------------------------------- construction
    @classmethod
    def create(cls, store, rank, world_size, group_id=0, timeout=None):
        """Standalone group over ``store`` (a TCPStore / c10d store), like ``core.ProcessGroupNCCL.create``."""
        import datetime

        tout = timeout if isinstance(timeout, datetime.timedelta) else datetime.timedelta(
            seconds=float(timeout) if timeout else 1800.0)
        if cls._backend_name == "nccl":
            opts = dist.ProcessGroupNCCL.Options()
            opts._timeout = tout
            pg = dist.ProcessGroupNCCL(store, rank, world_size, opts)
        else:
            pg = dist.ProcessGroupGloo(store, rank, world_size, tout)
        return cls(pg, gid=group_id)


class ProcessGroupNCCL(ProcessGroup):
    """RCCL over xGMI ("nccl" is RCCL on ROCm)."""

    _backend_name = "nccl"


class ProcessGroupGloo(ProcessGroup):
    _backend_name = "gloo"


class ProcessGroupMPI(ProcessGroup):
    """``core.ProcessGroupMPI`` (reference paddle/fluid/distributed/collective/process_group_mpi.cc): an
    MPI-launched group.  ``create`` takes rank / size from the MPI launcher's environment when not given and runs
    the collectives on gloo (the ROCm PyTorch build has no MPI transport; GPU traffic belongs on RCCL)."""

    _backend_name = "gloo"

    @classmethod
    def create(cls, store=None, rank=None, world_size=None, group_id=0, timeout=None):
        from . import collective as C

        rank = C._rank_env(0) if rank is None else rank
        world_size = C._world_env(1) if world_size is None else world_size
        if store is None:
            import os

            host = os.environ.get("MASTER_ADDR", "127.0.0.1")
            port = int(os.environ.get("MASTER_PORT", "29500"))
            store = dist.TCPStore(host, port, world_size, rank == 0)
        return super().create.__func__(cls, store, rank, world_size, group_id, timeout)

    def name(self):
        return self._name or "MPI"


def wrap(pg, name=None, gid=0):
    """ProcessGroup object for a registered c10d group."""
    backend = dist.get_backend(pg)
    cls = ProcessGroupNCCL if backend == "nccl" else ProcessGroupGloo
    return cls(pg, name=name, gid=gid)
