"""FleetExecutor front-end (reference: python/paddle/distributed/fleet/fleet_executor_utils.py TaskNode /
FleetExecutorUtils, paddle/fluid/distributed/fleet_executor/fleet_executor.cc).

The runtime is native (csrc/runtime/fleet_executor.cpp: Carrier + credit-based Compute / Amplifier / Source /
Sink interceptors on loop threads, TCP message bus between ranks).  Here a ``TaskNode`` holds what one
interceptor runs — a Python callable ``fn(step)`` or a static ``Program`` (run by the Executor with the
step's feed) — and its edges with buffer sizes; ``FleetExecutor`` builds a carrier for this rank, wires the
message bus through the process group's store and runs ``num_micro_batches`` steps.
``FleetExecutorUtils.construct_task_nodes_1f1b`` builds the reference's per-stage
lr / forward / backward / optimizer task graph for a pipeline of stages.
"""
from __future__ import annotations

import itertools

_ROLE = {"Compute": 0, "Amplifier": 1, "Source": 2, "Sink": 3}
_ids = itertools.count(1)


class TaskNode:
    def __init__(self, rank, max_run_times, role=None, node_type="Compute", task_id=None, ops=None, program=None,
                 lazy_initialize=False, cond_var_name=None, vars_to_dtype=None, vars_to_shape=None, fn=None,
                 feed_fn=None, fetch_list=None):
        if node_type not in _ROLE:
            raise ValueError(f"node_type must be one of {sorted(_ROLE)}, got {node_type!r}")
        self.rank = int(rank)
        self.max_run_times = int(max_run_times)
        self.role = role
        self.node_type = node_type
        self.id = int(task_id) if task_id is not None else next(_ids)
        self.program = program
        self.ops = ops
        self.fn = fn
        self.feed_fn = feed_fn
        self.fetch_list = fetch_list
        self.fetches = []
        self.upstream = {}
        self.downstream = {}
        self.run_pre_steps = 1
        self.run_at_offset = 0

    def task_node(self):
        return self

    def set_program(self, program):
        self.program = program

    def get_program(self):
        return self.program

    def set_run_pre_steps(self, steps):
        self.run_pre_steps = int(steps)

    def set_run_at_offset(self, offset):
        self.run_at_offset = int(offset)

    def add_upstream_task(self, upstream, buffer_size=2, depend_type=None):
        self.upstream[int(upstream)] = int(buffer_size)

    def add_downstream_task(self, downstream, buffer_size=2, depend_type=None):
        self.downstream[int(downstream)] = int(buffer_size)

    def task_id(self):
        return self.id

    def _run(self, step):
        if self.fn is not None:
            return self.fn(step)
        if self.program is not None:
            from ...static import Executor

            feed = self.feed_fn(step) if self.feed_fn is not None else {}
            out = Executor().run(self.program, feed=feed, fetch_list=self.fetch_list or [])
            self.fetches.append(out)
            return out
        return None

    def _spec(self):
        from ... import _runtime

        t = _runtime.FleetTask()
        t.id, t.rank, t.role = self.id, self.rank, _ROLE[self.node_type]
        t.max_run_times = self.max_run_times
        t.run_per_steps, t.run_at_offset = self.run_pre_steps, self.run_at_offset
        t.upstream = sorted(self.upstream.items())
        t.downstream = sorted(self.downstream.items())
        return t

    def __repr__(self):
        return (f"TaskNode(id={self.id}, rank={self.rank}, type={self.node_type}, role={self.role}, "
                f"up={self.upstream}, down={self.downstream})")


class FleetExecutor:
    """Runs a task graph: every rank builds the same ``task_nodes`` list and calls ``run()``."""

    def __init__(self, task_nodes, rank=0, num_threads=2, store=None, host="127.0.0.1"):
        from ... import _runtime

        self.nodes = {t.id: t for t in task_nodes}
        self.rank = int(rank)
        self._carrier = _runtime.FleetCarrier(self.rank, num_threads)
        for t in task_nodes:
            self._carrier.add_task(t._spec())
        self._carrier.set_compute(self._compute)
        ranks = sorted({t.rank for t in task_nodes})
        if len(ranks) > 1:
            if store is None:
                store = _default_store()
            port = self._carrier.listen(host)
            store.set(f"fleet_executor/addr/{self.rank}", f"{host}:{port}")
            for r in ranks:
                if r != self.rank:
                    h, p = store.get(f"fleet_executor/addr/{r}").decode().rsplit(":", 1)
                    self._carrier.set_peer(r, h, int(p))

    def _compute(self, task, step):
        self.nodes[task]._run(step)

    def run(self, timeout_s=-1.0):
        self._carrier.clear_trace()
        self._carrier.start()
        if not self._carrier.wait(timeout_s):
            raise TimeoutError("FleetExecutor.run timed out")
        return self._carrier.trace()

    def release(self):
        self._carrier.shutdown()

    def __del__(self):
        try:
            self._carrier.shutdown()
        except Exception:
            pass


def _default_store():
    """The process group's rendezvous store (torch c10d store or the native TCPStore behind it)."""
    import torch.distributed as dist

    if not dist.is_initialized():
        raise RuntimeError("a multi-rank FleetExecutor needs init_parallel_env() (or pass store=)")
    return dist.distributed_c10d._get_default_store()


class FleetExecutorUtils:
    """Task-graph builders (reference FleetExecutorUtils.construct_task_nodes_1f1b)."""

    def __init__(self, dist_strategy=None, rank=0, nrank=1, max_run_times=1):
        self.dist_strategy = dist_strategy or {}
        self.rank, self.nrank = rank, nrank
        self.max_run_times = max_run_times
        self.pp_degree = int(self.dist_strategy.get("pp_degree", nrank)) if isinstance(self.dist_strategy, dict) \
            else nrank

    def build_1f1b_dependency(self, task_node_map):
        """Chain stages: fwd_s -> fwd_{s+1}, bwd_{s+1} -> bwd_s; within a stage lr -> fwd -> bwd -> opt, with
        the 1F1B in-flight bound (stage s may hold pp_degree - s forward results)."""
        stages = sorted(task_node_map)
        for s in stages:
            n = task_node_map[s]
            lr, fwd, bwd, opt = n["lr"], n["fwd"], n["bwd"], n["opt"]
            inflight = self.pp_degree - s
            lr.add_downstream_task(fwd.id, 2)
            fwd.add_upstream_task(lr.id, 2)
            fwd.add_downstream_task(bwd.id, inflight)
            bwd.add_upstream_task(fwd.id, inflight)
            bwd.add_downstream_task(opt.id, 2)
            opt.add_upstream_task(bwd.id, 2)
            if s + 1 in task_node_map:
                nxt = task_node_map[s + 1]
                fwd.add_downstream_task(nxt["fwd"].id, 2)
                nxt["fwd"].add_upstream_task(fwd.id, 2)
                nxt["bwd"].add_downstream_task(bwd.id, 2)
                bwd.add_upstream_task(nxt["bwd"].id, 2)
        return task_node_map

    def construct_task_nodes_1f1b(self, stage_fns, num_micro_batches, stage_rank=None):
        """``stage_fns[s] = {"lr": f, "fwd": f, "bwd": f, "opt": f}`` (callables of the micro-step) ->
        the task node list.  lr / opt are Amplifiers that run once per mini-batch (first / last micro-step)."""
        stage_rank = stage_rank or (lambda s: s)
        nodes = {}
        for s, fns in enumerate(stage_fns):
            r = stage_rank(s)
            base = 1000 * (s + 1)
            lr = TaskNode(r, num_micro_batches, "lr", "Amplifier", base + 0, fn=fns.get("lr"))
            lr.set_run_pre_steps(num_micro_batches)
            lr.set_run_at_offset(0)
            fwd = TaskNode(r, num_micro_batches, "forward", "Compute", base + 1, fn=fns.get("fwd"))
            bwd = TaskNode(r, num_micro_batches, "backward", "Compute", base + 2, fn=fns.get("bwd"))
            opt = TaskNode(r, num_micro_batches, "optimizer", "Amplifier", base + 3, fn=fns.get("opt"))
            opt.set_run_pre_steps(num_micro_batches)
            opt.set_run_at_offset(num_micro_batches - 1)
            nodes[s] = {"lr": lr, "fwd": fwd, "bwd": bwd, "opt": opt}
        self.build_1f1b_dependency(nodes)
        return [t for s in sorted(nodes) for t in nodes[s].values()]
