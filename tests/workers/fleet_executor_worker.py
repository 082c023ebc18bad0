"""Rank worker: a 2-stage pipeline run by the FleetExecutor across 2 ranks (interceptor control messages over
the native message bus, activations over gloo send/recv inside the compute callbacks)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402
import torch.distributed as tdist  # noqa: E402

import paddle2_amd.distributed as dist  # noqa: E402
from _dist import write_result  # noqa: E402
from paddle2_amd.distributed.fleet.fleet_executor_utils import FleetExecutor, TaskNode  # noqa: E402

dist.init_parallel_env()
r = dist.get_rank()
M = 6
results = []
pending = []


def stage0(step):
    # asynchronous send: the downstream interceptor is only scheduled after this task reports DATA_IS_READY,
    # so a blocking send here would wait on a recv that cannot be posted yet
    x = torch.full((4,), float(step + 1)) * 2.0
    pending.append((tdist.isend(x, dst=1), x))


def stage1(step):
    y = torch.empty(4)
    tdist.recv(y, src=0)
    results.append(float((y + 1.0).sum()))


src = TaskNode(0, M, node_type="Source", task_id=1)
a = TaskNode(0, M, node_type="Compute", task_id=2, fn=stage0)
b = TaskNode(1, M, node_type="Compute", task_id=3, fn=stage1)
sink = TaskNode(1, M, node_type="Sink", task_id=4)
src.add_downstream_task(2, 2)
a.add_upstream_task(1, 2)
a.add_downstream_task(3, 2)
b.add_upstream_task(2, 2)
b.add_downstream_task(4, 2)
sink.add_upstream_task(3, 2)
fe = FleetExecutor([src, a, b, sink], rank=r, num_threads=2)
trace = fe.run(timeout_s=60)
first_trace = [list(t) for t in trace]
# repeated runs with rank 1 lagging: rank 0's next-run DATA_IS_READY reaches rank 1 before its start(); run
# epochs keep the runs apart (no wiped credits, no stale DATA_IS_USELESS from the previous run)
import time  # noqa: E402

for rep in range(4):
    if r == 1:
        time.sleep(0.05 * (rep % 2))
    fe.run(timeout_s=60)
for w, _ in pending:
    w.wait()
dist.barrier()
fe.release()
write_result({"results": results, "trace": first_trace})
