"""Rank worker: a static Program with recorded collectives (c_allreduce_sum, c_broadcast) run by the
Executor; checks results and the execution plan (comm-stream placement, garbage collection)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
r = dist.get_rank()
main, startup = paddle.static.Program(), paddle.static.Program()
paddle.enable_static()
try:
    with paddle.static.program_guard(main, startup):
        x = paddle.static.data("x", [3], "float32")
        y = x * 2.0
        dist.all_reduce(y)
        z = y + 1.0
        b = x * 1.0
        dist.broadcast(b, src=1)
        w = b - 0.5
finally:
    paddle.disable_static()
exe = paddle.static.Executor()
xv = np.array([1.0, 2.0, 3.0], "float32") * (r + 1)
z_out, w_out = exe.run(main, feed={"x": xv}, fetch_list=[z, w])
from paddle2_amd.static.executor import _plan  # noqa: E402

plan = _plan(main, {z._t._vid, w._t._vid})
names = [getattr(o.fn, "__name__", "") for o in main.ops]
write_result({
    "z": z_out.tolist(), "w": w_out.tolist(),
    "comm_ops": [n for n, s in zip(names, plan.stream_of) if s == "comm"],
    "freed": sum(len(f) for f in plan.free_after),
    "waits": sum(len(w_) for w_ in plan.waits),
})
dist.barrier()
