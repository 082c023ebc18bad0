"""Rank worker: one static program with device_guard stage annotations (a stage chain, then a generation
while-loop whose body spans every stage) split by HybridParallelInferenceHelper; every rank's result must
equal the unsplit program run locally."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import numpy as np  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed.fleet.utils.hybrid_parallel_inference import HybridParallelInferenceHelper  # noqa
from _dist import write_result  # noqa: E402

num_pp, num_mp = int(sys.argv[1]), int(sys.argv[2])
dist.init_parallel_env()
r = dist.get_rank()
paddle.seed(0)
pre = [paddle.nn.Linear(4, 4) for _ in range(num_pp)]
gen = [paddle.nn.Linear(4, 4) for _ in range(num_pp)]


def build():
    main, startup = paddle.static.Program(), paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, startup):
            with paddle.static.device_guard("gpu:0"):
                x = paddle.static.data("x", [-1, 4], "float32")
            h = x
            for k in range(num_pp):
                with paddle.static.device_guard(f"gpu:{k}"):
                    h = paddle.tanh(pre[k](h))
            with paddle.static.device_guard("gpu:all"):
                i0 = paddle.full([1], 0, "int64")
                n = paddle.full([1], 3, "int64")

            def cond(i, tok):
                return i < n

            def body(i, tok):
                t = tok
                for k in range(num_pp):
                    with paddle.static.device_guard(f"gpu:{k}"):
                        t = paddle.tanh(gen[k](t)) + 0.5 * tok
                with paddle.static.device_guard("gpu:all"):
                    i2 = i + 1
                return i2, t

            i_out, tok_out = paddle.static.nn.while_loop(cond, body, [i0, h])
    finally:
        paddle.disable_static()
    return main, startup, h, i_out, tok_out


xv = np.random.RandomState(1).randn(2, 4).astype("float32")
exe = paddle.static.Executor()
main, _, h, i_out, tok = build()
ref_h, ref_i, ref_tok = exe.run(main, feed={"x": xv}, fetch_list=[h, i_out, tok])
n_ops_full = len(main.ops)

main, startup, h, i_out, tok = build()
helper = HybridParallelInferenceHelper(startup, main, num_mp=num_mp, num_pp=num_pp)
prog = helper.gen_infer_program(["tok"], ["cond_int"])
stage = helper._stage
fetch = [i_out, tok] + ([h] if stage == num_pp - 1 else [])
outs = []
for _ in range(2):   # the split program runs repeatedly (sends drained every run)
    outs = exe.run(prog, feed={"x": xv}, fetch_list=fetch)
names = [o.name for o in prog.ops]
write_result({
    "rank": r, "stage": stage, "pp_group": helper.pp_group, "mp_group": helper.mp_group,
    "i_ok": bool(np.array_equal(outs[0], ref_i)),
    "tok_err": float(np.abs(outs[1] - ref_tok).max()),
    "h_err": float(np.abs(outs[2] - ref_h).max()) if stage == num_pp - 1 else 0.0,
    "n_ops": len(prog.ops), "n_ops_full": n_ops_full,
    "sends": sum("send_v2" in n for n in names), "recvs": sum("recv_v2" in n for n in names),
})
