"""Collective API + DataParallel on 2 gloo ranks."""
from _dist import run_workers


def test_collectives_and_dataparallel():
    res = run_workers("collective_worker.py", 2)
    r0, r1 = res
    for r in res:
        assert r["all_reduce"] == [3.0, 3.0, 3.0]
        assert r["all_reduce_max"] == [2.0]
        assert r["all_gather"] == [[0, 0], [1, 10]]
        assert r["broadcast"] == [6.0]
        assert r["all_gather_object"] == [{"rank": 0}, {"rank": 1}]
        assert r["broadcast_object_list"] == [{"x": 1}]
        assert r["group_sum"] == [2.0]
        assert r["dp_diff"] < 1e-5
    assert r0["reduce"] == [3.0]
    assert r0["reduce_scatter"] == [1.0, 4.0] and r1["reduce_scatter"] == [6.0, 4.0]
    assert r0["alltoall"] == [[0], [10]] and r1["alltoall"] == [[1], [11]]
    assert r0["scatter"] == [1.0, 1.0] and r1["scatter"] == [2.0, 2.0]
    assert r1["p2p"] == [42.0]
    assert r0["batch_p2p"] == [1.0] and r1["batch_p2p"] == [0.0]
    assert r1["partial_p2p"] == [100.0, 101.0, 102.0, 103.0, 4.0, 5.0, 6.0, 7.0]
    assert r0["partial_allgather"] == r1["partial_allgather"] == [0.0, 1.0, 2.0, 3.0]


def test_collectives_over_native_store():
    """Same collectives with the process group rendezvousing through the native C++ TCPStore."""
    res = run_workers("collective_worker.py", 2, extra_env={"PADDLE2_AMD_NATIVE_STORE": "1"})
    for r in res:
        assert r["all_reduce"] == [3.0, 3.0, 3.0] and r["dp_diff"] < 1e-5


def test_native_store_api():
    import threading
    import time

    from paddle2_amd.distributed.store import TCPStore

    master = TCPStore("127.0.0.1", 0, is_master=True, world_size=2, timeout=10)
    peer = TCPStore("127.0.0.1", master.port, is_master=False, world_size=2, timeout=10)
    master.set("k", "v")
    assert peer.get("k") == b"v"
    assert master.add("c", 2) == 2 and peer.add("c", 5) == 7
    threading.Timer(0.2, lambda: peer.set("late", b"1")).start()
    t = time.time()
    master.wait("late")
    assert time.time() - t >= 0.15
    th = threading.Thread(target=peer.barrier, args=("b0",))
    th.start()
    master.barrier("b0")
    th.join(5)
    assert not th.is_alive()
    master.shutdown()


def test_fused_comm_buffer_and_collective_perf():
    res = run_workers("fusion_worker.py", 2)
    r0, r1 = res
    assert r0["groups"] == [2]
    # grads after AVG all-reduce are identical on both ranks; x = rank+1+step over 2 steps:
    # d(sum(Wx+b))/dW[j, k] = sum_rows x = 3*x -> averaged over ranks and summed over steps
    exp_w = (3 * (1 + 2) + 3 * (2 + 3)) / 2.0
    assert r0["grads"]["ar"] == r1["grads"]["ar"]
    assert abs(r0["grads"]["ar"][0][0] - exp_w) < 1e-5
    assert abs(r0["grads"]["ar"][1][0] - 3 * 2) < 1e-5  # bias grad: 3 rows x 2 steps, averaged
    for r in res:  # reduce-scatter: each rank's shard holds the averaged values
        assert abs(r["grads"]["rs_shard_head"][0] - (exp_w if r["grads"]["rs_shard_rank"] == 0 else
                                                     r["grads"]["rs_shard_head"][0])) < 1e-5
    assert [p[:2] for p in r0["perf"]] == [[1 << 16, 2], [1 << 18, 2]] and all(p[2] and p[3] for p in r0["perf"])


def test_static_program_collectives_and_plan():
    """Recorded c_allreduce_sum / c_broadcast in a static Program, executed on 2 gloo ranks: values match,
    the stream analyzer puts both on the comm stream with event waits, and GC frees intermediates."""
    res = run_workers("static_comm_worker.py", 2)
    for r in res:
        assert r["z"] == [7.0, 13.0, 19.0]           # 2*(1x + 2x) + 1
        assert r["w"] == [1.5, 3.5, 5.5]             # rank 1's x (2x) - 0.5
        assert r["comm_ops"] == ["c_allreduce_sum", "c_broadcast"]
        assert r["waits"] >= 2 and r["freed"] >= 2


def test_collectives_under_torchrun_agent_store():
    """Launched by torch.distributed.run (the bench.py contract for N > 1): the elastic agent hosts the store on
    MASTER_PORT, so rank 0 must connect to it as a client instead of binding the port again (EADDRINUSE)."""
    import json
    import os
    import subprocess
    import sys
    import tempfile

    from _dist import ROOT, free_port, pypath

    out_dir = tempfile.mkdtemp(prefix="pd_trun_")
    env = dict(os.environ)
    env.update({"PYTHONPATH": pypath(ROOT), "PADDLE2_AMD_DEVICE": "cpu", "OMP_NUM_THREADS": "1",
                "PADDLE_DISTRI_BACKEND": "gloo", "PD_TEST_OUT_DIR": out_dir})
    env.pop("RANK", None)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), os.path.join(ROOT, "tests", "workers", "torchrun_worker.py")]
    p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert p.returncode == 0, p.stdout[-4000:]
    res = []
    for r in range(2):
        with open(os.path.join(out_dir, f"rank{r}.json")) as f:
            res.append(json.load(f))
    for r in res:
        assert r["all_reduce"] == [3.0, 3.0] and r["store"] == "agent"
