"""CommContextManager / GlooCommContext on 2 spawned gloo ranks, with NO default process group: communicators
are created from a bare TCPStore by key (paddle/phi/core/distributed/comm_context_manager.cc:61-147) and every
NCCLCommContext-style op is checked against its closed-form result."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, out_dir):
    import torch.distributed as dist

    from paddle2_amd.distributed.comm_context import CommContextManager

    store = dist.TCPStore("127.0.0.1", port, 2, rank == 0)
    mgr = CommContextManager.get_instance()
    ctx = CommContextManager.create_gloo_comm_context(store, "ring_7", rank, 2)
    assert mgr.has("ring_7") and mgr.get("ring_7") is ctx and not dist.is_initialized()
    res = {}
    t = torch.full((4,), float(rank + 1))
    ctx.all_reduce(t)
    res["sum"] = t.tolist()
    t = torch.full((4,), float(rank + 1))
    ctx.all_reduce(t, op="max")
    res["max"] = t.tolist()
    t = torch.full((4,), float(rank + 1))
    ctx.all_reduce(t, op=ctx.red_op_create_pre_mul_sum(0.5))
    res["premul"] = t.tolist()
    t = torch.full((2,), float(rank + 1))
    ctx.all_reduce(t, op="avg")
    res["avg"] = t.tolist()
    t = torch.full((2,), float(rank + 1))
    task = ctx.all_reduce(t, op="avg", sync_op=False)  # async AVG: the task finishes the scale on wait()
    task.wait()
    res["avg_async"] = t.tolist()
    t = torch.full((2,), float(rank + 1))
    ctx.reduce(t, root=0, op=ctx.red_op_create_pre_mul_sum(2.0))  # non-root send buffer must stay untouched
    res["reduce_premul"] = t.tolist()
    t = torch.arange(3.0) + 10 * rank
    ctx.broadcast(t, root=1)
    res["bcast"] = t.tolist()
    out = torch.empty(4)
    ctx.all_gather(out, torch.full((2,), float(rank)))
    res["ag"] = out.tolist()
    out = torch.empty(2)
    ctx.reduce_scatter(out, torch.arange(4.0) * (rank + 1))
    res["rs"] = out.tolist()
    t = torch.full((2,), float(rank + 1))
    ctx.reduce(t, root=0)
    res["reduce"] = t.tolist()
    out = torch.empty(4)
    ctx.all_to_all(out, torch.arange(4.0) + 100 * rank)
    res["a2a"] = out.tolist()
    peer = 1 - rank
    got = torch.empty(3)
    ctx.group_start()
    ctx.send(torch.full((3,), float(rank + 5)), peer)
    ctx.recv(got, peer)
    ctx.group_end()
    res["p2p"] = got.tolist()
    # a second communicator on its own key, same store
    ctx2 = CommContextManager.create_gloo_comm_context(store, "pair_0_1", rank, 2)
    t = torch.ones(1) * (rank + 3)
    ctx2.all_reduce(t)
    res["ctx2"] = t.tolist()
    # re-creating an existing key returns the existing communicator (reference comm_context_manager.cc:70)
    again = CommContextManager.create_gloo_comm_context(store, "ring_7", rank, 2)
    res["dup"] = "same" if again is ctx else "different"
    ctx.barrier()
    mgr.release()
    torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))


@pytest.mark.timeout(120)
def test_comm_context_manager_gloo(tmp_path):
    mp.start_processes(_worker, args=(_port(), str(tmp_path)), nprocs=2, start_method="spawn")
    r = [torch.load(tmp_path / f"r{i}.pt", weights_only=True) for i in range(2)]
    for rank, res in enumerate(r):
        assert res["sum"] == [3.0] * 4 and res["max"] == [2.0] * 4 and res["premul"] == [1.5] * 4
        assert res["avg"] == [1.5] * 2
        assert res["bcast"] == [10.0, 11.0, 12.0]
        assert res["ag"] == [0.0, 0.0, 1.0, 1.0]
        assert res["rs"] == ([0.0, 3.0] if rank == 0 else [6.0, 9.0])
        assert res["a2a"] == ([0.0, 1.0, 100.0, 101.0] if rank == 0 else [2.0, 3.0, 102.0, 103.0])
        assert res["p2p"] == [float((1 - rank) + 5)] * 3
        assert res["ctx2"] == [7.0] and res["dup"] == "same"
    assert r[0]["reduce"] == [3.0, 3.0]
