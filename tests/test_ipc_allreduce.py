"""IPC one-shot / two-shot all-reduce (csrc/kernels/ipc_allreduce.hip, distributed/ipc_allreduce.py).

CPU: the kernel's element-ownership model (every vector reduced exactly once, gathers cover the rest) and the
64-byte handle exchange over a 2-rank gloo group.  GPU: the kernel and its cross-"rank" flag barriers with
2-4 simulated ranks in one process (one stream each, buffers addressed directly) vs torch.sum in rank order,
and hipIpcGetMemHandle on the uncached allocation.  Multi-GPU timing needs an 8-GPU node (not run here)."""
import os

import pytest
import torch

from paddle2_amd.distributed import ipc_allreduce as IA


@pytest.mark.parametrize("nbytes", [16, 48, 4096, 1 << 20, (1 << 20) + 16 * 7])
@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
@pytest.mark.parametrize("blocks", [1, 7, 32])
def test_partition_covers_exactly_once(nbytes, nranks, blocks):
    nv = nbytes // 16
    p0 = IA.partition(nbytes, nranks, blocks, 0)
    for r in range(nranks):
        cov = [0] * nv
        for lo, hi in p0["reduce"][r]:
            for i in range(lo, hi):
                cov[i] += 1
        assert cov == [1] * nv
    p1 = IA.partition(nbytes, nranks, blocks, 1)
    seen = [0] * nv
    for r in range(nranks):
        for lo, hi in p1["reduce"][r]:
            for i in range(lo, hi):
                seen[i] += 1
    assert seen == [1] * nv  # reduce-scatter: disjoint slices covering the message
    for r in range(nranks):
        mine = {i for lo, hi in p1["reduce"][r] for i in range(lo, hi)}
        got = {i for lo, hi in p1["gather"][r] for i in range(lo, hi)}
        assert not (mine & got) and (mine | got) == set(range(nv))


def test_choose_mode():
    assert IA.choose_mode(1 << 10, 1 << 20, 32 << 20) == 0
    assert IA.choose_mode(4 << 20, 1 << 20, 32 << 20) == 1
    assert IA.choose_mode(64 << 20, 1 << 20, 32 << 20) is None


def _exchange_worker(rank, world, port, q):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class _Stub:
        group = None
        world = 2

    mine = (bytes([rank]) * 64, bytes([rank + 10]) * 64)
    out = IA.IpcAllReduce._exchange(_Stub(), mine)
    q.put((rank, out))
    dist.destroy_process_group()


def test_handle_exchange_gloo():
    import multiprocessing as mp
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_exchange_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(60)
    expect = [(bytes([r]) * 64, bytes([r + 10]) * 64) for r in range(2)]
    assert res[0] == expect and res[1] == expect


@pytest.mark.gpu
@pytest.mark.parametrize("R", [2, 3, 4])
@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("dtype,n", [(torch.bfloat16, 8), (torch.bfloat16, 1 << 16), (torch.float32, 12345 * 4),
                                     (torch.float16, 4096)])
def test_local_ranks_allreduce(R, mode, dtype, n):
    g = torch.Generator(device="cuda").manual_seed(R * 10 + mode)
    ts = [torch.randn(n, generator=g, device="cuda").to(dtype) for _ in range(R)]
    outs, err = IA.local_allreduce(ts, mode=mode, blocks=8)
    assert err == 0, f"barrier timeout mask {err:#x}"
    ref = ts[0].float()
    for t in ts[1:]:
        ref = ref + t.float()
    ref = ref.to(dtype)
    for o in outs:
        assert torch.equal(o, outs[0])  # bit-identical on every rank
        torch.testing.assert_close(o.float(), ref.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.gpu
def test_ipc_handle_of_uncached_buffer():
    from paddle2_amd.ops import _native as N

    C = N.native()
    p = C.ar_alloc(1 << 20)
    try:
        h = C.ar_get_handle(p)
        assert isinstance(h, bytes) and len(h) == 64
    finally:
        C.ar_free(p)


@pytest.mark.gpu
def test_two_process_ipc_allreduce_bit_exact():
    """Two processes on the one GPU exchange real IPC handles and all-reduce for 40 epochs x 4 sizes (one-shot and
    two-shot): the cross-process flag protocol must give the rank-order sum exactly, every epoch."""
    from tests._dist import run_workers

    res = run_workers("ipc_ar_worker.py", 2, timeout=240, extra_env={"PADDLE2_AMD_DEVICE": "gpu"})
    if not res[0]["ok"] and res[0]["err"].startswith("setup"):
        pytest.skip(res[0]["err"])
    for r in res:
        assert r["ok"], r
        assert r["checked"] == 160


@pytest.mark.gpu
def test_ipc_path_declines_inside_graph_capture(monkeypatch):
    """A captured all_reduce must not take the IPC path (its barrier epoch would be baked into the graph): during
    capture maybe_all_reduce declines even with the path forced on, outside capture it still takes the tensor."""
    calls = []

    class _Fake:
        def supports(self, t):
            return True

        def all_reduce(self, t):
            calls.append(t.numel())
            t.mul_(2)

    monkeypatch.setitem(IA._AUTO, "comm", _Fake())
    monkeypatch.setitem(IA._AUTO, "group", None)
    monkeypatch.setenv("PADDLE2_AMD_IPC_ALLREDUCE", "auto")
    x = torch.ones(256, device="cuda")
    assert IA.maybe_all_reduce(x) and calls == [256]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    taken = []
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            taken.append(IA.maybe_all_reduce(x))
            x.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    assert taken == [False] and calls == [256]
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.all(x == 5)
