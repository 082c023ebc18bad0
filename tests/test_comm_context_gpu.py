"""NCCLCommContext on one MI355X: an RCCL communicator created from a bare TCPStore by key (no default group);
every collective runs through RCCL kernels on the device."""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_nccl_comm_context_one_rank():
    import torch.distributed as dist

    from paddle2_amd.distributed.comm_context import CommContextManager

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    store = dist.TCPStore("127.0.0.1", port, 1, True)
    torch.cuda.set_device(0)
    ctx = CommContextManager.create_nccl_comm_context(store, "gpu_ring_0", 0, 1)
    try:
        t = torch.arange(8.0, device="cuda")
        ctx.all_reduce(t)
        ctx.all_reduce(t, op=ctx.red_op_create_pre_mul_sum(2.0))
        assert t.tolist() == [2.0 * i for i in range(8)]
        out = torch.empty(8, device="cuda")
        ctx.all_gather(out, t)
        assert torch.equal(out, t)
        rs = torch.empty(8, device="cuda")
        ctx.reduce_scatter(rs, t, op="avg")
        assert torch.equal(rs, t)
        ctx.broadcast(t, root=0)
        a2a = torch.empty(8, device="cuda")
        ctx.all_to_all(a2a, t)
        assert torch.equal(a2a, t)
        ctx.barrier()
        torch.cuda.synchronize()
    finally:
        CommContextManager.get_instance().release("gpu_ring_0")
