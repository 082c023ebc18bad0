"""Rank of the multi-process IPC all-reduce test: both ranks run on cuda:0 (the only GPU of the box), map each
other's uncached buffers through real hipIpc handles exchanged over gloo, and all-reduce deterministic inputs
for many epochs, one-shot and two-shot; every result must equal the rank-order sum bit for bit."""
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
from paddle2_amd.distributed import ipc_allreduce as IA  # noqa: E402
from tests._dist import write_result  # noqa: E402

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
dist.init_process_group("gloo", rank=rank, world_size=world)
torch.cuda.set_device(0)
res = {"rank": rank, "ok": True, "checked": 0, "err": ""}
try:
    comm = IA.IpcAllReduce(None, capacity=8 << 20, oneshot_max=64 << 10, blocks=16, timeout_ms=20000)
except Exception as e:  # no same-device IPC on this driver: report, the test skips
    res.update(ok=False, err=f"setup: {type(e).__name__}: {e}")
    write_result(res)
    dist.destroy_process_group()
    sys.exit(0)


def inp(r, ep, n, dtype):
    g = torch.Generator().manual_seed(1000 * ep + r)
    return torch.randn(n, generator=g).to(dtype)


bad = []
for ep in range(int(os.environ.get("PD_IPC_EPOCHS", "40"))):
    for dtype, n in ((torch.float32, 1024), (torch.bfloat16, 40000), (torch.float32, 300000), (torch.bfloat16, 2 << 20)):
        t = inp(rank, ep, n, dtype).cuda()
        comm.all_reduce(t)
        ref = inp(0, ep, n, dtype).float()
        for r in range(1, world):
            ref = ref + inp(r, ep, n, dtype).float()
        ref = ref.to(dtype)
        got = t.cpu()
        res["checked"] += 1
        if not torch.equal(got, ref):
            bad.append((ep, str(dtype), n, float((got.float() - ref.float()).abs().max())))
comm.raise_on_timeout()
torch.cuda.synchronize()
res["ok"] = not bad
res["bad"] = bad[:10]
comm.close()
write_result(res)
dist.barrier()
dist.destroy_process_group()
