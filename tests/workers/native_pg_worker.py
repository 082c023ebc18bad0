"""1-rank worker for the framework's own RCCL process group (backend "pdrccl", csrc/comm/rccl_group.cpp)."""
import faulthandler
import json
import os
import sys

faulthandler.enable()

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from paddle2_amd.distributed import rccl_pg  # noqa: E402

torch.cuda.set_device(0)
rccl_pg.register()
dist.init_process_group(rccl_pg.BACKEND, rank=0, world_size=1,
                        init_method=f"tcp://127.0.0.1:{os.environ['MASTER_PORT']}")
pg = dist.group.WORLD
res = {"backend": type(pg).__name__, "name": pg.getBackendName() if hasattr(pg, "getBackendName") else ""}
dev = torch.device("cuda", 0)

x = torch.arange(1, 9, dtype=torch.float32, device=dev)
dist.all_reduce(x)
res["sum"] = x.tolist()
print("ok sum", flush=True)
dist.all_reduce(x, op=dist.ReduceOp.AVG)
res["avg"] = x.tolist()
print("ok avg", flush=True)
dist.all_reduce(x, op=dist.ReduceOp.MAX)
res["max"] = x.tolist()
print("ok max", flush=True)
w = pg.all_reduce_native(x, premul=0.5)
w.wait()
res["premul"] = x.tolist()
print("ok premul", flush=True)
xb = torch.arange(1, 9, dtype=torch.bfloat16, device=dev)
pg.all_reduce_native(xb, premul=2.0).wait()
res["premul_bf16"] = xb.float().tolist()
print("ok premul_bf16", flush=True)

# non-contiguous input: result copied back into the strided view
m = torch.arange(12, dtype=torch.float32, device=dev).reshape(3, 4)
v = m.t()
dist.all_reduce(v, op=dist.ReduceOp.SUM)
res["noncontig"] = m.tolist()
print("ok noncontig", flush=True)

# async + stream ordering: a long GEMM writes the tensor on the current stream, the collective must see it
a = torch.randn(4096, 4096, device=dev)
y = torch.empty(4096, 4096, device=dev)
torch.matmul(a, a, out=y)
ref = y.clone()
work = dist.all_reduce(y, async_op=True)
work.wait()
res["async_exact"] = bool(torch.equal(y, ref))
print("ok async_exact", flush=True)

b = torch.tensor([3.0, 4.0], device=dev)
dist.broadcast(b, src=0)
res["bcast"] = b.tolist()
print("ok bcast", flush=True)
r = torch.tensor([5.0, 6.0], device=dev)
dist.reduce(r, dst=0)
res["reduce"] = r.tolist()
print("ok reduce", flush=True)

inp = torch.tensor([1.0, 2.0, 3.0], device=dev)
out = torch.empty(3, device=dev)
dist.all_gather_into_tensor(out, inp)
res["ag"] = out.tolist()
print("ok ag", flush=True)
lst = [torch.empty(3, device=dev)]
dist.all_gather(lst, inp)
res["ag_list"] = lst[0].tolist()
print("ok ag_list", flush=True)
rs_out = torch.empty(4, device=dev)
dist.reduce_scatter_tensor(rs_out, torch.tensor([1.0, 2.0, 3.0, 4.0], device=dev))
res["rs"] = rs_out.tolist()
print("ok rs", flush=True)
a2a = torch.empty(4, device=dev)
dist.all_to_all_single(a2a, torch.tensor([9.0, 8.0, 7.0, 6.0], device=dev))
res["a2a"] = a2a.tolist()
print("ok a2a", flush=True)
a2av = torch.empty(3, device=dev)
dist.all_to_all_single(a2av, torch.tensor([1.0, 2.0, 3.0], device=dev), [3], [3])
res["a2av"] = a2av.tolist()
print("ok a2av", flush=True)
ol = [torch.empty(2, device=dev)]
dist.all_to_all(ol, [torch.tensor([4.0, 5.0], device=dev)])
res["a2a_list"] = ol[0].tolist()
print("ok a2a_list", flush=True)

# coalesced all-reduce (one RCCL group, one task)
ts = [torch.full((5,), 2.0, device=dev), torch.full((7,), 3.0, device=dev, dtype=torch.bfloat16)]
pg.allreduce_coalesced(ts, dist.AllreduceCoalescedOptions()).wait()
res["coalesced"] = [ts[0].sum().item(), ts[1].float().sum().item()]
print("ok coalesced", flush=True)

# send / recv to self in one coalesced group (a same-stream send-then-recv pair needs the group)
src = torch.arange(6, dtype=torch.float32, device=dev)
dst = torch.zeros(6, device=dev)
ws = rccl_pg.batch_isend_irecv([dist.P2POp(dist.isend, src, 0), dist.P2POp(dist.irecv, dst, 0)])
for w in ws:
    w.wait()
res["p2p_self"] = dst.tolist()
print("ok p2p_self", flush=True)

dist.barrier()
torch.cuda.synchronize()
res["num_comms"] = pg._g.num_comms()
print("ok num_comms", flush=True)
# the start-up check init_parallel_env runs on a default ProcessGroupRCCL (1 rank: p2p to self)
ok, verdicts = rccl_pg.canary(dist.distributed_c10d._get_default_store(), 0, 1)
res["canary"] = [ok, verdicts]
print("ok canary", verdicts, flush=True)
dist.destroy_process_group()
with open(os.environ["PD_TEST_OUT"], "w") as f:
    json.dump(res, f)
