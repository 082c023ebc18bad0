"""Rank worker: an mpirun-style launch -- only the MPI launcher's variables (Open MPI or PMI flavour) carry rank /
size -- with backend "mpi" (ProcessGroupMPI semantics over gloo)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

flavour = sys.argv[1]
r, w = os.environ["RANK"], os.environ["WORLD_SIZE"]
for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "PADDLE_TRAINER_ID", "PADDLE_TRAINERS_NUM"):
    os.environ.pop(k)
if flavour == "ompi":
    os.environ.update(OMPI_COMM_WORLD_RANK=r, OMPI_COMM_WORLD_SIZE=w, OMPI_COMM_WORLD_LOCAL_RANK=r)
else:
    os.environ.update(PMI_RANK=r, PMI_SIZE=w, MPI_LOCALRANKID=r)
os.environ["PADDLE_DISTRI_BACKEND"] = "mpi"

import paddle2_amd as paddle  # noqa: E402
import paddle2_amd.distributed as dist  # noqa: E402
from _dist import write_result  # noqa: E402

res = {"env_rank": dist.get_rank(), "env_world": dist.get_world_size(), "dev": dist.ParallelEnv().device_id}
dist.init_parallel_env()
x = paddle.to_tensor([float(dist.get_rank() + 1)] * 3)
dist.all_reduce(x)
res["all_reduce"] = x.numpy().tolist()
res["backend"] = dist.get_backend()
# a standalone ProcessGroupMPI (core.ProcessGroupMPI.create) on its own store / port
os.environ["MASTER_PORT"] = str(int(os.environ["MASTER_PORT"]) + 1)
pg = dist.ProcessGroupMPI.create()
y = paddle.to_tensor([float(pg.rank())])
pg.all_reduce(y).wait()
res.update(pg_name=pg.name(), pg_rank=pg.rank(), pg_size=pg.size(), pg_sum=float(y.numpy()[0]))
write_result(res)
