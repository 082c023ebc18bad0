"""Rank worker: the framework's own DistTensor (auto_parallel/dist_tensor.py) — aten-level SPMD dispatch on plain torch
ops (forward and autograd backward) against the same computation on full tensors, on a 1-D mesh (2 ranks) or a
2x2 mesh (4 ranks)."""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402

import paddle2_amd.distributed as dist  # noqa: E402
from paddle2_amd.distributed.auto_parallel import dist_tensor as DT  # noqa: E402
from paddle2_amd.distributed.auto_parallel.placement import Partial, Replicate, Shard  # noqa: E402
from paddle2_amd.distributed.auto_parallel.reshard import COMM_LOG  # noqa: E402
from _dist import write_result  # noqa: E402

dist.init_parallel_env()
world = torch.distributed.get_world_size()
two_d = world == 4
pm = dist.ProcessMesh([[0, 1], [2, 3]] if two_d else [0, 1], dim_names=["dp", "mp"] if two_d else ["mp"])
mesh = pm._device_mesh()
R, S, P = Replicate, Shard, Partial
out = {"is_own_type": True, "checks": {}}


def full(t):
    return t.full_tensor() if isinstance(t, DT.DistTensor) else t


def check(name, got, ref, tol=1e-5):
    g = full(got).detach()
    out["checks"][name] = float((g - ref.detach()).abs().max()) if g.shape == ref.shape else f"shape {list(g.shape)}"
    return g


def dist_(t, *pl):
    pl = list(pl) if two_d else list(pl[-1:])
    return DT.distribute_tensor(t, mesh, pl)


gen = torch.Generator().manual_seed(0)
A = torch.randn(8, 6, generator=gen)
B = torch.randn(6, 4, generator=gen)
V = torch.randn(4, generator=gen)

# ---- matmul rules: column-parallel, row-parallel (partial output), data-parallel rows
a_dp = dist_(A, S(0), R())
b_col = dist_(B, R(), S(1))
c = torch.mm(a_dp, b_col)
out["col_out"] = [str(p) for p in c.placements]
check("mm_col", c, A @ B)
a_row = dist_(A, R(), S(1))
b_row = dist_(B, R(), S(0))
c2 = torch.mm(a_row, b_row)
out["row_out"] = [str(p) for p in c2.placements]
check("mm_row_partial", c2, A @ B)
# partial + bias: the bias is added once
check("mm_row_bias", c2 + V, A @ B + V)
# nonlinear on a partial value: reduced first
check("relu_partial", torch.relu(c2), torch.relu(A @ B))

# ---- elementwise broadcasting, reductions, softmax, views, transpose
x = dist_(A, S(0), S(1))
check("ew", x * 2 + torch.sin(x) - x / 3, A * 2 + torch.sin(A) - A / 3)
check("ew_bcast", x + dist_(torch.ones(6) * 0.5, R(), R()), A + 0.5)
check("sum_all", x.sum(), A.sum())
check("sum_dim0", x.sum(0), A.sum(0))
check("mean_dim1", x.mean(1, keepdim=True), A.mean(1, keepdim=True))
check("softmax1", torch.softmax(x, 1), torch.softmax(A, 1))
check("view", x.view(4, 12), A.view(4, 12))
check("view_merge", dist_(A.view(2, 4, 6), S(0), R()).reshape(8, 6), A)
check("t", x.t(), A.t())
check("layer_norm", torch.nn.functional.layer_norm(x, (6,)), torch.nn.functional.layer_norm(A, (6,)))
ids = torch.tensor([[1, 3], [0, 2]])
E = torch.randn(5, 6, generator=gen)
check("embedding_col", torch.nn.functional.embedding(ids, dist_(E, R(), S(1))), torch.nn.functional.embedding(ids, E))

# ---- shape ops: slicing / selecting / splitting along a replicated axis keeps the other axis' shards
xs_ = dist_(A, S(0), S(1))
check("slice", xs_[:, 1:5], A[:, 1:5])
check("select", xs_[:, 2], A[:, 2])
check("split", torch.cat(torch.split(xs_, 2, dim=1), 0), torch.cat(torch.split(A, 2, dim=1), 0))
check("cat", torch.cat([xs_, xs_ * 2], 1), torch.cat([A, A * 2], 1))
check("stack", torch.stack([xs_, xs_], 0), torch.stack([A, A], 0))

# ---- autograd through a tensor-parallel MLP (col -> gelu -> row), data-parallel input rows
W1 = torch.randn(6, 8, generator=gen) * 0.3
W2 = torch.randn(8, 6, generator=gen) * 0.3
b1 = torch.randn(8, generator=gen) * 0.1
X = torch.randn(8, 6, generator=gen)
w1 = dist_(W1, R(), S(1)).requires_grad_()
w2 = dist_(W2, R(), S(0)).requires_grad_()
bb = dist_(b1, R(), S(0)).requires_grad_()
xd = dist_(X, S(0), R())
loss = (torch.nn.functional.gelu(xd @ w1 + bb) @ w2).pow(2).mean()
loss.backward()
W1r, W2r, b1r = (t.clone().requires_grad_() for t in (W1, W2, b1))
lr = (torch.nn.functional.gelu(X @ W1r + b1r) @ W2r).pow(2).mean()
lr.backward()
check("mlp_loss", loss, lr)
check("mlp_dw1", w1.grad, W1r.grad)
check("mlp_dw2", w2.grad, W2r.grad)
check("mlp_db1", bb.grad, b1r.grad)
out["dw1_placements"] = [str(p) for p in w1.grad.placements]

# ---- an optimizer-style in-place update with a partial gradient (all-reduced into the replicated parameter)
p = dist_(W2.clone(), R(), R())
g_part = DT.DistTensor(torch.ones(8, 6) * (1.0 if mesh.get_local_rank(mesh.ndim - 1) == 0 else 2.0), mesh,
                       ((R(),) if two_d else ()) + (P(),), (8, 6))
p.sub_(g_part * 0.5)
check("inplace_partial", p, W2 - 1.5)
out["comm"] = sorted({k for k, _ in COMM_LOG})
out["fallbacks"] = sorted({t[0] for t in DT.TRACE if len(t) == 2})
write_result(out)
