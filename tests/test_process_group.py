"""group.process_group exposes the reference ProcessGroup bindings (distributed_py.cc): every collective with
its *_on_calc_stream twin, partial all-gather / send / recv, tasks; 3 gloo ranks vs closed-form results."""
from _dist import run_workers


def test_process_group_methods_three_ranks():
    w = 3
    res = run_workers("process_group_worker.py", w)
    total = sum(range(1, w + 1))
    for r, x in enumerate(res):
        assert x["rank"] == r and x["size"] == w and x["name"] == "GLOO"
        assert x["all_reduce"] == [float(total)] * 4
        assert x["avg"] == [total / w] * 2 and x["task"][0]
        assert x["bcast"] == [float(w - 1)] * 3
        assert x["gather_list"] == [float(i) for i in range(w)]
        assert x["gather_tensor"] == [v for i in range(w) for v in (float(i), i + 0.5)]
        assert x["gather_partial"] == [float(10 * i + i) for i in range(w)]
        assert x["reduce_scatter"] == [float(w * (2 * r)), float(w * (2 * r + 1))]
        assert x["all_to_all"] == [float(100 * i + r) for i in range(w)]
        assert x["scatter"] == float(7 * r)
    assert res[0]["gather"] == [float(i * i) for i in range(w)] and res[1]["gather"] == []
    assert res[0]["reduce_root"] == float(total)
    assert res[1]["recv"] == [1.0, 2.0, 3.0, 4.0]
    assert res[1]["recv_partial"] == [0.0, 0.0, 7.0, 8.0]


import pytest  # noqa: E402


@pytest.mark.parametrize("flavour", ["ompi", "pmi"])
def test_mpi_launch_env_and_process_group_mpi(flavour):
    """mpirun-launched ranks (reference ProcessGroupMPI, process_group_mpi.cc): rank / size / local rank from the
    MPI launcher's variables, backend "mpi" -> collectives on gloo; ProcessGroupMPI.create() without arguments."""
    w = 2
    res = run_workers("mpi_pg_worker.py", w, args=(flavour,))
    for r, x in enumerate(res):
        assert (x["env_rank"], x["env_world"], x["dev"]) == (r, w, r)
        assert x["all_reduce"] == [3.0] * 3
        assert (x["pg_name"], x["pg_rank"], x["pg_size"], x["pg_sum"]) == ("MPI", r, w, 1.0)
