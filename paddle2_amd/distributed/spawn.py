"""paddle.distributed.spawn (reference: python/paddle/distributed/spawn.py — start ``nprocs``
processes with the multiprocessing ``spawn`` context, each with the collective env contract,
run ``func(*args)`` and join, re-raising a child's exception in the parent)."""
from __future__ import annotations

import multiprocessing as mp
import os
import socket
import traceback


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(func, args, rank, nprocs, port, err_q, backend, options):
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(nprocs), "LOCAL_RANK": str(rank),
                       "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "PADDLE_TRAINER_ID": str(rank),
                       "PADDLE_TRAINERS_NUM": str(nprocs), "PADDLE_LOCAL_RANK": str(rank),
                       "FLAGS_selected_gpus": str(rank)})
    if backend:
        os.environ["PADDLE_DISTRI_BACKEND"] = backend
    for k, v in options.get("env", {}).items():
        os.environ[k] = str(v)
    try:
        func(*args)
    except Exception:  # pragma: no cover - re-raised in the parent
        err_q.put((rank, traceback.format_exc()))
        raise SystemExit(1)


class MultiprocessContext:
    def __init__(self, procs, err_q):
        self.processes = procs
        self._err = err_q

    def join(self, timeout=None):
        for p in self.processes:
            p.join(timeout)
        if not self._err.empty():
            rank, tb = self._err.get()
            for p in self.processes:
                if p.is_alive():
                    p.terminate()
            raise RuntimeError(f"process {rank} terminated with an exception:\n{tb}")
        for p in self.processes:
            if p.exitcode not in (0, None):
                raise RuntimeError(f"process {p.pid} exited with code {p.exitcode}")
        return True


def spawn(func, args=(), nprocs=-1, join=True, daemon=False, **options):
    if nprocs == -1:
        try:
            import torch

            nprocs = max(1, torch.cuda.device_count())
        except Exception:  # pragma: no cover
            nprocs = 1
    ctx = mp.get_context("spawn")
    err_q = ctx.SimpleQueue()
    port = _free_port()
    backend = options.get("backend")
    procs = []
    for r in range(nprocs):
        p = ctx.Process(target=_entry, args=(func, args, r, nprocs, port, err_q, backend, options), daemon=daemon)
        p.start()
        procs.append(p)
    c = MultiprocessContext(procs, err_q)
    if join:
        c.join()
    return c
