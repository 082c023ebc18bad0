"""Collective hang watchdog (reference: phi/core/distributed/comm_task_manager.cc, nccl_comm_task.cc).

With ``FLAGS_enable_async_trace`` every collective records a start event on the current HIP stream
and an end event after launch; a background thread polls the events every 10 s and reports
tasks that were started but not finished after ``FLAGS_comm_timeout_s`` (with op, group ranks,
sequence number, shape/dtype) — the reference's "started-not-finished" classification.
"""
from __future__ import annotations

import contextlib
import itertools
import logging
import os
import threading
import time

import torch

from ..framework import flags

_log = logging.getLogger("paddle2_amd.distributed.watchdog")
_tasks = {}
_lock = threading.Lock()
_seq = itertools.count()
_thread = None
_stop = threading.Event()


class CommTask:
    __slots__ = ("seq", "op", "ranks", "shape", "dtype", "t0", "start_ev", "end_ev", "reported")

    def __init__(self, seq, op, ranks, shape, dtype):
        self.seq, self.op, self.ranks, self.shape, self.dtype = seq, op, ranks, shape, dtype
        self.t0 = time.time()
        self.start_ev = self.end_ev = None
        self.reported = False

    def finished(self):
        if self.end_ev is None:
            return True
        return self.end_ev.query()


def enabled():
    return bool(flags.flag("FLAGS_enable_async_trace", False))


@contextlib.contextmanager
def track(op, group, tensor):
    if not enabled():
        yield
        return
    t = tensor._t if hasattr(tensor, "_t") else tensor
    ranks = getattr(group, "ranks", None)
    task = CommTask(next(_seq), op, ranks, tuple(t.shape), str(t.dtype))
    if t.device.type == "cuda":
        task.start_ev = torch.cuda.Event()
        task.start_ev.record()
    try:
        yield
    finally:
        if t.device.type == "cuda":
            task.end_ev = torch.cuda.Event()
            task.end_ev.record()
        with _lock:
            _tasks[task.seq] = task


def check_once(timeout_s=None):
    """Return descriptions of tasks started but not finished past the timeout; drop finished ones."""
    timeout_s = timeout_s if timeout_s is not None else float(flags.flag("FLAGS_comm_timeout_s", 1800))
    now = time.time()
    hung = []
    with _lock:
        for seq in list(_tasks):
            tk = _tasks[seq]
            if tk.finished():
                del _tasks[seq]
            elif now - tk.t0 > timeout_s and not tk.reported:
                tk.reported = True
                hung.append(f"[watchdog] collective seq={tk.seq} op={tk.op} ranks={tk.ranks} shape={tk.shape} "
                            f"dtype={tk.dtype} started {now - tk.t0:.1f}s ago and has not finished")
    for h in hung:
        _log.error(h)
    return hung


def _loop(interval):
    while not _stop.wait(interval):
        try:
            check_once()
        except Exception:  # pragma: no cover
            pass


def maybe_start(interval=10.0):
    global _thread
    if not enabled() or _thread is not None:
        return
    _thread = threading.Thread(target=_loop, args=(interval,), daemon=True, name="pd-comm-watchdog")
    _thread.start()


def pending():
    with _lock:
        return len(_tasks)
