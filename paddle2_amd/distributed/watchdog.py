"""Collective hang watchdog (reference: phi/core/distributed/comm_task_manager.cc, nccl_comm_task.cc).

With ``FLAGS_enable_async_trace`` every collective records a HIP event on the current stream after
its launch and registers (description, deadline, event) with the NATIVE watchdog
(csrc/runtime/watchdog.cpp): a C++ thread polls ``hipEventQuery`` on the in-flight events and
reports — or with ``FLAGS_comm_abort_on_timeout`` aborts the process — for any collective
started but not finished after ``FLAGS_comm_timeout_s`` (the reference's "started-not-finished"
classification), with op, group ranks, sequence number, shape and dtype.  CPU (gloo) collectives
are host-synchronous; they register without an event and deregister on return.
"""
from __future__ import annotations

import contextlib
import itertools
import logging
import threading

import torch

from ..framework import flags

_log = logging.getLogger("paddle2_amd.distributed.watchdog")
_events = {}          # native task id -> torch Event kept alive until the native thread reports it done
_lock = threading.Lock()
_seq = itertools.count()
_started = False


def _rt():
    from .. import _rt

    return _rt.get()


def enabled():
    return bool(flags.flag("FLAGS_enable_async_trace", False))


def _timeout():
    return float(flags.flag("FLAGS_comm_timeout_s", 1800))


def _prune():
    done = _rt().watchdog_take_finished()
    if done:
        with _lock:
            for i in done:
                _events.pop(i, None)


@contextlib.contextmanager
def track(op, group, tensor):
    if not enabled():
        yield
        return
    maybe_start()
    t = tensor._t if hasattr(tensor, "_t") else tensor
    desc = (f"seq={next(_seq)} op={op} ranks={getattr(group, 'ranks', None)} shape={tuple(t.shape)} "
            f"dtype={t.dtype}")
    rt = _rt()
    if t.device.type != "cuda":
        tid = rt.watchdog_begin(desc, _timeout(), 0)
        try:
            yield
        finally:
            rt.watchdog_end(tid)
        return
    try:
        yield
    finally:
        ev = torch.cuda.Event()
        ev.record()
        tid = rt.watchdog_begin(desc, _timeout(), int(ev.cuda_event))
        with _lock:
            _events[tid] = ev
        _prune()


def check_once(timeout_s=None):
    """Descriptions of every collective the native watchdog has reported as timed out."""
    _prune()
    return list(_rt().watchdog_timed_out())


def maybe_start(interval=1.0):
    global _started
    if _started or not enabled():
        return
    _rt().watchdog_start(float(interval), bool(flags.flag("FLAGS_comm_abort_on_timeout", False)))
    _started = True


def pending():
    _prune()
    return int(_rt().watchdog_inflight())
