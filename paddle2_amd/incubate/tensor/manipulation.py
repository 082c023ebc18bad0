"""Asynchronous device<->host offload (reference: fluid/distributed/collective/async_load.h:35-57
``AsyncLoad`` / ``Task``, python/paddle/incubate/tensor/manipulation.py:103-135 ``create_async_load``,
``async_offload``, ``async_reload``).

MI355X design: one dedicated HIP copy stream per device (SDMA engines move the bytes while the
compute queue keeps running GEMMs).  ``offload`` makes the copy stream wait on an event recorded on
the current (compute) stream, copies into PINNED host memory (DMA-able, so the copy is truly
asynchronous), and records a completion event.  ``Task.cuda_wait()`` makes the compute stream wait
on that event (no host block, like ``UpdateWaitChain``); ``Task.cpu_wait()`` / ``wait()`` blocks the
host (``Synchronize``).  The caching allocator is told the source/destination are used on the copy
stream (``record_stream``) so their memory is not recycled under the DMA.
"""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor


class _Task:
    def __init__(self, event=None, keep=None):
        self._event = event
        self._keep = keep

    def is_completed(self):
        return self._event is None or self._event.query()

    def cpu_wait(self):
        if self._event is not None:
            self._event.synchronize()

    def cuda_wait(self):
        if self._event is not None:
            torch.cuda.current_stream().wait_event(self._event)

    def wait(self):
        self.cpu_wait()

    # reference spellings
    IsCompleted = is_completed
    Synchronize = cpu_wait
    UpdateWaitChain = cuda_wait


class AsyncLoad:
    def __init__(self):
        self._streams = {}

    def _stream(self, device):
        """The device context's H2D copy stream (shared with every other async host->device copy)."""
        s = self._streams.get(device)
        if s is None:
            from ...device.context import get_context

            s = get_context(device).h2d_stream()
            self._streams[device] = s
        return s

    def _copy(self, src, dst_factory):
        if src.device.type != "cuda" and not torch.cuda.is_available():
            dst = dst_factory()
            dst.copy_(src)
            return dst, _Task()
        dev = src.device if src.device.type == "cuda" else torch.device("cuda", torch.cuda.current_device())
        stream = self._stream(dev)
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(dev))
        dst = dst_factory()
        with torch.cuda.stream(stream):
            stream.wait_event(ready)
            dst.copy_(src, non_blocking=True)
            done = torch.cuda.Event()
            done.record(stream)
        for t in (src, dst):
            if t.device.type == "cuda":
                t.record_stream(stream)
        return dst, _Task(done, keep=(src, dst))

    def offload(self, src):
        """Device -> pinned host copy; returns (host tensor, task)."""
        pin = torch.cuda.is_available()
        return self._copy(src, lambda: torch.empty(src.shape, dtype=src.dtype, device="cpu", pin_memory=pin))

    def reload(self, src, device=None):
        """Host -> device copy; returns (device tensor, task)."""
        if not torch.cuda.is_available():
            return self._copy(src, lambda: torch.empty_like(src))
        dev = device or torch.device("cuda", torch.cuda.current_device())
        if not src.is_pinned():
            src = src.pin_memory()
        return self._copy(src, lambda: torch.empty(src.shape, dtype=src.dtype, device=dev))


def create_async_load():
    return AsyncLoad()


def _impl(src_tensor, fn):
    t = src_tensor._t if isinstance(src_tensor, Tensor) else src_tensor
    out, task = fn(t.detach())
    if isinstance(src_tensor, Tensor):
        w = Tensor._wrap(out)
        w.stop_gradient = src_tensor.stop_gradient
        return w, task
    return out, task


def async_offload(src_tensor, async_load):
    """Offload ``src_tensor`` to pinned host memory asynchronously: returns (dest, task)."""
    return _impl(src_tensor, async_load.offload)


def async_reload(src_tensor, async_load):
    """Reload a host tensor onto the current device asynchronously: returns (dest, task)."""
    return _impl(src_tensor, async_load.reload)
