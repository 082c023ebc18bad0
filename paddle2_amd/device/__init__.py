"""paddle.device (reference: python/paddle/device/__init__.py, device/cuda/{__init__,streams,graphs}.py).

Streams/events are HIP streams/events (torch.cuda on ROCm); ``CUDAGraph`` captures with
hipGraph (reference: phi/backends/gpu/rocm/hip_graph.cc).
"""
from __future__ import annotations

import contextlib

import torch

from . import allocator, context  # noqa: F401
from .context import DeviceContextPool, GPUContext, get_context  # noqa: F401
from ..framework.place import (CPUPlace, CUDAPlace, get_device, is_compiled_with_cinn,  # noqa: F401
                               is_compiled_with_cuda, is_compiled_with_custom_device, is_compiled_with_distribute,
                               is_compiled_with_rocm, is_compiled_with_xpu, set_device)


def get_all_device_type():
    return ["cpu", "gpu"] if torch.cuda.is_available() else ["cpu"]


def get_all_custom_device_type():
    return []


def get_available_device():
    if torch.cuda.is_available():
        return [f"gpu:{i}" for i in range(torch.cuda.device_count())]
    return ["cpu"]


def get_available_custom_device():
    return []


def device_count(device_type=None):
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


def synchronize(device=None):
    if torch.cuda.is_available():
        torch.cuda.synchronize()


class Stream:
    """A HIP stream (paddle.device.Stream)."""

    def __init__(self, device=None, priority=2, stream_base=None):
        if stream_base is not None:
            self._s = stream_base
        else:
            # paddle priority: 1 = high, 2 = normal
            self._s = torch.cuda.Stream(priority=-1 if priority == 1 else 0)

    @property
    def cuda_stream(self):
        return self._s.cuda_stream

    def wait_event(self, event):
        self._s.wait_event(event._e)

    def wait_stream(self, stream):
        self._s.wait_stream(stream._s)

    def record_event(self, event=None):
        event = event or Event()
        event.record(self)
        return event

    def query(self):
        return self._s.query()

    def synchronize(self):
        self._s.synchronize()


class Event:
    def __init__(self, device=None, enable_timing=False, blocking=False, interprocess=False):
        self._e = torch.cuda.Event(enable_timing=enable_timing, blocking=blocking, interprocess=interprocess)

    def record(self, stream=None):
        self._e.record(stream._s if stream is not None else None)

    def query(self):
        return self._e.query()

    def synchronize(self):
        self._e.synchronize()

    def elapsed_time(self, end_event):
        return self._e.elapsed_time(end_event._e)


def current_stream(device=None):
    return Stream(stream_base=torch.cuda.current_stream())


def set_stream(stream):
    prev = current_stream()
    torch.cuda.set_stream(stream._s)
    return prev


@contextlib.contextmanager
def stream_guard(stream):
    if stream is None:
        yield
        return
    with torch.cuda.stream(stream._s):
        yield


def _dev(device):
    from .context import _device_index

    return _device_index(device)


class cuda:
    """paddle.device.cuda namespace."""

    Stream = Stream
    Event = Event
    current_stream = staticmethod(current_stream)
    stream_guard = staticmethod(stream_guard)
    synchronize = staticmethod(synchronize)

    @staticmethod
    def device_count():
        return device_count()

    @staticmethod
    def empty_cache():
        if torch.cuda.is_available():
            if allocator.is_active():
                allocator.empty_cache(_dev(None))
            else:
                torch.cuda.empty_cache()

    @staticmethod
    def max_memory_allocated(device=None):
        if allocator.is_active():
            return allocator.stats(_dev(device))["peak_allocated"]
        return torch.cuda.max_memory_allocated(device) if torch.cuda.is_available() else 0

    @staticmethod
    def max_memory_reserved(device=None):
        if allocator.is_active():
            return allocator.stats(_dev(device))["peak_reserved"]
        return torch.cuda.max_memory_reserved(device) if torch.cuda.is_available() else 0

    @staticmethod
    def memory_allocated(device=None):
        if allocator.is_active():
            return allocator.stats(_dev(device))["allocated"]
        return torch.cuda.memory_allocated(device) if torch.cuda.is_available() else 0

    @staticmethod
    def memory_reserved(device=None):
        if allocator.is_active():
            return allocator.stats(_dev(device))["reserved"]
        return torch.cuda.memory_reserved(device) if torch.cuda.is_available() else 0

    @staticmethod
    def reset_max_memory_allocated(device=None):
        if allocator.is_active():
            allocator.reset_peak(_dev(device))
        elif torch.cuda.is_available():
            torch.cuda.reset_peak_memory_stats(device)

    @staticmethod
    def get_device_properties(device=None):
        return torch.cuda.get_device_properties(device or 0)

    @staticmethod
    def get_device_name(device=None):
        return torch.cuda.get_device_name(device or 0)

    @staticmethod
    def get_device_capability(device=None):
        return torch.cuda.get_device_capability(device or 0)


class CUDAGraph:
    """hipGraph capture/replay (reference: python/paddle/device/cuda/graphs.py:43)."""

    def __init__(self, place=None, mode="thread_local", pool_id=None):
        self._g = torch.cuda.CUDAGraph()
        self._pool = pool_id
        self._stream = torch.cuda.Stream()
        self._ctx = None

    def capture_begin(self):
        from ..ops import fp8

        fp8.before_capture()   # eager fp8 scale updates land before, not inside, the capture
        self._stream.wait_stream(torch.cuda.current_stream())
        self._ctx = torch.cuda.graph(self._g, pool=self._pool, stream=self._stream)
        self._ctx.__enter__()

    def capture_end(self):
        self._ctx.__exit__(None, None, None)
        self._ctx = None

    def replay(self):
        self._g.replay()

    def reset(self):
        self._g.reset()

    def print_to_dot_files(self, dirname, flags=None):
        self._g.debug_dump(str(dirname))


def is_cuda_graph_supported():
    return torch.cuda.is_available()
