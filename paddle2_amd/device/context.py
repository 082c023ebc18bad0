"""Per-device execution context (reference: paddle/phi/backends/gpu/gpu_context.h GPUContext,
paddle/phi/core/platform/device_context.h DeviceContextPool).

``GPUContext`` owns, for one MI355X: the compute stream (torch's current stream on that device), a
high-priority communication stream, H2D / D2H copy streams, a side stream for HIP-graph warm-up, a recycled
event pool and the device facts the kernels tile for (CU count, XCDs, LDS per CU, wavefront size, HBM
capacity).  Framework pieces that overlap work — AsyncLoad, the IPC all-reduce, graph capture in the static
executor and the serving decode loop — take their streams from here instead of creating private ones, so
one process has one comm stream and one pair of copy streams per device.  ``DeviceContextPool`` maps places
to contexts (created lazily, one per device).
"""
from __future__ import annotations

import threading

import torch

_HW_DEFAULTS = {"num_cus": 256, "num_xcds": 8, "lds_bytes_per_cu": 160 * 1024, "wavefront_size": 64}


class GPUContext:
    def __init__(self, device=0):
        self.device = int(device)
        self._lock = threading.Lock()
        self._streams = {}
        self._events = []

    # ---------------------------------------------------------------- streams
    def _stream(self, name, priority=0):
        with self._lock:
            s = self._streams.get(name)
            if s is None:
                s = torch.cuda.Stream(device=self.device, priority=priority)
                self._streams[name] = s
            return s

    def stream(self):
        """The compute stream: torch's current stream on this device (kernels launch here)."""
        return torch.cuda.current_stream(self.device)

    def comm_stream(self):
        """High-priority stream for collectives / peer copies that overlap compute."""
        return self._stream("comm", priority=-1)

    def h2d_stream(self):
        return self._stream("h2d")

    def d2h_stream(self):
        return self._stream("d2h")

    def capture_stream(self):
        """Side stream for HIP-graph warm-up and capture."""
        return self._stream("capture")

    # ---------------------------------------------------------------- events
    def get_event(self):
        with self._lock:
            if self._events:
                return self._events.pop()
        return torch.cuda.Event()

    def recycle_event(self, e):
        with self._lock:
            self._events.append(e)

    def record(self, stream=None):
        """Record an event on ``stream`` (default: compute) and return it (caller recycles it)."""
        e = self.get_event()
        e.record(stream if stream is not None else self.stream())
        return e

    def wait(self, waiter, producer):
        """Make stream ``waiter`` wait for all work queued so far on ``producer`` (device-side)."""
        e = self.record(producer)
        waiter.wait_event(e)
        self.recycle_event(e)

    # ---------------------------------------------------------------- handles / facts
    def blas_handle(self):
        with torch.cuda.device(self.device):
            return torch.cuda.current_blas_handle()

    def properties(self):
        p = torch.cuda.get_device_properties(self.device)
        facts = dict(_HW_DEFAULTS)
        facts.update(name=p.name, num_cus=p.multi_processor_count, total_memory=p.total_memory,
                     arch=getattr(p, "gcnArchName", ""), l2_bytes=getattr(p, "L2_cache_size", 0))
        ws = getattr(p, "warp_size", None)
        if ws:
            facts["wavefront_size"] = ws
        return facts

    def synchronize(self):
        torch.cuda.synchronize(self.device)

    def __repr__(self):
        return f"GPUContext(device={self.device}, streams={sorted(self._streams)})"


class DeviceContextPool:
    _inst = None
    _lock = threading.Lock()

    def __init__(self):
        self._ctx = {}

    @classmethod
    def instance(cls):
        with cls._lock:
            if cls._inst is None:
                cls._inst = cls()
            return cls._inst

    def get(self, place=None):
        dev = _device_index(place)
        with self._lock:
            c = self._ctx.get(dev)
            if c is None:
                c = GPUContext(dev)
                self._ctx[dev] = c
            return c

    def size(self):
        return len(self._ctx)


def _device_index(place):
    if place is None:
        return torch.cuda.current_device() if torch.cuda.is_available() else 0
    if isinstance(place, int):
        return place
    if isinstance(place, torch.device):
        return place.index if place.index is not None else torch.cuda.current_device()
    if isinstance(place, str):
        return int(place.split(":")[1]) if ":" in place else 0
    for attr in ("get_device_id", "device_id"):
        v = getattr(place, attr, None)
        if v is not None:
            return v() if callable(v) else int(v)
    return 0


def get_context(place=None):
    """The GPUContext of ``place`` (default: current device)."""
    return DeviceContextPool.instance().get(place)
