"""paddle.profiler (reference: python/paddle/profiler/profiler.py, timer.py Benchmark).

Host events come from ``RecordEvent`` scopes; device activity is collected through torch's
profiler, which on ROCm is backed by roctracer / rocprofiler-sdk — the reference's ROCm build has
host-only traces, here HIP kernels (including ours) appear in the chrome trace.
"""
from __future__ import annotations

import contextlib
import enum
import json
import os
import time

import torch


class ProfilerTarget(enum.Enum):
    CPU = 0
    GPU = 1
    CUSTOM_DEVICE = 3


class ProfilerState(enum.Enum):
    CLOSED = 0
    READY = 1
    RECORD = 2
    RECORD_AND_RETURN = 3


class SortedKeys(enum.Enum):
    CPUTotal = 0
    CPUAvg = 1
    CPUMax = 2
    CPUMin = 3
    GPUTotal = 4
    GPUAvg = 5
    GPUMax = 6
    GPUMin = 7


def make_scheduler(closed=0, ready=0, record=1, repeat=0, skip_first=0):
    def sched(step):
        if step < skip_first:
            return ProfilerState.CLOSED
        s = step - skip_first
        period = closed + ready + record
        if repeat > 0 and s // period >= repeat:
            return ProfilerState.CLOSED
        m = s % period
        if m < closed:
            return ProfilerState.CLOSED
        if m < closed + ready:
            return ProfilerState.READY
        return ProfilerState.RECORD_AND_RETURN if m == period - 1 else ProfilerState.RECORD

    return sched


def export_chrome_tracing(dir_name, worker_name=None):
    def handler(prof):
        os.makedirs(dir_name, exist_ok=True)
        name = worker_name or f"host_{os.getpid()}"
        prof._export(os.path.join(dir_name, f"{name}_{int(time.time() * 1000)}.paddle_trace.json"))

    return handler


def export_protobuf(dir_name, worker_name=None):
    return export_chrome_tracing(dir_name, worker_name)


class RecordEvent:
    """Named host range (also visible in rocprof/roctx traces through torch's record_function)."""

    def __init__(self, name, event_type=None):
        self.name = name
        self._cm = None

    def begin(self):
        self._cm = torch.profiler.record_function(self.name)
        self._cm.__enter__()

    def end(self):
        if self._cm is not None:
            self._cm.__exit__(None, None, None)
            self._cm = None

    def __enter__(self):
        self.begin()
        return self

    def __exit__(self, *a):
        self.end()


class Profiler:
    def __init__(self, targets=None, scheduler=None, on_trace_ready=None, record_shapes=False, profile_memory=False,
                 timer_only=False, emit_nvtx=False, custom_device_types=[], with_flops=False):
        targets = targets or [ProfilerTarget.CPU] + ([ProfilerTarget.GPU] if torch.cuda.is_available() else [])
        acts = [torch.profiler.ProfilerActivity.CPU]
        if ProfilerTarget.GPU in targets and torch.cuda.is_available():
            acts.append(torch.profiler.ProfilerActivity.CUDA)
        self._acts = acts
        if isinstance(scheduler, (tuple, list)):
            a, b = scheduler
            scheduler = make_scheduler(closed=a, record=b - a, repeat=1)
        self._sched = scheduler
        self._on_ready = on_trace_ready
        self._timer_only = timer_only
        self._record_shapes, self._profile_memory = record_shapes, profile_memory
        self._prof = None
        self._step = 0
        self._benchmark = Benchmark()

    def _make(self):
        return torch.profiler.profile(activities=self._acts, record_shapes=self._record_shapes,
                                      profile_memory=self._profile_memory)

    def start(self):
        self._benchmark.begin()
        if self._timer_only:
            return
        if self._sched is None or self._sched(self._step) in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN):
            self._prof = self._make()
            self._prof.__enter__()

    def stop(self):
        self._benchmark.end()
        if self._prof is not None:
            self._prof.__exit__(None, None, None)
            if self._on_ready is not None:
                self._on_ready(self)
            self._last = self._prof
            self._prof = None

    def step(self, num_samples=None):
        self._benchmark.step(num_samples)
        if self._timer_only:
            return
        self._step += 1
        if self._sched is None:
            return
        st = self._sched(self._step)
        recording = st in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN)
        if self._prof is not None and (not recording or self._sched(self._step - 1) == ProfilerState.RECORD_AND_RETURN):
            self._prof.__exit__(None, None, None)
            self._last = self._prof
            self._prof = None
            if self._on_ready is not None:
                self._on_ready(self)
        if recording and self._prof is None:
            self._prof = self._make()
            self._prof.__enter__()

    def step_info(self, unit=None):
        return self._benchmark.step_info(unit)

    def _export(self, path):
        p = getattr(self, "_last", None) or self._prof
        if p is not None:
            p.export_chrome_trace(path)

    def export(self, path="", format="json"):
        self._export(path)

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False, time_unit="ms", views=None):
        p = getattr(self, "_last", None)
        if p is None:
            return ""
        key = "cuda_time_total" if sorted_by in (SortedKeys.GPUTotal, SortedKeys.GPUAvg) else "cpu_time_total"
        s = p.key_averages().table(sort_by=key, row_limit=50)
        print(s)
        return s

    def __enter__(self):
        self.start()
        return self

    def __exit__(self, *a):
        self.stop()


class Benchmark:
    """reader_cost / batch_cost / ips timer (reference: profiler/timer.py:351)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self._t = None
        self._costs = []
        self._samples = []

    def begin(self):
        self._t = time.perf_counter()

    def step(self, num_samples=None):
        now = time.perf_counter()
        if self._t is not None:
            self._costs.append(now - self._t)
            self._samples.append(num_samples or 0)
        self._t = now

    def end(self):
        pass

    def step_info(self, unit=None):
        if not self._costs:
            return ""
        c = sum(self._costs[-10:]) / len(self._costs[-10:])
        s = sum(self._samples[-10:]) / len(self._samples[-10:]) if self._samples else 0
        ips = s / c if c > 0 and s else 1.0 / c if c > 0 else 0
        return f"batch_cost: {c:.5f} s ips: {ips:.3f} {unit or 'steps/s'}"


def load_profiler_result(filename):
    with open(filename) as f:
        return json.load(f)


@contextlib.contextmanager
def _nvtx_range(name):
    with torch.profiler.record_function(name):
        yield
