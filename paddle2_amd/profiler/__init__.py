"""paddle.profiler (reference: python/paddle/profiler/profiler.py, timer.py Benchmark,
phi/api/profiler/host_tracer.cc, chrome_tracing_logger.cc).

Host events: ``RecordEvent`` scopes and the framework's own ranges (optimizer step, data loader,
collectives) go to the NATIVE host tracer (csrc/runtime/tracer.cpp — per-thread buffers, interned
names, steady-clock ns), which costs one bool test when profiling is off.  Device activity comes
from torch's profiler, backed on ROCm by rocprofiler-sdk, so HIP kernels (ours included) appear in
the same chrome trace: ``export`` merges the native host events into the device trace file.
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


class TracerEventType(enum.Enum):
    UserDefined = 0
    Operator = 1
    Communication = 2
    Dataloader = 3
    Optimization = 4
    Forward = 5
    Backward = 6
    ProfileStep = 7


_TYPE_CODE = {TracerEventType.UserDefined: 0, TracerEventType.Operator: 1, TracerEventType.Communication: 2,
              TracerEventType.Dataloader: 3, TracerEventType.Optimization: 4, TracerEventType.Forward: 1,
              TracerEventType.Backward: 1, TracerEventType.ProfileStep: 0}
_host_on = False  # fast path: framework ranges cost one global read when profiling is off


def _rt():
    from .. import _rt as R

    return R.get()


@contextlib.contextmanager
def host_range(name, etype=0):
    """Framework-internal range for the native tracer (no-op unless a Profiler is recording)."""
    if not _host_on:
        yield
        return
    rt = _rt()
    rt.tracer_push(name, etype)
    try:
        yield
    finally:
        rt.tracer_pop()


class RecordEvent:
    """Named host range: native host tracer + torch record_function (so it also brackets device work
    in rocprofiler traces)."""

    def __init__(self, name, event_type=TracerEventType.UserDefined):
        self.name = name
        self._code = _TYPE_CODE.get(event_type, 0) if isinstance(event_type, TracerEventType) else 0
        self._cm = None
        self._native = False

    def begin(self):
        if _host_on:
            _rt().tracer_push(self.name, self._code)
            self._native = True
        self._cm = torch.profiler.record_function(self.name)
        self._cm.__enter__()

    def end(self):
        if self._cm is not None:
            self._cm.__exit__(None, None, None)
            self._cm = None
        if self._native:
            _rt().tracer_pop()
            self._native = False

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

    def _host(self, on):
        global _host_on
        _host_on = on
        rt = _rt()
        if on:
            rt.tracer_clear()
        rt.tracer_enable(on)

    def start(self):
        self._benchmark.begin()
        if self._timer_only:
            return
        self._host(True)
        if self._sched is None or self._sched(self._step) in (ProfilerState.RECORD, ProfilerState.RECORD_AND_RETURN):
            self._prof = self._make()
            self._prof.__enter__()

    def stop(self):
        self._benchmark.end()
        if not self._timer_only:
            self._host_events = _rt().tracer_events()
            self._host(False)
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
        """One chrome trace: torch/rocprofiler device+op events merged with the native host events."""
        p = getattr(self, "_last", None) or self._prof
        trace = {"traceEvents": []}
        if p is not None:
            tmp = path + ".tmp"
            p.export_chrome_trace(tmp)
            with open(tmp) as f:
                trace = json.load(f)
            os.remove(tmp)
        host = getattr(self, "_host_events", None) or _rt().tracer_events()
        if host:
            # align the native steady clock to the device trace's time base by its earliest event
            ev = trace.get("traceEvents", [])
            ts0 = min((e.get("ts", 0) for e in ev if isinstance(e.get("ts"), (int, float))), default=0)
            h0 = min(e[3] for e in host)
            cats = ["UserDefined", "Operator", "Communication", "Dataloader", "Optimization"]
            pid = os.getpid()
            for name, code, tid, s_ns, e_ns in host:
                ev.append({"name": name, "cat": cats[code] if code < 5 else "UserDefined", "ph": "X",
                           "pid": f"host {pid}", "tid": tid, "ts": ts0 + (s_ns - h0) / 1000.0,
                           "dur": (e_ns - s_ns) / 1000.0})
            trace["traceEvents"] = ev
        with open(path, "w") as f:
            json.dump(trace, f)

    def export(self, path="", format="json"):
        self._export(path)

    def host_statistics(self):
        """{name: (calls, total_ms, avg_ms, max_ms, min_ms)} over the native host events."""
        stats = {}
        for name, code, tid, s_ns, e_ns in getattr(self, "_host_events", None) or []:
            d = (e_ns - s_ns) / 1e6
            c, t, mx, mn = stats.get(name, (0, 0.0, 0.0, float("inf")))
            stats[name] = (c + 1, t + d, max(mx, d), min(mn, d))
        return {k: (c, t, t / c, mx, mn) for k, (c, t, mx, mn) in stats.items()}

    def summary(self, sorted_by=SortedKeys.CPUTotal, op_detail=True, thread_sep=False, time_unit="ms", views=None):
        lines = []
        hs = self.host_statistics()
        if hs:
            lines.append(f"{'Event':<48}{'Calls':>8}{'Total(ms)':>12}{'Avg(ms)':>10}{'Max(ms)':>10}{'Min(ms)':>10}")
            for k, (c, t, a, mx, mn) in sorted(hs.items(), key=lambda kv: -kv[1][1]):
                lines.append(f"{k[:47]:<48}{c:>8}{t:>12.3f}{a:>10.3f}{mx:>10.3f}{mn:>10.3f}")
        p = getattr(self, "_last", None)
        if p is not None:
            key = "cuda_time_total" if sorted_by in (SortedKeys.GPUTotal, SortedKeys.GPUAvg) else "cpu_time_total"
            lines.append(p.key_averages().table(sort_by=key, row_limit=50))
        s = "\n".join(lines)
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
