"""Named device-synchronised timers (reference: fleet/utils/timer_helper.py:113)."""
from __future__ import annotations

import time

import torch


class _Timer:
    def __init__(self, name):
        self.name = name
        self.elapsed_ = 0.0
        self.started_ = False
        self.start_time = 0.0

    @staticmethod
    def _sync():
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            torch.cuda.synchronize()

    def start(self):
        assert not self.started_, f"timer {self.name} already started"
        self._sync()
        self.start_time = time.time()
        self.started_ = True

    def stop(self):
        assert self.started_, f"timer {self.name} not started"
        self._sync()
        self.elapsed_ += time.time() - self.start_time
        self.started_ = False

    def reset(self):
        self.elapsed_ = 0.0
        self.started_ = False

    def elapsed(self, reset=True):
        started = self.started_
        if started:
            self.stop()
        e = self.elapsed_
        if reset:
            self.reset()
        if started:
            self.start()
        return e


class Timers:
    def __init__(self):
        self.timers = {}

    def __call__(self, name):
        if name not in self.timers:
            self.timers[name] = _Timer(name)
        return self.timers[name]

    def log(self, names, normalizer=1.0, reset=True):
        s = "time (ms)"
        for n in names:
            s += f" | {n}: {self.timers[n].elapsed(reset) * 1000.0 / normalizer:.2f}"
        print(s, flush=True)
        return s


_GLOBAL_TIMERS = None


def get_timers():
    return _GLOBAL_TIMERS


def set_timers():
    global _GLOBAL_TIMERS
    _GLOBAL_TIMERS = Timers()
    return _GLOBAL_TIMERS
