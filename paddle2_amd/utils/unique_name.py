"""paddle.utils.unique_name."""
import collections
import contextlib

_counters = collections.defaultdict(int)


def generate(key):
    n = _counters[key]
    _counters[key] += 1
    return f"{key}_{n}"


@contextlib.contextmanager
def guard(new_generator=None):
    global _counters
    saved = _counters
    _counters = collections.defaultdict(int)
    try:
        yield
    finally:
        _counters = saved


def switch(new_generator=None, new_para_name_checker=None):
    global _counters
    old = _counters
    _counters = collections.defaultdict(int)
    return old
