"""Rendezvous key-value store (reference: phi/core/distributed/store/tcp_store.h, exposed as
``paddle.base.core.TCPStore`` and used by ``init_parallel_env`` / the launcher).

``TCPStore`` wraps the native C++ daemon/client (csrc/runtime/tcp_store.cpp).  ``TorchStore``
adapts it to ``torch.distributed.Store`` so RCCL/gloo process groups can rendezvous through the
native store (``init_parallel_env``'s default store: collective._rendezvous_store).
"""
from __future__ import annotations

import datetime

import torch.distributed as dist


def _rt():
    from .. import _rt

    return _rt.get()


class TCPStore:
    def __init__(self, hostname="127.0.0.1", port=0, is_master=False, world_size=1, timeout=900):
        rt = _rt()
        self._server = rt.TCPStoreServer(hostname if is_master else "0.0.0.0", int(port)) if is_master else None
        self.port = self._server.port if self._server is not None else int(port)
        self.host = hostname
        self.world_size = world_size
        self.timeout = timeout
        self._client = rt.TCPStoreClient(hostname, self.port, float(timeout))

    # Paddle API
    def set(self, key, value):
        if isinstance(value, str):
            value = value.encode()
        elif not isinstance(value, (bytes, bytearray)):
            value = bytes(value)
        self._client.set(key, bytes(value))

    def get(self, key):
        return self._client.get(key)

    def add(self, key, value):
        return self._client.add(key, int(value))

    def wait(self, key):
        self._client.wait([key] if isinstance(key, str) else list(key))

    def check(self, keys):
        return self._client.check([keys] if isinstance(keys, str) else list(keys))

    def delete_key(self, key):
        return self._client.delete_key(key)

    def num_keys(self):
        return self._client.num_keys()

    def barrier(self, name, world_size=None, rank=None):
        """All ``world_size`` participants arrive before anyone leaves."""
        n = world_size or self.world_size
        cnt = self.add(f"__barrier/{name}", 1)
        if cnt == n:
            self.set(f"__barrier/{name}/done", b"1")
        self.wait(f"__barrier/{name}/done")

    def shutdown(self):
        if self._server is not None:
            self._server.shutdown()
            self._server = None


_LIVE = []


def release_clones():
    """Drop the per-group clone connections once every process group is gone (destroy_process_group of the
    world): c10d then holds none of them, and each one's socket closes with its client."""
    _LIVE[:] = [s for s in _LIVE if not getattr(s, "_is_clone", False)]


class TorchStore(dist.Store):
    """torch.distributed.Store backed by the native TCPStore client."""

    def __init__(self, store: TCPStore):
        super().__init__()
        self._s = store
        self._c = store._client
        # c10d keeps only the C++ half of a Python-subclassed store alive; once the Python object is collected its
        # overrides are gone and every call fails ("Not implemented"), so the job holds every instance
        _LIVE.append(self)

    def set(self, key, value):
        self._c.set(key, value.encode() if isinstance(value, str) else bytes(value))

    def get(self, key):
        return self._c.get(key)

    def add(self, key, value):
        return self._c.add(key, int(value))

    def compare_set(self, key, expected, desired):
        e = expected.encode() if isinstance(expected, str) else bytes(expected)
        d = desired.encode() if isinstance(desired, str) else bytes(desired)
        return self._c.compare_set(key, e, d)

    def wait(self, keys, timeout=None):
        self._c.wait(list(keys))

    def check(self, keys):
        return self._c.check(list(keys))

    def delete_key(self, key):
        return self._c.delete_key(key)

    def num_keys(self):
        return self._c.num_keys()

    def set_timeout(self, timeout):
        self._c.set_timeout(timeout.total_seconds() if isinstance(timeout, datetime.timedelta) else float(timeout))

    def clone(self):
        """A second client connection to the same daemon (ProcessGroupGloo clones the store for every group).
        Clones are held (see _LIVE) until the job's groups are destroyed, then released (release_clones)."""
        c = TorchStore(TCPStore(self._s.host, self._s.port, False, self._s.world_size, self._s.timeout))
        c._is_clone = True
        return c

    def multi_get(self, keys):
        return [self._c.get(k) for k in keys]

    def multi_set(self, keys, values):
        for k, v in zip(keys, values):
            self.set(k, v)

    def append(self, key, value):
        # one server-side command: concurrent appends (identical bytes included) all land, in arrival order
        v = value.encode() if isinstance(value, str) else bytes(value)
        self._c.append(key, v)

    def has_extended_api(self):
        return False


_global_store = None


def create_or_get_global_tcp_store(rank=None, world=None, host=None, port=None, timeout=900):
    """One store per job: rank 0 hosts the daemon at MASTER_ADDR:MASTER_PORT, every rank connects."""
    global _global_store
    if _global_store is None:
        import os

        rank = int(os.environ.get("RANK", os.environ.get("PADDLE_TRAINER_ID", 0))) if rank is None else rank
        world = int(os.environ.get("WORLD_SIZE", os.environ.get("PADDLE_TRAINERS_NUM", 1))) if world is None else world
        host = host or os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(port or os.environ.get("MASTER_PORT", 29500))
        _global_store = TCPStore(host, port, rank == 0, world, timeout)
    return _global_store
