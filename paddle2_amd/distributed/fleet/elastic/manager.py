"""Elastic membership over the native TCPStore (reference: python/paddle/distributed/fleet/elastic/
manager.py:125 ``ElasticManager`` — etcd host registry with lease TTL :251-296, scale in/out
watch :237-309, exit codes 101/102 :33-34).

The reference keeps its host registry in etcd; here it lives in the job's own C++ TCPStore
(csrc/runtime/tcp_store.cpp) hosted by the launcher of node 0, so no external service is needed:

  * ``register()`` claims a slot (atomic ``add``) and starts a heartbeat thread that bumps
    ``hb/<slot>`` every ttl/4 on its own store connection;
  * liveness is judged by each observer on its own clock — a slot is alive while its heartbeat
    counter keeps changing within ``ttl`` (no cross-host clock comparison);
  * ``rendezvous(round)``: the lowest alive slot waits until the alive set is stable and its
    size is within [min_np, max_np], then publishes the round's member list and the torch
    master endpoint; every member derives its node rank from the sorted slots;
  * ``watch(members)`` -> RESTART when the alive set changes (scale in / out), COMPLETED when
    some node finished the job, else HOLD.
The launcher (distributed/launch/main.py) stops the pod and re-rendezvouses on RESTART; the
training script resumes from its checkpoint with the new world size (exit code 101 asks for a
restart explicitly, as in the reference).
"""
from __future__ import annotations

import threading
import time

ELASTIC_EXIT_CODE = 101
ELASTIC_AUTO_PARALLEL_EXIT_CODE = 102
ELASTIC_TIMEOUT = 2 * 60
ELASTIC_TTL = 60


class ElasticStatus:
    COMPLETED = "completed"
    ERROR = "error"
    HOLD = "hold"
    RESTART = "restart"
    EXIT = "exit"


class LauncherInterface:
    def __init__(self, args):
        self.args = args
        self.procs = []


def _parse_np(np):
    s = str(np)
    if ":" in s:
        lo, hi = s.split(":")
        return int(lo), int(hi)
    return int(s), int(s)


class ElasticManager:
    def __init__(self, store, job_id, host, nproc=1, np="1", ttl=ELASTIC_TTL, stable_secs=None, store_addr=None):
        self.store, self.job, self.host, self.nproc = store, job_id, host, nproc
        self.min_np, self.max_np = _parse_np(np)
        self.ttl = float(ttl)
        self.stable = float(stable_secs if stable_secs is not None else min(5.0, self.ttl / 2))
        self.store_addr = store_addr  # (host, port) for the heartbeat thread's own connection
        self.slot = None
        self._seen = {}  # slot -> (counter, local time of last change)
        self._stop = threading.Event()
        self._hb = None
        self.elastic_startup_time = None

    def _k(self, *parts):
        return "/".join((self.job, "elastic") + tuple(str(p) for p in parts))

    # ---------------------------------------------------------------- registry
    def register(self):
        self.slot = self.store.add(self._k("slots"), 1) - 1
        self.store.set(self._k("host", self.slot), f"{self.host}|{self.nproc}")
        self.store.add(self._k("hb", self.slot), 1)
        self._hb = threading.Thread(target=self._heartbeat, daemon=True)
        self._hb.start()
        self.elastic_startup_time = time.time()
        return self.slot

    def _heartbeat(self):
        from ...store import TCPStore

        st = self.store
        if self.store_addr is not None:
            st = TCPStore(self.store_addr[0], self.store_addr[1], is_master=False, timeout=self.ttl)
        while not self._stop.wait(max(0.2, self.ttl / 4)):
            try:
                st.add(self._k("hb", self.slot), 1)
            except Exception:  # store gone (master exited): stop beating
                return

    def alive_slots(self):
        n = int(self.store.add(self._k("slots"), 0))
        now = time.monotonic()
        alive = []
        for s in range(n):
            if self.store.check([self._k("exit", s)]):
                continue
            v = int(self.store.add(self._k("hb", s), 0))
            last = self._seen.get(s)
            if last is None or last[0] != v:
                self._seen[s] = (v, now)
                alive.append(s)
            elif now - last[1] < self.ttl:
                alive.append(s)
        return alive

    def completed(self):
        return self.store.check([self._k("completed")])

    # ---------------------------------------------------------------- rendezvous
    def rendezvous(self, round_id, free_port, timeout=ELASTIC_TIMEOUT):
        """Block until round ``round_id``'s membership is decided; -> (members, torch_master)
        where members = [(slot, host, nproc), ...] sorted by slot, or (None, None) when this node
        is not part of the round (more nodes than max_np)."""
        key = self._k("round", round_id)
        deadline = time.monotonic() + timeout
        stable_since, last = time.monotonic(), None
        while not self.store.check([key]):
            if time.monotonic() > deadline:
                raise TimeoutError(f"elastic rendezvous round {round_id} timed out")
            alive = self.alive_slots()
            if alive != last:
                last, stable_since = alive, time.monotonic()
            if alive and alive[0] == self.slot and self.min_np <= len(alive) and \
                    time.monotonic() - stable_since >= self.stable:
                members = alive[: self.max_np]
                self.store.set(key, f"{','.join(map(str, members))}|{self.host}:{free_port()}")
                break
            time.sleep(0.2)
        slots, master = self.store.get(key).decode().split("|")
        members = [int(s) for s in slots.split(",")]
        if self.slot not in members:
            return None, None
        out = []
        for s in members:
            h, n = self.store.get(self._k("host", s)).decode().split("|")
            out.append((s, h, int(n)))
        mh, mp = master.rsplit(":", 1)
        self._members = members
        return out, (mh, int(mp))

    def publish_ports(self, round_id, ports):
        self.store.set(self._k("round", round_id, "ports", self.slot), ",".join(map(str, ports)))

    def gather_ports(self, round_id, members):
        eps = []
        for s, h, _ in members:
            k = self._k("round", round_id, "ports", s)
            self.store.wait(k)
            eps += [f"{h}:{p}" for p in self.store.get(k).decode().split(",")]
        return eps

    # ---------------------------------------------------------------- watch / exit
    def watch(self, members=None):
        if self.completed():
            return ElasticStatus.COMPLETED
        members = [m[0] if isinstance(m, tuple) else m for m in (members or getattr(self, "_members", []))]
        alive = self.alive_slots()
        if sorted(alive[: self.max_np]) != sorted(members):
            if len(alive) >= self.min_np:
                return ElasticStatus.RESTART
            return ElasticStatus.HOLD
        return None

    def exit(self, completed=False):
        if completed:
            self.store.set(self._k("completed"), b"1")
        if self.slot is not None:
            self.store.set(self._k("exit", self.slot), b"1")
        self._stop.set()
