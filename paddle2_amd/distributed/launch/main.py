"""``python -m paddle2_amd.distributed.launch`` — collective job launcher.

Reference: python/paddle/distributed/launch/ (main.py, context/args_envs.py, controllers/
collective.py:91-200 ``_build_pod_with_args`` / ``_build_pod_with_master``, controllers/watcher.py,
controllers/master.py HTTPMaster, job/container.py log files ``workerlog.N``), and the legacy fleet/launch.py.

One process per GPU.  Multi-node jobs rendezvous through the native C++ TCPStore
(csrc/runtime/tcp_store.cpp) hosted by node 0 at ``--master``: every node registers its address
and process count, node ranks / global rank offsets are derived from the registration order
(or ``--rank``), and each worker gets both Paddle's env contract (PADDLE_TRAINER_ID,
PADDLE_TRAINERS_NUM, PADDLE_CURRENT_ENDPOINT, PADDLE_TRAINER_ENDPOINTS, PADDLE_MASTER,
FLAGS_selected_gpus, ...) and torch.distributed's (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).
``--master http://host:port`` rendezvouses through the HTTP key-value master instead (launch/master.py, the
reference's default master).  The GPU watcher (launch/watcher.py, ``--enable_gpu_log``) samples every
device's utilisation and memory from the amdgpu sysfs into ``<log_dir>/<job_id>.gpu.log``.
The launcher restarts the whole pod up to ``--max_restart`` times when a worker fails (fault
tolerance level 1) and otherwise tears the pod down and exits with the failing worker's code.

Elastic mode (``--nnodes MIN:MAX``, reference fleet/elastic): membership is tracked by the
ElasticManager over the same TCPStore (heartbeats, TTL); when nodes join or leave, every
surviving launcher stops its pod, re-rendezvouses with the new node set and restarts the
workers with the new world size (workers resume from their checkpoint).  A worker exiting with
code 101 (ELASTIC_EXIT_CODE) also triggers a re-rendezvous.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import threading
import time


def _parse(argv=None):
    ap = argparse.ArgumentParser("paddle2_amd.distributed.launch")
    ap.add_argument("--master", default=None, help="host:port of the rendezvous store (node 0)")
    ap.add_argument("--nnodes", default="1", help="number of nodes (N or MIN:MAX for elastic)")
    ap.add_argument("--rank", type=int, default=-1, help="node rank (-1: assigned at rendezvous)")
    ap.add_argument("--nproc_per_node", "--nproc-per-node", type=int, default=None)
    ap.add_argument("--devices", "--gpus", dest="devices", default=None, help="comma separated device ids")
    ap.add_argument("--log_dir", "--log-dir", dest="log_dir", default="log")
    ap.add_argument("--job_id", "--job-id", dest="job_id", default="default")
    ap.add_argument("--run_mode", "--run-mode", dest="run_mode", default="collective")
    ap.add_argument("--max_restart", "--max-restart", dest="max_restart", type=int, default=0)
    ap.add_argument("--elastic_level", type=int, default=-1)
    ap.add_argument("--elastic_ttl", "--elastic-ttl", dest="elastic_ttl", type=float, default=60.0,
                    help="elastic: seconds without heartbeat before a node is considered gone")
    ap.add_argument("--auto_tuner_json", "--auto-tuner-json", dest="auto_tuner_json", default=None,
                    help="run the hybrid-parallel auto tuner with this config instead of a single job")
    ap.add_argument("--host", default=None, help="this node's address")
    ap.add_argument("--start_port", type=int, default=None)
    ap.add_argument("--enable_gpu_log", "--enable-gpu-log", dest="enable_gpu_log", default="True",
                    help="GPU utilisation / memory log <log_dir>/<job_id>.gpu.log (True / False)")
    ap.add_argument("--gpu_log_interval", type=float, default=5.0, help="seconds between GPU log samples")
    ap.add_argument("training_script")
    ap.add_argument("training_script_args", nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def _free_port(host="127.0.0.1"):
    s = socket.socket()
    s.bind((host, 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _local_ip():
    return os.environ.get("POD_IP", "127.0.0.1")


def _device_list(args):
    if args.devices:
        return [d for d in args.devices.split(",") if d != ""]
    env = os.environ.get("CUDA_VISIBLE_DEVICES") or os.environ.get("HIP_VISIBLE_DEVICES")
    if env:
        return [d for d in env.split(",") if d != ""]
    try:
        import torch

        n = torch.cuda.device_count()  # counting devices does not initialise the GPU on this image
    except Exception:  # pragma: no cover
        n = 0
    return [str(i) for i in range(n)] if n else []


class _Rendezvous:
    """Node-level rendezvous over the native TCPStore: -> (node_rank, nnodes, world, rank_offset, endpoints)."""

    def __init__(self, args, nproc, host):
        self.args, self.nproc, self.host = args, nproc, host

    def run(self):
        nnodes = int(str(self.args.nnodes).split(":")[-1])
        if nnodes == 1:
            ports = [self.args.start_port + i if self.args.start_port else _free_port() for i in range(self.nproc)]
            eps = [f"{self.host}:{p}" for p in ports]
            return 0, 1, self.nproc, 0, eps, None
        if self.args.master.startswith("http://"):
            return self._run_http(nnodes)
        from ..store import TCPStore

        mhost, mport = self.args.master.rsplit(":", 1)
        is_master = self.args.rank == 0 or (self.args.rank < 0 and self.host == mhost and _try_bind(mhost, int(mport)))
        store = TCPStore(mhost, int(mport), is_master=is_master, world_size=nnodes, timeout=600)
        job = self.args.job_id
        node_rank = self.args.rank if self.args.rank >= 0 else store.add(f"{job}/node_counter", 1) - 1
        ports = [_free_port() for _ in range(self.nproc)]
        store.set(f"{job}/node/{node_rank}", f"{self.host}|{self.nproc}|{','.join(map(str, ports))}")
        infos = []
        for r in range(nnodes):
            store.wait(f"{job}/node/{r}")
            infos.append(store.get(f"{job}/node/{r}").decode().split("|"))
        offset = sum(int(i[1]) for i in infos[:node_rank])
        world = sum(int(i[1]) for i in infos)
        eps = [f"{h}:{p}" for h, _, ps in infos for p in ps.split(",")]
        return node_rank, nnodes, world, offset, eps, store


    def _run_http(self, nnodes):
        """Rendezvous through the HTTP KV master (reference controllers/master.py HTTPMaster.sync_peers)."""
        from .master import HTTPMaster

        ep = self.args.master[len("http://"):]
        mhost = ep.rsplit(":", 1)[0]
        if self.args.rank >= 0:
            is_main = self.args.rank == 0
        else:
            is_main = None if mhost in ("127.0.0.1", "localhost", self.host) else False
        master = HTTPMaster(ep, is_main=is_main)
        ports = [_free_port() for _ in range(self.nproc)]
        val = f"{self.host}|{self.nproc}|{','.join(map(str, ports))}"
        vals, node_rank = master.sync_peers(f"{self.args.job_id}/nodes", f"{self.host}:{os.getpid()}", val, nnodes,
                                            self.args.rank)
        infos = [v.split("|") for v in vals]
        offset = sum(int(i[1]) for i in infos[:node_rank])
        world = sum(int(i[1]) for i in infos)
        eps = [f"{h}:{p}" for h, _, ps in infos for p in ps.split(",")]
        return node_rank, nnodes, world, offset, eps, master


def _try_bind(host, port):
    s = socket.socket()
    try:
        s.bind((host if host not in ("localhost",) else "127.0.0.1", port))
        return True
    except OSError:
        return False
    finally:
        s.close()


def _worker_env(args, local_rank, node_rank, nnodes, world, offset, eps, devices, torch_master):
    grank = offset + local_rank
    env = dict(os.environ)
    # more ranks than devices (e.g. gloo ranks sharing one GPU): ranks wrap around the device list
    dev = devices[local_rank % len(devices)] if devices else str(local_rank)
    env.update({
        "RANK": str(grank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(local_rank),
        "LOCAL_WORLD_SIZE": str(args.nproc_per_node or (len(devices) if devices else 1)), "GROUP_RANK": str(node_rank),
        "MASTER_ADDR": torch_master[0], "MASTER_PORT": str(torch_master[1]),
        "PADDLE_TRAINER_ID": str(grank), "PADDLE_GLOBAL_RANK": str(grank), "PADDLE_LOCAL_RANK": str(local_rank),
        "PADDLE_TRAINERS_NUM": str(world), "PADDLE_GLOBAL_SIZE": str(world), "PADDLE_NNODES": str(nnodes),
        "PADDLE_CURRENT_ENDPOINT": eps[grank], "PADDLE_TRAINER_ENDPOINTS": ",".join(eps),
        "PADDLE_MASTER": f"{torch_master[0]}:{torch_master[1]}", "PADDLE_JOB_ID": args.job_id,
        "FLAGS_selected_gpus": dev, "FLAGS_selected_accelerators": dev,
    })
    if devices and (args.nproc_per_node or len(devices)) <= len(devices):
        env.setdefault("PADDLE_DISTRI_BACKEND", "nccl")   # RCCL needs one device per rank
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _tee(src, f):
    for line in iter(src.readline, b""):
        sys.stdout.buffer.write(line)
        sys.stdout.flush()
        f.write(line)
        f.flush()


class Pod:
    def __init__(self, args, cmd, envs):
        self.args, self.cmd, self.envs = args, cmd, envs
        self.procs, self.logs, self.tees = [], [], []

    def start(self):
        os.makedirs(self.args.log_dir, exist_ok=True)
        for i, env in enumerate(self.envs):
            path = os.path.join(self.args.log_dir, f"workerlog.{i}")
            f = open(path, "ab")
            self.logs.append(f)
            if env["RANK"] == "0":
                # global rank 0: tee to the console and its log file
                p = subprocess.Popen(self.cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
                t = threading.Thread(target=_tee, args=(p.stdout, f), daemon=True)
                t.start()
                self.tees.append(t)
            else:
                p = subprocess.Popen(self.cmd, env=env, stdout=f, stderr=subprocess.STDOUT)
            self.procs.append(p)

    def poll(self):
        """-> None while running, 0 when all succeeded, else the first failing exit code."""
        codes = [p.poll() for p in self.procs]
        for c in codes:
            if c not in (None, 0):
                return c
        if all(c == 0 for c in codes):
            return 0
        return None

    def stop(self, grace=10.0):
        for p in self.procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        t = time.time()
        for p in self.procs:
            while p.poll() is None and time.time() - t < grace:
                time.sleep(0.1)
            if p.poll() is None:
                p.kill()
        for t in self.tees:  # rank 0's last console lines (e.g. a benchmark's JSON) must reach stdout
            t.join(timeout=grace)
        for f in self.logs:
            f.close()


def _launch_elastic(args, nproc, devices, host):
    from ..fleet.elastic.manager import ELASTIC_EXIT_CODE, ElasticManager, ElasticStatus
    from ..store import TCPStore

    mhost, mport = args.master.rsplit(":", 1)
    is_master = args.rank == 0 or (args.rank < 0 and _try_bind(mhost, int(mport)))
    store = TCPStore(mhost, int(mport), is_master=is_master, world_size=1, timeout=600)
    mgr = ElasticManager(store, args.job_id, host, nproc, args.nnodes, ttl=args.elastic_ttl,
                         store_addr=(mhost, int(mport)))
    mgr.register()
    cmd = [sys.executable, "-u", args.training_script] + list(args.training_script_args)
    round_id, restarts = 0, 0
    try:
        while True:
            members, torch_master = mgr.rendezvous(round_id, _free_port)
            if members is None:  # more nodes than MAX: wait for a later round
                round_id += 1
                time.sleep(1.0)
                continue
            node_rank = [m[0] for m in members].index(mgr.slot)
            world = sum(m[2] for m in members)
            offset = sum(m[2] for m in members[:node_rank])
            mgr.publish_ports(round_id, [_free_port() for _ in range(nproc)])
            eps = mgr.gather_ports(round_id, members)
            print(f"[launch] elastic round {round_id}: {len(members)} node(s), world {world}, node rank {node_rank}",
                  file=sys.stderr, flush=True)
            envs = [_worker_env(args, i, node_rank, len(members), world, offset, eps, devices, torch_master)
                    for i in range(nproc)]
            pod = Pod(args, cmd, envs)
            pod.start()
            status, code = None, None
            while code is None and status is None:
                time.sleep(0.5)
                code = pod.poll()
                if code is None:
                    status = mgr.watch(members)
                    if status == ElasticStatus.COMPLETED:
                        status = None  # a peer finished: let our workers finish too
            pod.stop()
            if code == 0:
                mgr.exit(completed=True)
                return 0
            if status == ElasticStatus.RESTART or code == ELASTIC_EXIT_CODE or restarts < args.max_restart:
                if code not in (None, ELASTIC_EXIT_CODE):
                    restarts += 1
                print(f"[launch] elastic restart (membership change or exit {code})", file=sys.stderr, flush=True)
                round_id += 1
                continue
            mgr.exit()
            return code
    finally:
        mgr._stop.set()


def launch(argv=None):
    args = _parse(argv)
    if args.auto_tuner_json:
        import json

        from ..auto_tuner.launch import run as _tune

        with open(args.auto_tuner_json) as f:
            tuner_cfg = json.load(f)
        raw = sys.argv[1:] if argv is None else list(argv)
        i = raw.index("--auto_tuner_json") if "--auto_tuner_json" in raw else raw.index("--auto-tuner-json")
        rest = raw[:i] + raw[i + 2:]
        j = rest.index(args.training_script)
        best, _ = _tune(tuner_cfg, rest[:j], args.training_script, rest[j + 1:],
                        log_root=os.path.join(args.log_dir, "auto_tuner"))
        print(f"[auto_tuner] best config: {best}", flush=True)
        return 0 if best is not None else 1
    devices = _device_list(args)
    nproc = args.nproc_per_node or (len(devices) if devices else 1)
    if devices and len(devices) > nproc:
        devices = devices[:nproc]
    host = args.host or _local_ip()
    if ":" in str(args.nnodes):
        if not args.master:
            raise SystemExit("elastic mode (--nnodes MIN:MAX) needs --master host:port")
        return _launch_elastic(args, nproc, devices, host)
    node_rank, nnodes, world, offset, eps, store = _Rendezvous(args, nproc, host).run()
    if args.master and nnodes > 1:
        mep = args.master[len("http://"):] if args.master.startswith("http://") else args.master
        mhost = mep.rsplit(":", 1)[0]
        torch_port = int(mep.rsplit(":", 1)[1]) + 1
        torch_master = (mhost, torch_port)
    else:
        torch_master = ("127.0.0.1", _free_port())
    watcher = None
    if str(args.enable_gpu_log).lower() in ("1", "true", "yes"):
        from .watcher import Watcher

        watcher = Watcher(args.log_dir, args.job_id, devices, args.gpu_log_interval)
    try:
        return _run_pods(args, nproc, devices, node_rank, nnodes, world, offset, eps, torch_master)
    finally:
        if watcher is not None:
            watcher.stop()
        if hasattr(store, "stop"):
            store.stop()


def _run_pods(args, nproc, devices, node_rank, nnodes, world, offset, eps, torch_master):
    cmd = [sys.executable, "-u", args.training_script] + list(args.training_script_args)
    restarts = 0
    while True:
        envs = [_worker_env(args, i, node_rank, nnodes, world, offset, eps, devices, torch_master)
                for i in range(nproc)]
        pod = Pod(args, cmd, envs)
        pod.start()

        def _forward(sig, frm, pod=pod):
            pod.stop(grace=5.0)
            sys.exit(128 + sig)

        signal.signal(signal.SIGINT, _forward)
        signal.signal(signal.SIGTERM, _forward)
        code = None
        while code is None:
            time.sleep(0.5)
            code = pod.poll()
        pod.stop()
        if code == 0:
            return 0
        if restarts < args.max_restart:
            restarts += 1
            print(f"[launch] worker failed with exit code {code}; restarting pod ({restarts}/{args.max_restart})",
                  file=sys.stderr, flush=True)
            if nnodes == 1:
                torch_master = ("127.0.0.1", _free_port())
            continue
        print(f"[launch] worker failed with exit code {code}; see {args.log_dir}/workerlog.*", file=sys.stderr,
              flush=True)
        return code


def main():
    sys.exit(launch())


if __name__ == "__main__":
    main()
