"""Launcher HTTP KV master and GPU watcher (reference: python/paddle/distributed/launch/controllers/master.py
HTTPMaster, utils/kv_server.py / kv_client.py, controllers/watcher.py)."""
import os
import socket
import subprocess
import sys
import threading

from _dist import pypath as _pypath

from paddle2_amd.distributed.launch.master import HTTPMaster, KVClient, KVServer
from paddle2_amd.distributed.launch.watcher import Watcher, amd_gpus, sample

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_kv_server_roundtrip():
    srv = KVServer(0, host="127.0.0.1")
    srv.start()
    try:
        c = KVClient(f"127.0.0.1:{srv.port}")
        assert c.wait_server_ready(2.0)
        assert c.get("missing") is None
        assert c.put("job/a/0", "x|1|2") and c.put("job/b/1", b"\x00\xffraw") and c.put("other", "z")
        assert c.get("job/a/0") == b"x|1|2"
        assert c.get("job/b/1") == b"\x00\xffraw"
        got = c.get_prefix("job/")
        assert set(got) == {"job/a/0", "job/b/1"} and got["job/a/0"] == "x|1|2"
        assert c.delete("job/a/0") and c.get("job/a/0") is None
    finally:
        srv.stop()
    assert not KVClient(f"127.0.0.1:{srv.port}", timeout=0.5).wait_server_ready(0.3)


def test_sync_peers_orders_nodes():
    port = _port()
    out = {}

    def node(i, main):
        m = HTTPMaster(f"127.0.0.1:{port}", is_main=main, timeout=30)
        out[i] = m.sync_peers("job/nodes", f"host{i}", f"v{i}", 3)
        if main:
            m.stop(linger=0.5)

    ts = [threading.Thread(target=node, args=(0, True))]
    ts += [threading.Thread(target=node, args=(i, False)) for i in (1, 2)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    vals = out[0][0]
    assert vals[0] == "v0"                              # the hosting node sorts first
    assert sorted(vals) == ["v0", "v1", "v2"]
    assert all(out[i][0] == vals for i in range(3))     # every node sees one order
    assert sorted(out[i][1] for i in range(3)) == [0, 1, 2]
    assert all(vals[out[i][1]] == f"v{i}" for i in range(3))


def test_sync_peers_explicit_ranks():
    port = _port()
    out = {}

    def node(rank):
        m = HTTPMaster(f"127.0.0.1:{port}", is_main=rank == 0, timeout=30)
        out[rank] = m.sync_peers("j", f"zz{rank}", f"r{rank}", 2, rank=rank)
        if rank == 0:
            m.stop(linger=0.5)

    ts = [threading.Thread(target=node, args=(r,)) for r in (1, 0)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    assert out[0] == (["r0", "r1"], 0) and out[1] == (["r0", "r1"], 1)


WORKER = r'''
import os, sys
sys.path.insert(0, %r)
import paddle2_amd as paddle
import paddle2_amd.distributed as dist
dist.init_parallel_env()
t = paddle.to_tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
assert float(t) == 3.0, float(t)
print("OK rank", dist.get_rank(), "of", dist.get_world_size(), os.environ["PADDLE_TRAINER_ENDPOINTS"], flush=True)
''' % ROOT


def test_two_node_launch_over_http_master(tmp_path):
    """Two launcher processes (one rank each) rendezvous through --master http://127.0.0.1:P."""
    w = tmp_path / "w.py"
    w.write_text(WORKER)
    port = _port()
    env = dict(os.environ, PYTHONPATH=_pypath(ROOT), PADDLE2_AMD_DEVICE="cpu", PADDLE_DISTRI_BACKEND="gloo")
    procs = []
    for n in range(2):
        procs.append(subprocess.Popen(
            [sys.executable, "-m", "paddle2_amd.distributed.launch", "--master", f"http://127.0.0.1:{port}",
             "--nnodes", "2", "--rank", str(n), "--nproc_per_node", "1", "--enable_gpu_log", "False",
             "--log_dir", str(tmp_path / f"log{n}"), str(w)],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = [p.communicate(timeout=240)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), "\n----\n".join(outs)
    assert "OK rank 0 of 2" in outs[0]
    assert "OK rank 1 of 2" in (tmp_path / "log1" / "workerlog.0").read_text()


def _fake_card(root, n, pci, busy, total, used, vendor="0x1002"):
    pdir = root / "devices" / pci
    pdir.mkdir(parents=True)
    (pdir / "vendor").write_text(vendor + "\n")
    if vendor == "0x1002":
        (pdir / "gpu_busy_percent").write_text(f"{busy}\n")
        (pdir / "mem_info_vram_total").write_text(f"{total}\n")
        (pdir / "mem_info_vram_used").write_text(f"{used}\n")
        (pdir / "unique_id").write_text(f"uid{n}\n")
        (pdir / "vbios_version").write_text("113-MI355X\n")
    card = root / "class" / "drm" / f"card{n}"
    card.mkdir(parents=True)
    (card / "device").symlink_to(pdir)


def test_watcher_samples_amdgpu_sysfs(tmp_path, monkeypatch):
    root = tmp_path / "sys"
    gib = 1 << 30
    _fake_card(root, 1, "0000:85:00.0", 37, 288 * gib, 100 * gib)
    _fake_card(root, 0, "0000:05:00.0", 99, 288 * gib, 262 * gib)
    _fake_card(root, 2, "0000:09:00.0", 0, 0, 0, vendor="0x8086")   # not an AMD GPU: skipped
    monkeypatch.setenv("PADDLE2_AMD_SYSFS_ROOT", str(root))
    gpus = amd_gpus()
    assert [os.path.basename(os.path.realpath(d)) for _, d in gpus] == ["0000:05:00.0", "0000:85:00.0"]
    assert sample(gpus[0][1]) == (99, 288 * 1024, 262 * 1024, 26 * 1024)
    w = Watcher(str(tmp_path / "log"), "job", devices=["1"], interval=0.05)
    import time

    time.sleep(0.3)
    w.stop()
    text = (tmp_path / "log" / "job.gpu.log").read_text().splitlines()
    assert text[0] == Watcher.INFO_KEY and text[1].startswith("1,0000:85:00.0,uid1,113-MI355X")
    rows = [ln for ln in text if ln.startswith("1,37,")]
    assert len(rows) >= 2 and rows[0].split(",")[2:5] == ["294912", "102400", "192512"]


def test_watcher_without_gpus_is_a_noop(tmp_path, monkeypatch):
    monkeypatch.setenv("PADDLE2_AMD_SYSFS_ROOT", str(tmp_path / "empty"))
    w = Watcher(str(tmp_path / "log"), "job")
    assert w.path is None
    w.stop()
    assert not (tmp_path / "log").exists()
