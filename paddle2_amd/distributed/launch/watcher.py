"""GPU utilisation / memory watcher of the launcher (``--enable_gpu_log``, on by default).

Reference behaviour: python/paddle/distributed/launch/controllers/watcher.py — a daemon thread that writes
``<log_dir>/<job_id>.gpu.log``: a device-info block, then one CSV row per device every ``interval`` seconds
(index, utilisation, memory total / used / free, timestamp).  The reference reads nvidia-smi and returns early
on ROCm builds; here the source is the amdgpu driver's sysfs files, so there is no tool process per sample:

    /sys/class/drm/cardN/device/gpu_busy_percent       utilisation (%)
    /sys/class/drm/cardN/device/mem_info_vram_total    bytes
    /sys/class/drm/cardN/device/mem_info_vram_used     bytes
    /sys/class/drm/cardN/device/{unique_id,vbios_version,current_link_speed}

Devices are the amdgpu cards (vendor 0x1002 with a gpu_busy_percent file) in PCI-address order, which is the HIP
enumeration order of a node without HIP_VISIBLE_DEVICES; ``PADDLE2_AMD_SYSFS_ROOT`` relocates /sys for tests.
"""
from __future__ import annotations

import os
import threading
import time

_MB = 1 << 20


def _sysfs_root():
    return os.environ.get("PADDLE2_AMD_SYSFS_ROOT", "/sys")


def _read(path, default=None):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def amd_gpus():
    """-> [(index, device_dir)] of the amdgpu cards, in PCI-address order."""
    drm = os.path.join(_sysfs_root(), "class", "drm")
    found = []
    try:
        names = os.listdir(drm)
    except OSError:
        return []
    for n in names:
        if not n.startswith("card") or not n[4:].isdigit():
            continue
        dev = os.path.join(drm, n, "device")
        if _read(os.path.join(dev, "vendor"), "") != "0x1002" or not os.path.exists(os.path.join(dev, "gpu_busy_percent")):
            continue
        pci = os.path.basename(os.path.realpath(dev))
        found.append((pci, dev))
    found.sort()
    return [(i, d) for i, (_, d) in enumerate(found)]


def sample(dev):
    """One reading of a device directory: (util %, total MiB, used MiB, free MiB)."""
    util = int(_read(os.path.join(dev, "gpu_busy_percent"), "0") or 0)
    total = int(_read(os.path.join(dev, "mem_info_vram_total"), "0") or 0) // _MB
    used = int(_read(os.path.join(dev, "mem_info_vram_used"), "0") or 0) // _MB
    return util, total, used, max(total - used, 0)


class Watcher:
    UTIL_KEY = "index,utilization_gpu,memory_total,memory_used,memory_free,timestamp"
    INFO_KEY = "index,pci,unique_id,vbios_version,link_speed"

    def __init__(self, log_dir, job_id="default", devices=None, interval=5.0):
        self.interval = float(interval)
        gpus = amd_gpus()
        if devices:
            want = {int(d) for d in devices}
            gpus = [(i, d) for i, d in gpus if i in want]
        self.gpus = gpus
        self._stop = threading.Event()
        self._th = None
        self.path = None
        if not gpus:
            return
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, f"{job_id}.gpu.log")
        self._f = open(self.path, "w")
        self._write_info()
        self._th = threading.Thread(target=self._watch, daemon=True)
        self._th.start()

    def _write_info(self):
        f = self._f
        f.write(self.INFO_KEY + "\n")
        for i, d in self.gpus:
            f.write(",".join([str(i), os.path.basename(os.path.realpath(d)), _read(os.path.join(d, "unique_id"), ""),
                              _read(os.path.join(d, "vbios_version"), ""),
                              _read(os.path.join(d, "current_link_speed"), "")]) + "\n")
        f.write("\n" + self.UTIL_KEY + "\n")
        f.flush()

    def _row(self):
        ts = time.strftime("%Y/%m/%d %H:%M:%S")
        for i, d in self.gpus:
            u, tot, used, free = sample(d)
            self._f.write(f"{i},{u},{tot},{used},{free},{ts}\n")
        self._f.flush()

    def _watch(self):
        while not self._stop.is_set():
            try:
                self._row()
            except (OSError, ValueError):   # a vanished card or a torn read: skip this sample
                pass
            self._stop.wait(self.interval)

    def stop(self):
        if self._th is not None:
            self._stop.set()
            self._th.join(timeout=self.interval + 1.0)
            try:
                self._row()   # final sample at job end
            except (OSError, ValueError):
                pass
            self._f.close()
            self._th = None
