"""train_epoch_range with resume (see the package doc)."""
from __future__ import annotations

import json
import os
import shutil
import time

__all__ = ["train_epoch_range", "register", "reset"]

_REGISTERED = {}


def register(obj, name=None):
    """Track ``obj`` (state_dict / set_state_dict) in the auto checkpoint."""
    _REGISTERED[name or f"obj{len(_REGISTERED)}"] = obj
    return obj


def reset():
    _REGISTERED.clear()


def _dir(checkpoint_dir):
    d = checkpoint_dir or os.environ.get("PADDLE_CHECKPOINT_PATH") or os.environ.get("PADDLE_EDL_HDFS_CHECKPOINT_PATH")
    if not d:
        return None
    job = os.environ.get("PADDLE_JOB_ID", "job")
    return os.path.join(d, job)


def _save(d, epoch):
    from ... import save

    tmp = d + ".tmp"
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(tmp)
    for name, obj in _REGISTERED.items():
        save(obj.state_dict(), os.path.join(tmp, name + ".pdparams"))
    with open(os.path.join(tmp, "meta.json"), "w") as f:
        json.dump({"epoch_no": epoch, "names": sorted(_REGISTERED)}, f)
    shutil.rmtree(d, ignore_errors=True)
    os.replace(tmp, d)


def _load(d):
    from ... import load

    meta = os.path.join(d, "meta.json")
    if not os.path.exists(meta):
        return -1
    with open(meta) as f:
        m = json.load(f)
    for name in m.get("names", []):
        if name in _REGISTERED:
            _REGISTERED[name].set_state_dict(load(os.path.join(d, name + ".pdparams")))
    return int(m["epoch_no"])


def train_epoch_range(max_epoch_num, save_checkpoint_inter=None, checkpoint_dir=None):
    d = _dir(checkpoint_dir)
    start = 0
    if d is not None:
        start = _load(d) + 1
    inter = 0.0 if save_checkpoint_inter is None else float(save_checkpoint_inter)
    last = time.time()
    for epoch in range(start, max_epoch_num):
        yield epoch
        if d is not None and (time.time() - last >= inter or epoch == max_epoch_num - 1):
            _save(d, epoch)
            last = time.time()
