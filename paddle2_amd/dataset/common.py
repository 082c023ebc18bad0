"""paddle.dataset.common (reference python/paddle/dataset/common.py): the data cache root and offline helpers."""
from __future__ import annotations

import glob
import hashlib
import os
import pickle

__all__ = ["DATA_HOME", "download", "md5file", "split", "cluster_files_reader", "must_mkdirs"]

DATA_HOME = os.path.expanduser(os.environ.get("PADDLE_DATA_HOME", "~/.cache/paddle/dataset"))


def must_mkdirs(path):
    os.makedirs(path, exist_ok=True)


def md5file(fname):
    h = hashlib.md5()
    with open(fname, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest()


def download(url, module_name, md5sum, save_name=None):
    """-> the cached path of ``url`` under DATA_HOME/module_name (must already be there: no network)."""
    d = os.path.join(DATA_HOME, module_name)
    path = os.path.join(d, save_name or url.split("/")[-1])
    if not os.path.exists(path):
        raise FileNotFoundError(f"{path} is missing and downloads are disabled here; place the file from {url} there")
    if md5sum and md5file(path) != md5sum:
        raise OSError(f"md5 mismatch for {path}")
    return path


def _local(module_name, fname):
    return download("local://" + fname, module_name, None, fname)


def split(reader, line_count, suffix="%05d.pickle", dumper=pickle.dump):
    """Write the reader's samples into files of ``line_count`` samples each (names from ``suffix``)."""
    lines, idx = [], 0
    for s in reader():
        lines.append(s)
        if len(lines) >= line_count:
            with open(suffix % idx, "wb") as f:
                dumper(lines, f)
            lines, idx = [], idx + 1
    if lines:
        with open(suffix % idx, "wb") as f:
            dumper(lines, f)


def cluster_files_reader(files_pattern, trainer_count, trainer_id, loader=None):
    """Reader over this trainer's share (round-robin) of the files matching ``files_pattern``; ``loader`` reads
    one file into a list of samples (the caller's own files: use a safe loader, e.g. json / numpy)."""
    if loader is None:
        raise ValueError("cluster_files_reader needs an explicit loader (no implicit unpickling)")

    def r():
        files = sorted(glob.glob(files_pattern))
        for i, fn in enumerate(files):
            if i % trainer_count == trainer_id:
                with open(fn, "rb") as f:
                    yield from loader(f)

    return r
