"""paddle.utils.download (reference: python/paddle/utils/download.py).  There is no network on the MI355X hosts
this framework targets by default: ``get_path_from_url`` resolves a URL to its cache path under ``root_dir``
(``WEIGHTS_HOME`` for weights), decompressing archives already placed there, and raises a clear error when the
file is missing instead of downloading it.  An md5 check applies when ``md5sum`` is given."""
from __future__ import annotations

import hashlib
import os
import os.path as osp
import tarfile
import zipfile

__all__ = ["get_weights_path_from_url", "get_path_from_url", "is_url", "WEIGHTS_HOME"]

WEIGHTS_HOME = osp.expanduser(os.environ.get("PADDLE_WEIGHTS_HOME", "~/.cache/paddle/hapi/weights"))


def is_url(path):
    return path.startswith("http://") or path.startswith("https://")


def _map_path(url, root_dir):
    return osp.join(root_dir, osp.split(url)[-1])


def _md5check(fullname, md5sum=None):
    if md5sum is None:
        return True
    h = hashlib.md5()
    with open(fullname, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 20), b""):
            h.update(chunk)
    return h.hexdigest() == md5sum


def _decompress(fname):
    """Extract a .tar(.gz)/.tgz/.zip next to itself; -> the extracted top-level path."""
    root = osp.dirname(fname)
    if tarfile.is_tarfile(fname):
        with tarfile.open(fname) as tf:
            names = tf.getnames()
            tf.extractall(root, filter="data")
    elif zipfile.is_zipfile(fname):
        with zipfile.ZipFile(fname) as zf:
            names = zf.namelist()
            zf.extractall(root)
    else:
        raise TypeError(f"unsupported archive {fname}")
    tops = {n.split("/")[0] for n in names}
    return osp.join(root, tops.pop()) if len(tops) == 1 else root


def get_path_from_url(url, root_dir, md5sum=None, check_exist=True, decompress=True, method="get"):
    if not is_url(url):
        raise ValueError(f"{url} is not a URL")
    fullpath = _map_path(url, root_dir)
    if not osp.exists(fullpath):
        raise FileNotFoundError(
            f"{fullpath} is not present and downloads are disabled here; place the file from {url} there")
    if not _md5check(fullpath, md5sum):
        raise OSError(f"md5 mismatch for {fullpath}")
    if decompress and (tarfile.is_tarfile(fullpath) or zipfile.is_zipfile(fullpath)):
        return _decompress(fullpath)
    return fullpath


def get_weights_path_from_url(url, md5sum=None):
    return get_path_from_url(url, WEIGHTS_HOME, md5sum, decompress=False)
