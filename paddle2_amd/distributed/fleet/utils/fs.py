"""File-system clients (reference: fleet/utils/fs.py — ``LocalFS``; ``HDFSClient`` shells out to
``hadoop fs``, which is unavailable here and raises on use)."""
from __future__ import annotations

import os
import shutil


class FSFileExistsError(Exception):
    pass


class FSFileNotExistsError(Exception):
    pass


class FS:
    pass


class LocalFS(FS):
    def ls_dir(self, fs_path):
        if not self.is_exist(fs_path):
            return [], []
        dirs, files = [], []
        for f in os.listdir(fs_path):
            (dirs if os.path.isdir(os.path.join(fs_path, f)) else files).append(f)
        return dirs, files

    def mkdirs(self, fs_path):
        assert not os.path.isfile(fs_path), f"{fs_path} is already a file"
        os.makedirs(fs_path, exist_ok=True)

    def rename(self, fs_src_path, fs_dst_path):
        os.rename(fs_src_path, fs_dst_path)

    def _rmr(self, fs_path):
        shutil.rmtree(fs_path)

    def _rm(self, fs_path):
        os.remove(fs_path)

    def delete(self, fs_path):
        if not self.is_exist(fs_path):
            return
        if os.path.isfile(fs_path):
            return self._rm(fs_path)
        return self._rmr(fs_path)

    def need_upload_download(self):
        return False

    def is_file(self, fs_path):
        return os.path.isfile(fs_path)

    def is_dir(self, fs_path):
        return os.path.isdir(fs_path)

    def is_exist(self, fs_path):
        return os.path.exists(fs_path)

    def touch(self, fs_path, exist_ok=True):
        if self.is_exist(fs_path):
            if exist_ok:
                return
            raise FSFileExistsError(fs_path)
        open(fs_path, "a").close()

    def mv(self, src_path, dst_path, overwrite=False, test_exists=False):
        if not self.is_exist(src_path):
            raise FSFileNotExistsError(src_path)
        if overwrite and self.is_exist(dst_path):
            self.delete(dst_path)
        if self.is_exist(dst_path):
            raise FSFileExistsError(dst_path)
        return self.rename(src_path, dst_path)

    def list_dirs(self, fs_path):
        return self.ls_dir(fs_path)[0]

    def cat(self, fs_path=None):
        with open(fs_path) as f:
            return f.read()

    def upload(self, local_path, fs_path):
        shutil.copy(local_path, fs_path) if os.path.isfile(local_path) else shutil.copytree(local_path, fs_path)

    download = upload


class HDFSClient(FS):
    def __init__(self, hadoop_home=None, configs=None, time_out=300000, sleep_inter=1000):
        self._home = hadoop_home

    def __getattr__(self, name):
        def fail(*a, **k):
            raise RuntimeError("HDFSClient needs a hadoop installation, which is not available on this system")

        return fail
