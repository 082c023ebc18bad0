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


class ExecuteError(Exception):
    pass


class FSTimeOut(Exception):
    pass


class HDFSClient(FS):
    """HDFS through the hadoop CLI (reference fleet/utils/fs.py HDFSClient): every call runs
    ``{hadoop_home}/bin/hadoop fs [-D k=v ...] -<cmd> <args>`` as an argument vector (no shell), retried up to
    ``retry_times`` with ``sleep_inter`` ms between attempts and bounded by ``time_out`` ms overall."""

    def __init__(self, hadoop_home=None, configs=None, time_out=5 * 60 * 1000, sleep_inter=1000):
        home = hadoop_home or os.environ.get("HADOOP_HOME", "")
        self._bin = os.path.join(home, "bin", "hadoop") if home else "hadoop"
        self._pre = [self._bin, "fs"]
        for k, v in (configs or {}).items():
            self._pre += ["-D", f"{k}={v}"]
        self._time_out = time_out
        self._sleep_inter = sleep_inter

    # ------------------------------------------------------------------ command plumbing
    def _run_cmd(self, cmd, retry_times=5, redirect_stderr=False):
        import subprocess
        import time

        argv = self._pre + ["-" + cmd[0]] + list(cmd[1:])
        deadline = time.time() + self._time_out / 1000.0
        ret, out = 1, ""
        for i in range(max(1, retry_times)):
            left = deadline - time.time()
            if left <= 0:
                raise FSTimeOut(" ".join(argv))
            try:
                r = subprocess.run(argv, capture_output=True, text=True, timeout=left)
            except subprocess.TimeoutExpired as e:
                raise FSTimeOut(" ".join(argv)) from e
            ret = r.returncode
            out = r.stdout + (r.stderr if redirect_stderr else "")
            if ret == 0:
                break
            if i + 1 < retry_times:
                time.sleep(self._sleep_inter / 1000.0)
        return ret, out.splitlines()

    # ------------------------------------------------------------------ queries
    def _ls(self, fs_path):
        if not self.is_exist(fs_path):
            return [], []
        ret, lines = self._run_cmd(["ls", fs_path])
        if ret != 0:
            raise ExecuteError(f"ls {fs_path}")
        dirs, files = [], []
        for ln in lines:
            parts = ln.split()
            if len(parts) < 8 or not parts[0][:1] in ("d", "-"):
                continue  # "Found N items" header
            name = os.path.basename(parts[-1].rstrip("/"))
            (dirs if parts[0].startswith("d") else files).append(name)
        return dirs, files

    def ls_dir(self, fs_path):
        return self._ls(fs_path)

    def list_dirs(self, fs_path):
        return self._ls(fs_path)[0]

    def _test(self, flag, fs_path):
        ret, _ = self._run_cmd(["test", flag, fs_path], retry_times=1, redirect_stderr=True)
        return ret == 0

    def is_exist(self, fs_path):
        return self._test("-e", fs_path)

    def is_dir(self, fs_path):
        return self._test("-d", fs_path)

    def is_file(self, fs_path):
        return self.is_exist(fs_path) and not self.is_dir(fs_path)

    def need_upload_download(self):
        return True

    # ------------------------------------------------------------------ mutations
    def mkdirs(self, fs_path):
        if self.is_exist(fs_path):
            return
        ret, _ = self._run_cmd(["mkdir", "-p", fs_path])
        if ret != 0:
            raise ExecuteError(f"mkdir -p {fs_path}")

    def upload(self, local_path, fs_path, multi_processes=1, overwrite=False):
        if not os.path.exists(local_path):
            raise FSFileNotExistsError(local_path)
        if self.is_exist(fs_path):
            if not overwrite:
                raise FSFileExistsError(fs_path)
            self.delete(fs_path)
        ret, _ = self._run_cmd(["put", local_path, fs_path])
        if ret != 0:
            raise ExecuteError(f"put {local_path} {fs_path}")

    def upload_dir(self, local_dir, dest_dir, overwrite=False):
        self.upload(local_dir, dest_dir, overwrite=overwrite)

    def download(self, fs_path, local_path, multi_processes=1, overwrite=False):
        if not self.is_exist(fs_path):
            raise FSFileNotExistsError(fs_path)
        if os.path.exists(local_path):
            if not overwrite:
                raise FSFileExistsError(local_path)
            shutil.rmtree(local_path) if os.path.isdir(local_path) else os.remove(local_path)
        ret, _ = self._run_cmd(["get", fs_path, local_path])
        if ret != 0:
            raise ExecuteError(f"get {fs_path} {local_path}")

    def mv(self, fs_src_path, fs_dst_path, overwrite=False, test_exists=True):
        if test_exists and not self.is_exist(fs_src_path):
            raise FSFileNotExistsError(fs_src_path)
        if self.is_exist(fs_dst_path):
            if not overwrite:
                raise FSFileExistsError(fs_dst_path)
            self.delete(fs_dst_path)
        ret, _ = self._run_cmd(["mv", fs_src_path, fs_dst_path], retry_times=1)
        if ret != 0:
            raise ExecuteError(f"mv {fs_src_path} {fs_dst_path}")

    rename = mv

    def delete(self, fs_path):
        if not self.is_exist(fs_path):
            return
        ret, _ = self._run_cmd(["rmr" if self.is_dir(fs_path) else "rm", fs_path])
        if ret != 0:
            raise ExecuteError(f"delete {fs_path}")

    def touch(self, fs_path, exist_ok=True):
        if self.is_exist(fs_path):
            if exist_ok:
                return
            raise FSFileExistsError(fs_path)
        ret, _ = self._run_cmd(["touchz", fs_path])
        if ret != 0:
            raise ExecuteError(f"touchz {fs_path}")

    def cat(self, fs_path=None):
        if not self.is_file(fs_path):
            return ""
        ret, lines = self._run_cmd(["cat", fs_path], retry_times=1)
        if ret != 0:
            raise ExecuteError(f"cat {fs_path}")
        return "\n".join(lines)

    def _split_files(self, files, trainer_id, trainers):
        """Contiguous share of ``files`` for ``trainer_id`` of ``trainers`` (remainder to the first ones)."""
        n = len(files)
        per, extra = divmod(n, trainers)
        start = trainer_id * per + min(trainer_id, extra)
        return files[start:start + per + (1 if trainer_id < extra else 0)]

    def list_files_info(self, path_list):
        out = []
        for p in path_list:
            ret, lines = self._run_cmd(["ls", p])
            for ln in lines:
                parts = ln.split()
                if len(parts) >= 8 and parts[0].startswith("-"):
                    out.append({"path": parts[-1], "size": int(parts[4])})
        return out
