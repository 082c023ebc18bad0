"""fleet.utils: pipeline-agnostic PipelineLayer checkpoints + offline pp re-partitioning (pp_parallel_adaptor),
DistributedLogger / rotate logger / check_memory_usage (reference: fleet/utils/pp_parallel_adaptor.py,
log_util.py)."""
import logging
import pytest
import os

import torch

import paddle2_amd as paddle
from paddle2_amd.distributed.fleet.meta_parallel.parallel_layers.pp_layers import LayerDesc, PipelineLayer
from paddle2_amd.distributed.fleet.utils import log_util
from paddle2_amd.distributed.fleet.utils.pp_parallel_adaptor import ParallelConfig, PipeLineModelAdaptor


class _Emb(paddle.nn.Layer):
    def __init__(self):
        super().__init__()
        self.w = paddle.nn.Linear(4, 8)

    def forward(self, x):
        return self.w(x)


def _descs(n_blocks):
    return [LayerDesc(_Emb)] + [LayerDesc(paddle.nn.Linear, 8, 8) for _ in range(n_blocks)] + \
        [LayerDesc(paddle.nn.Linear, 8, 2)]


def test_pp_adaptor_resplits_and_preserves(tmp_path):
    paddle.seed(0)
    n = 6
    full = PipelineLayer(_descs(n), num_stages=1)
    gsd = full.global_state_dict()
    assert all(k.startswith("layers.") for k in gsd)
    # write a pp=2 source checkpoint by splitting the global dict with the adaptor's own segmentation
    src = ParallelConfig(mp=1, pp=2)
    ad = PipeLineModelAdaptor(src, src, transformer_layer_num=n)
    ids = sorted({int(k.split(".")[1]) for k in gsd})
    for k, seg in enumerate(ad.segment(ids, 2)):
        d = tmp_path / "src" / f"mp_00_sharding_00_pp_{k:02d}"
        os.makedirs(d)
        paddle.save({kk: v for kk, v in gsd.items() if int(kk.split(".")[1]) in seg}, str(d / "model.pdparams"))
    for dst_pp in (4, 1):
        dst = ParallelConfig(mp=1, pp=dst_pp)
        PipeLineModelAdaptor(src, dst, transformer_layer_num=n).apply(str(tmp_path / "src"),
                                                                      str(tmp_path / f"dst{dst_pp}"))
        merged = {}
        for k in range(dst_pp):
            merged.update(paddle.load(str(tmp_path / f"dst{dst_pp}" / f"mp_00_sharding_00_pp_{k:02d}" / "model.pdparams")))
        assert merged.keys() == gsd.keys()
        for kk in gsd:
            assert torch.equal(merged[kk]._t, gsd[kk]._t)
    # a fresh model loads the merged global dict and reproduces the original outputs
    other = PipelineLayer(_descs(n), num_stages=1)
    other.set_global_state_dict(merged)
    x = paddle.randn([3, 4])
    torch.testing.assert_close(other(x)._t, full(x)._t)


def test_stage_balance_keeps_extras_at_ends():
    ad = PipeLineModelAdaptor(ParallelConfig(1, 2), ParallelConfig(1, 4), transformer_layer_num=8)
    segs = ad.segment(range(10), 4)  # 1 embedding + 8 blocks + 1 head
    assert segs[0][0] == 0 and segs[-1][-1] == 9 and [len(s) for s in segs] == [3, 2, 2, 3]


def test_distributed_logger_and_memory(tmp_path, monkeypatch, caplog):
    monkeypatch.chdir(tmp_path)
    lg = log_util.get_rotate_file_logger("INFO", "t")
    monkeypatch.setenv("FLAGS_distributed_debug_logger", "1")
    lg.info("hello")
    for h in lg.handlers:
        h.flush()
    text = (tmp_path / "hybrid_parallel" / "worker_0.log").read_text()
    assert "Distributed Debug" in text and "hello" in text
    monkeypatch.setenv("FLAGS_distributed_debug_logger", "0")
    lg.info("quiet")
    assert "quiet" not in (tmp_path / "hybrid_parallel" / "worker_0.log").read_text()
    with caplog.at_level(logging.INFO, logger="paddle2_amd.fleet"):
        out = log_util.check_memory_usage("step 1")
    assert "host_rss_size" in out and out["host_rss_size"] > 0


_FAKE_HADOOP = r"""#!/bin/bash
# minimal `hadoop fs` emulation over $FAKE_HDFS_ROOT (test double for HDFSClient)
R="$FAKE_HDFS_ROOT"
shift  # "fs"
while [ "$1" = "-D" ]; do shift 2; done
op="$1"; shift
case "$op" in
  -ls) p="$R$1"; [ -e "$p" ] || exit 1
       for f in "$p"/*; do [ -e "$f" ] || continue
         if [ -d "$f" ]; then t=drwxr-xr-x; s=0; else t=-rw-r--r--; s=$(stat -c %s "$f"); fi
         echo "$t   - u g $s 2024-01-01 00:00 ${f#$R}"; done ;;
  -test) flag="$1"; p="$R$2"; [ $flag "$p" ] ;;
  -mkdir) [ "$1" = "-p" ] && shift; mkdir -p "$R$1" ;;
  -put) cp -r "$1" "$R$2" ;;
  -get) cp -r "$R$1" "$2" ;;
  -mv) mv "$R$1" "$R$2" ;;
  -rmr) rm -rf "$R$1" ;;
  -rm) rm -f "$R$1" ;;
  -touchz) touch "$R$1" ;;
  -cat) cat "$R$1" ;;
  *) exit 2 ;;
esac
"""


def test_hdfs_client_over_cli(tmp_path, monkeypatch):
    from paddle2_amd.distributed.fleet.utils.fs import FSFileExistsError, HDFSClient

    home = tmp_path / "hadoop"
    (home / "bin").mkdir(parents=True)
    exe = home / "bin" / "hadoop"
    exe.write_text(_FAKE_HADOOP)
    exe.chmod(0o755)
    root = tmp_path / "hdfs"
    root.mkdir()
    monkeypatch.setenv("FAKE_HDFS_ROOT", str(root))
    fs = HDFSClient(str(home), {"fs.default.name": "hdfs://x", "hadoop.job.ugi": "u,p"}, sleep_inter=10)
    fs.mkdirs("/a/b")
    assert fs.is_dir("/a/b") and fs.is_exist("/a") and not fs.is_file("/a")
    local = tmp_path / "f.txt"
    local.write_text("hello\nworld")
    fs.upload(str(local), "/a/b/f.txt")
    assert fs.is_file("/a/b/f.txt") and fs.cat("/a/b/f.txt") == "hello\nworld"
    with pytest.raises(FSFileExistsError):
        fs.upload(str(local), "/a/b/f.txt")
    fs.touch("/a/b/g")
    dirs, files = fs.ls_dir("/a/b")
    assert dirs == [] and sorted(files) == ["f.txt", "g"]
    assert fs.list_dirs("/a") == ["b"]
    fs.mv("/a/b/g", "/a/h")
    assert fs.is_file("/a/h") and not fs.is_exist("/a/b/g")
    fs.download("/a/b/f.txt", str(tmp_path / "back.txt"))
    assert (tmp_path / "back.txt").read_text() == "hello\nworld"
    info = fs.list_files_info(["/a/b"])
    assert info[0]["size"] == len("hello\nworld")
    fs.delete("/a")
    assert not fs.is_exist("/a")
    assert fs._split_files(list(range(10)), 1, 3) == [4, 5, 6]
