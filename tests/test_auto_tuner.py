"""Auto tuner (reference tests: test/auto_tuner/ — prune rules, search, recorder) incl. the
launcher integration with a real trial script."""
import json
import os
import subprocess
import sys

from paddle2_amd.distributed.auto_tuner import AutoTuner, HistoryRecorder, estimate_memory_gb
from paddle2_amd.distributed.auto_tuner.launch import read_metric_log, run

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLAMA7B = {"hidden_size": 4096, "num_layers": 32, "num_attention_heads": 32, "vocab_size": 32000,
           "seq_length": 4096, "global_batch_size": 64, "intermediate_size": 11008}


def test_prune_and_order():
    cfg = {"num_gpus": 8, "gpus_per_node": 8, "model_cfg": dict(LLAMA7B, num_attention_heads=12)}
    t = AutoTuner(cfg)
    for c in t.algo.all_tasks:
        assert c["dp_degree"] * c["mp_degree"] * c["pp_degree"] * c["sharding_degree"] == 8
        assert 12 % c["mp_degree"] == 0 and 32 % c["pp_degree"] == 0
        assert c["estimated_memory_gb"] <= 288 * 0.92
    est = [c["estimated_step_time_s"] for c in t.algo.all_tasks]
    assert est == sorted(est)
    # stage 3 sharding needs less memory than stage 1 which needs less than pure dp
    m = LLAMA7B
    assert estimate_memory_gb(m, {"sharding_degree": 8, "sharding_stage": 3}) < \
        estimate_memory_gb(m, {"sharding_degree": 8, "sharding_stage": 1}) < estimate_memory_gb(m, {})
    # calibrated against the measured 7B single-GPU step: 8 x 4096 tokens, 241 GB peak
    assert abs(estimate_memory_gb(m, {"micro_batch_size": 8}) - 241) < 15


def test_trials_record_best(tmp_path):
    cfg = {"num_gpus": 4, "model_cfg": dict(LLAMA7B, num_layers=8, global_batch_size=8), "task_limit": 6,
           "metric_cfg": {"name": "tokens_per_sec", "OptimizationDirection": "Maximize"}}

    def fake_runner(c, env, argv, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        tps = 1000 * c["micro_batch_size"] / c["mp_degree"] / c["pp_degree"]
        with open(os.path.join(log_dir, "workerlog.0"), "w") as f:
            f.write(json.dumps({"tokens_per_sec": tps}) + "\n")
        return 0

    best, tuner = run(cfg, [], "train.py", [], log_root=str(tmp_path), runner=fake_runner)
    assert best["tokens_per_sec"] == max(h["tokens_per_sec"] for h in tuner.recorder.history)
    assert os.path.exists(tmp_path / "history.csv") and os.path.exists(tmp_path / "best_cfg.json")
    rec = HistoryRecorder()
    hist, err = rec.load_history(str(tmp_path / "history.csv"))
    assert not err and len(hist) == 6


def test_read_metric_log(tmp_path):
    p = tmp_path / "log"
    p.write_text("step 1 interval_runtime: 2.0\nstep 2 interval_runtime: 1.5\n")
    assert read_metric_log(str(p), "interval_runtime") == (1.5, None)
    p.write_text("RuntimeError: HIP out of memory\n")
    assert read_metric_log(str(p), "interval_runtime")[1] == "OOM"


def test_launch_auto_tuner_end_to_end(tmp_path):
    script = tmp_path / "trial.py"
    script.write_text("import os\nmb = int(os.environ['PADDLE_AUTO_TUNER_MICRO_BATCH'])\n"
                      "print(f'step_time: {1.0 / mb}')\n")
    cfg = {"num_gpus": 1, "model_cfg": dict(LLAMA7B, num_layers=4, global_batch_size=4),
           "search_algo": {"name": "customize"},
           "configs": [{"dp_degree": 1, "mp_degree": 1, "pp_degree": 1, "sharding_degree": 1, "micro_batch_size": m}
                       for m in (1, 2, 4)],
           "metric_cfg": {"name": "step_time", "OptimizationDirection": "Minimize"}}
    cj = tmp_path / "tuner.json"
    cj.write_text(json.dumps(cfg))
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-m", "paddle2_amd.distributed.launch", "--auto_tuner_json", str(cj),
                        "--log_dir", str(tmp_path / "logs"), str(script)], env=env, cwd=ROOT, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    best = json.load(open(tmp_path / "logs" / "auto_tuner" / "best_cfg.json"))
    assert best["micro_batch_size"] == 4 and abs(best["step_time"] - 0.25) < 1e-9
