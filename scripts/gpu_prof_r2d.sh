#!/bin/bash
# rocprofv3 kernel-trace profile of the default bench (Llama-2-7B b=8 s=4096, stage-3 sharding, native wgrad
# GEMMs), 1 warmup + 2 timed steps; plus an un-profiled 10-step bench of the same tree.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2d -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 > gpurun_out/r2d_bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/r2d_bench_prof.log
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY' > gpurun_out/r2d_top_kernels.txt
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_r2d/run_kernel_stats.csv")))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over 3 steps (incl. init)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:45]:
    print(f"{float(r['TotalDurationNs'])/3e6:8.2f} ms/step {int(r['Calls'])/3:7.1f} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
cat gpurun_out/r2d_top_kernels.txt | head -30
