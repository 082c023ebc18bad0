#!/bin/bash
# GPU tests + rocprofv3 kernel profile of the 7B step + batch sweep. Stops at the first fault.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
    python bench.py --steps 2 --warmup 1 --micro-batch 2 > gpurun_out/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/bench_prof.log
ok $rc || exit $rc
for b in 2 4; do
  timeout -k 10 900 python bench.py --steps 4 --warmup 2 --micro-batch $b > gpurun_out/bench_b$b.log 2>&1
  rc=$?; echo "bench b$b rc=$rc"; tail -2 gpurun_out/bench_b$b.log
  ok $rc || exit $rc
done
python - <<'PY' > gpurun_out/top_kernels.txt
import csv
rows = list(csv.DictReader(open("gpurun_out/prof/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    print(f"{float(r['TotalDurationNs'])/3e6:8.2f} ms/step {int(r['Calls'])/3:7.1f} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:100]}")
PY
