#!/bin/bash
# Re-measure the headline bench on the current tree (caching vs native allocator) and take a fresh
# rocprofv3 kernel-stats profile of the default configuration.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2c_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r2c_bench.log
[ $rc -eq 0 ] || exit $rc
FLAGS_use_native_allocator=1 timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/r2c_bench_nativealloc.log 2>&1
rc=$?; echo "bench(native alloc) rc=$rc"; tail -1 gpurun_out/r2c_bench_nativealloc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2c -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 > gpurun_out/r2c_bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/r2c_bench_prof.log
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY' > gpurun_out/r2c_top_kernels.txt
import csv
rows = list(csv.DictReader(open("gpurun_out/prof_r2c/run_kernel_stats.csv")))
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms over 3 steps (incl. init)")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:45]:
    print(f"{float(r['TotalDurationNs'])/3e6:8.2f} ms/step {int(r['Calls'])/3:7.1f} calls {float(r['AverageNs'])/1e3:9.1f} us  {r['Name'][:110]}")
PY
head -30 gpurun_out/r2c_top_kernels.txt
