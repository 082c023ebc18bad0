#!/bin/bash
# rocprofv3 kernel trace of the bench (1 warmup + 2 steps); routing from the environment (GEMM pass backends).
# usage: gpu_prof_r3.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 > gpurun_out/${TAG}_bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -1 gpurun_out/${TAG}_bench_prof.log | cut -c1-300
[ $rc -eq 0 ] || exit $rc
python3 scripts/kernel_table.py gpurun_out/prof_$TAG/run_kernel_trace.csv > gpurun_out/${TAG}_kernels.txt
head -45 gpurun_out/${TAG}_kernels.txt
