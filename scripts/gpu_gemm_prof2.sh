#!/bin/bash
# Counter comparison: dgrad (both K-major) vs wgrad (both MN-major) on 32768x4096x4096, + counter list.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gprof2
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/gprof2/counters.txt 2>&1; echo "list rc=$?"
for ps in dgrad wgrad fwd; do
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS -d gpurun_out/gprof2/$ps -o run --output-format csv -- python3 scripts/prof_gemm_one.py $ps 4096 4096 10 > gpurun_out/gprof2/$ps.log 2>&1
echo "$ps rc=$?"
done
