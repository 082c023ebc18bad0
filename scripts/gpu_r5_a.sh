#!/bin/bash
# Round 5 (a): the new GPU tests (forced-comm stage 3, IPC capture guard, GELU double backward, comm context on
# ProcessGroupRCCL), then the 7B bench with the N > 1 stage-3 path forced on one GPU vs the default, and a
# kernel table of the forced-comm step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5a
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_stage3_force_comm.py tests/test_ipc_allreduce.py tests/test_fused_act.py tests/test_comm_context_gpu.py \
  tests/test_native_pg_gpu.py > $O/tests.log 2>&1
r=$?; tail -3 $O/tests.log; [ $r -ne 0 ] && { grep -E "FAIL|Error" $O/tests.log | head -20; exit $r; }
PADDLE2_AMD_STAGE3_FORCE_COMM=1 timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_force.log 2>&1
r=$?; tail -2 $O/bench_force.log; [ $r -ne 0 ] && { tail -30 $O/bench_force.log; exit $r; }
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_plain.log 2>&1
r=$?; tail -2 $O/bench_plain.log; [ $r -ne 0 ] && { tail -30 $O/bench_plain.log; exit $r; }
PADDLE2_AMD_STAGE3_FORCE_COMM=1 timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_force -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof_force.log 2>&1
r=$?; echo "prof rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_force.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_force -name "*kernel_trace.csv" | head -1) > $O/kernels_force.txt 2>&1; head -40 $O/kernels_force.txt
rm -rf $O/prof_force/*/*.csv.gz 2>/dev/null
exit 0
