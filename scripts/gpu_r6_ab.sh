#!/bin/bash
# Round 6 (ab): the delta pass's slab zeroing with streaming stores — flash dQ tests and the Llama step kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ab
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_flash_gpu.py tests/test_flash_dq_modes_gpu.py tests/test_rope_fold_gpu.py > $O/tests.log 2>&1
r=$?; tail -1 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_7b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof_7b.log 2>&1
r=$?; echo "prof 7b rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_7b.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_7b -name "*kernel_trace.csv" | head -1) > $O/kernels_7b.txt 2>&1; head -18 $O/kernels_7b.txt
rm -f $(find $O/prof_7b -name "*kernel_trace.csv") 2>/dev/null
exit 0
