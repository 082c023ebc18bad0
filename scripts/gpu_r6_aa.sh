#!/bin/bash
# Round 6 (aa): dQ slab zeroing folded into the flash backward's delta pass — flash GPU tests, the bwd timing at the
# Llama shape, and the Llama step (bench + kernel table).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6aa
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_flash_gpu.py tests/test_flash_ext_gpu.py tests/test_flash_dq_modes_gpu.py tests/test_flash_dq_split_gpu.py tests/test_flash_fwd_rb2_gpu.py tests/test_rope_fold_gpu.py tests/test_mem_eff_attention.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL|Error" $O/tests.log | head -30; exit $r; }
timeout -k 10 300 python -u scripts/exp_flash_bwd_opt.py > $O/bwd.jsonl 2> $O/bwd.err
r=$?; head -1 $O/bwd.jsonl; [ $r -ne 0 ] && { tail -10 $O/bwd.err; exit $r; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1
r=$?; tail -1 $O/bench.log | cut -c1-200; [ $r -ne 0 ] && { tail -30 $O/bench.log; exit $r; }
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_7b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof_7b.log 2>&1
r=$?; echo "prof 7b rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_7b.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_7b -name "*kernel_trace.csv" | head -1) > $O/kernels_7b.txt 2>&1; head -22 $O/kernels_7b.txt
rm -f $(find $O/prof_7b -name "*kernel_trace.csv") 2>/dev/null
exit 0
