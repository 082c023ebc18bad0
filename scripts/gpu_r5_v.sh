#!/bin/bash
# Round 5 (v): the gate|up forward as the fused SwiGLU-epilogue GEMM vs plain GEMM + SwiGLU pass
# (PADDLE2_AMD_SWIGLU_FWD=split) — Llama GPU numerics under split, then both 7B benches on one box and the split
# step's kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5v
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
PADDLE2_AMD_SWIGLU_FWD=split timeout -k 10 400 python -u -m pytest -x -q --timeout 240 --timeout-method thread \
  -p no:cacheprovider -m gpu tests/test_llama_gpu.py tests/test_kernels_gpu.py > $O/tests.log 2>&1
r=$?; tail -2 $O/tests.log; [ $r -ne 0 ] && { grep -E "^E |FAIL" $O/tests.log | head -30; exit $r; }
for v in fused split fused split; do
  PADDLE2_AMD_SWIGLU_FWD=$v timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > $O/bench_$v.log 2>&1
  r=$?; echo "$v: $(tail -1 $O/bench_$v.log | cut -c1-200)"; [ $r -ne 0 ] && { tail -30 $O/bench_$v.log; exit $r; }
done
PADDLE2_AMD_SWIGLU_FWD=split timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_7b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof_7b.log 2>&1
r=$?; echo "prof 7b rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_7b.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_7b -name "*kernel_trace.csv" | head -1) > $O/kernels_7b.txt 2>&1; head -22 $O/kernels_7b.txt
rm -f $(find $O/prof_7b -name "*kernel_trace.csv") 2>/dev/null
exit 0
