#!/bin/bash
# Round 4: the Llama-2-7B step (bench.py, 1 GPU) with the new default routes, the RoPE-in-GEMM / RoPE^T-in-flash
# on / off comparison and the rocprofv3 kernel table.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4bench
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '"metric"' $O/bench.log | cut -c1-250; [ $rc -ne 0 ] && { tail -30 $O/bench.log; exit $rc; }
PADDLE2_AMD_ROPE_IN_GEMM=0 timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/bench_norope.log 2>&1
rc=$?; echo "bench no-rope-fusion rc=$rc"; grep '"metric"' $O/bench_norope.log | cut -c1-250; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/kernel_table.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kernels.txt 2>&1; head -45 $O/kernels.txt
exit 0
