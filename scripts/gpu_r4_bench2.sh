#!/bin/bash
# Round 4: SwiGLU-backward-in-dgrad MLP node — GPU tests, then the Llama-2-7B step with the node on / off and the
# rocprofv3 kernel table of the default.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4bench2
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_gpu.py -x -q -k "dswiglu or swiglu_mlp or rope" --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python3 -u scripts/bench_swiglu_groupm.py > $O/swiglu_groupm.jsonl 2> $O/swiglu_groupm.err
echo "swiglu group_m rc=$?"; cat $O/swiglu_groupm.jsonl
timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '"metric"' $O/bench.log | cut -c1-200; [ $rc -ne 0 ] && { tail -30 $O/bench.log; exit $rc; }
PADDLE2_AMD_SWIGLU_MLP_NODE=0 timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/bench_nomlp.log 2>&1
rc=$?; echo "bench mlp-node-off rc=$rc"; grep '"metric"' $O/bench_nomlp.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/kernel_table.py $(find $O/prof -name "*kernel_trace.csv" | head -1) > $O/kernels.txt 2>&1; head -24 $O/kernels.txt
exit 0
