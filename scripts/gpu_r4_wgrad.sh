#!/bin/bash
# Round 4: GEMM GPU tests (incl. the GELU epilogues), the spread wgrad kernel (v5) bench, native 1x1 conv tests
# and the ResNet-50 step with 1x1 convs on MIOpen vs the native GEMM.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4wg
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python3 -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 $O/gemm_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python3 -u scripts/bench_gemm_wgrad.py > $O/bench.jsonl 2> $O/bench.err
echo "bench rc=$?"; cat $O/bench.jsonl
timeout -k 10 300 python3 -u -m pytest tests/test_conv1x1_gpu.py -x -q --timeout 120 --timeout-method thread > $O/conv_tests.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -3 $O/conv_tests.log; [ $rc -ne 0 ] && exit $rc
for m in miopen native; do
  PADDLE2_AMD_CONV1X1=$m timeout -k 10 300 python3 -u scripts/bench_resnet50.py --steps 20 --warmup 5 > $O/resnet_$m.log 2>&1
  rc=$?; echo "resnet $m rc=$rc"; tail -1 $O/resnet_$m.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_resnet -o run -- python3 scripts/bench_resnet50.py --steps 5 --warmup 3 > $O/prof_resnet.log 2>&1
echo "resnet prof rc=$?"
exit 0
