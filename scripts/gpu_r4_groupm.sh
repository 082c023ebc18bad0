#!/bin/bash
# Llama-2-7B step: tile-group height of the forward / SwiGLU / dgrad passes (2 vs the default 4).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4gm
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/base.log 2>&1
rc=$?; echo "base rc=$rc"; grep '"metric"' $O/base.log | cut -c80-200; [ $rc -ne 0 ] && exit $rc
PADDLE2_AMD_GEMM_GROUP_M_FWD=2 PADDLE2_AMD_GEMM_GROUP_M_SWIGLU=2 timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/fwd2.log 2>&1
rc=$?; echo "fwd/swiglu gm2 rc=$rc"; grep '"metric"' $O/fwd2.log | cut -c80-200; [ $rc -ne 0 ] && exit $rc
PADDLE2_AMD_GEMM_GROUP_M_FWD=2 PADDLE2_AMD_GEMM_GROUP_M_SWIGLU=2 PADDLE2_AMD_GEMM_GROUP_M_DGRAD=2 timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/all2.log 2>&1
rc=$?; echo "fwd/swiglu/dgrad gm2 rc=$rc"; grep '"metric"' $O/all2.log | cut -c80-200; [ $rc -ne 0 ] && exit $rc
PADDLE2_AMD_GEMM_GROUP_M_WGRAD=4 timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/wg4.log 2>&1
rc=$?; echo "wgrad gm4 rc=$rc"; grep '"metric"' $O/wg4.log | cut -c80-200; [ $rc -ne 0 ] && exit $rc
PADDLE2_AMD_GEMM_GROUP_M_WGRAD=16 timeout -k 10 420 python3 -u bench.py --steps 10 --warmup 3 > $O/wg16.log 2>&1
rc=$?; echo "wgrad gm16 rc=$rc"; grep '"metric"' $O/wg16.log | cut -c80-200; [ $rc -ne 0 ] && exit $rc
exit 0
