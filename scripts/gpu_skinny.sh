#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/skinny
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/bench_skinny_gemm.py > gpurun_out/skinny/gemm.jsonl 2> gpurun_out/skinny/err.log
rc=$?; cat gpurun_out/skinny/gemm.jsonl; tail -3 gpurun_out/skinny/err.log; exit $rc
