#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fskip
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/bench_flash_fwd.py > gpurun_out/fskip/fwd.jsonl 2> gpurun_out/fskip/err.log
rc=$?; cat gpurun_out/fskip/fwd.jsonl; tail -3 gpurun_out/fskip/err.log; exit $rc
