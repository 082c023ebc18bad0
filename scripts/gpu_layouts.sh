#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/bench_wgrad_splitk.py > gpurun_out/layouts.log 2>&1
rc=$?; cat gpurun_out/layouts.log | grep -v amdgpu.ids; exit $rc
