#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/fmt
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_serving.py  \
> gpurun_out/fmt/tests.log 2>&1
rc=$?; tail -2 gpurun_out/fmt/tests.log; grep -E "FAILED|ERROR" gpurun_out/fmt/tests.log | head; exit $rc
