#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_ipc_allreduce.py \
  > gpurun_out/ipc_tests.log 2>&1
rc=$?; tail -6 gpurun_out/ipc_tests.log; echo "tests rc=$rc"; exit $rc
