#!/bin/bash
# quick GPU check of selected test files: bash scripts/gpu_quick.sh tests/a.py tests/b.py
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu "$@" > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -8 gpurun_out/quick_tests.log; echo "tests rc=$rc"; exit $rc
