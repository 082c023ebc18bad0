#!/bin/bash
# flash attention coverage (fp16, D=256/padded, S=4096/8192) + the existing kernel suite's flash tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_flash_gpu.py \
  tests/test_kernels_gpu.py -k "flash" > gpurun_out/flash_tests.log 2>&1
rc=$?
tail -5 gpurun_out/flash_tests.log
echo "tests rc=$rc"
exit $rc
