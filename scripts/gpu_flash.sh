cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_flash_ext_gpu.py tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_fa.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" gpurun_out/pytest_fa.log | tail -15
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/bench_flash.py > gpurun_out/bench_flash.log 2>&1
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_flash.log | tail -8
exit $rc
