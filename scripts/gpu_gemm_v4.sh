set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/check_gemm_variant.py 4 > gpurun_out/v4_check.log 2>&1 || { echo CHECK_FAILED; tail -30 gpurun_out/v4_check.log; exit 1; }
tail -8 gpurun_out/v4_check.log
timeout -k 10 300 python -u scripts/bench_gemm_native.py 32768 0,4 > gpurun_out/v4_bench.jsonl 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/v4_bench.jsonl; exit 1; }
cat gpurun_out/v4_bench.jsonl
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_ipc_allreduce.py -m gpu > gpurun_out/ipc_tests.log 2>&1 || { echo IPC_FAILED; tail -30 gpurun_out/ipc_tests.log; exit 1; }
tail -5 gpurun_out/ipc_tests.log
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_native_allocator.py -m gpu > gpurun_out/alloc_tests.log 2>&1 || { echo ALLOC_FAILED; tail -30 gpurun_out/alloc_tests.log; exit 1; }
tail -5 gpurun_out/alloc_tests.log
