set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_gpu.py > gpurun_out/gemm_tests.log 2>&1 || { echo GEMM_TESTS_FAILED; tail -30 gpurun_out/gemm_tests.log; exit 1; }
tail -3 gpurun_out/gemm_tests.log
timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench_mixed.log 2>&1 || { echo BENCH_MIXED_FAILED; tail -20 gpurun_out/bench_mixed.log; exit 1; }
tail -1 gpurun_out/bench_mixed.log
PADDLE2_AMD_GEMM_FWD=native PADDLE2_AMD_GEMM_DGRAD=native timeout -k 10 420 python -u bench.py --steps 6 --warmup 2 > gpurun_out/bench_native.log 2>&1 || { echo BENCH_NATIVE_FAILED; tail -20 gpurun_out/bench_native.log; exit 1; }
tail -1 gpurun_out/bench_native.log
