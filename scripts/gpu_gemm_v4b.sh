set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 240 python -u scripts/check_gemm_variant.py 6 > gpurun_out/v4_check.log 2>&1 || { echo CHECK_FAILED; tail -30 gpurun_out/v4_check.log; exit 1; }
tail -3 gpurun_out/v4_check.log
timeout -k 10 300 python -u scripts/bench_gemm_native.py 32768 4,6 > gpurun_out/v4_bench.jsonl 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/v4_bench.jsonl; exit 1; }
cat gpurun_out/v4_bench.jsonl
