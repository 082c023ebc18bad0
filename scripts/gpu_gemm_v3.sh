set -o pipefail
cd /root/repo
timeout -k 10 180 python -u scripts/check_gemm_v3.py > gpurun_out/v3_check.log 2>&1 || { echo CHECK_FAILED; tail -20 gpurun_out/v3_check.log; exit 1; }
tail -4 gpurun_out/v3_check.log
timeout -k 10 240 python -u scripts/bench_gemm_native.py 32768 0,3 > gpurun_out/v3_bench.jsonl 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/v3_bench.jsonl; exit 1; }
cat gpurun_out/v3_bench.jsonl
