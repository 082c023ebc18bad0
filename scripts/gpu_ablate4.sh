set -o pipefail
cd /root/repo
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/exp_gemm_ablate_v4.py 4096 > gpurun_out/ablate4_k4096.jsonl 2>&1 || { echo FAILED; tail gpurun_out/ablate4_k4096.jsonl; exit 1; }
timeout -k 10 200 python -u scripts/exp_gemm_ablate_v4.py 12288 > gpurun_out/ablate4_k12288.jsonl 2>&1 || { echo FAILED; tail gpurun_out/ablate4_k12288.jsonl; exit 1; }
cat gpurun_out/ablate4_k4096.jsonl gpurun_out/ablate4_k12288.jsonl
