set -o pipefail
cd /root/repo
timeout -k 10 120 env PADDLE2_AMD_FA_DQ_ATOMIC=0 FA_DUMP=gpurun_out/fa_ref.pt python -u scripts/bench_flash_bwd.py > gpurun_out/fa_atomic2.log 2>&1
timeout -k 10 120 env PADDLE2_AMD_FA_DQ_ATOMIC=1 FA_REF=gpurun_out/fa_ref.pt python -u scripts/bench_flash_bwd.py >> gpurun_out/fa_atomic2.log 2>&1
rm -f gpurun_out/fa_ref.pt
grep -v amdgpu.ids gpurun_out/fa_atomic2.log
timeout -k 10 300 python -u -m pytest tests -m gpu -q -x -k "flash or attn or attention" --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
