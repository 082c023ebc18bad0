#!/bin/bash
# Counter comparison v4 vs hipBLASLt on the qkv dgrad (both K-major) and fwd shapes.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/gprof4
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for impl in 4 blas; do
for ps in dgrad fwd; do
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/${ps}_${impl}_a -o run --output-format csv -- python3 scripts/prof_gemm_cmp.py $ps 4096 12288 6 $impl > $O/${ps}_${impl}_a.log 2>&1 || { echo "FAIL $ps $impl a"; exit 1; }
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_MFMA -d $O/${ps}_${impl}_b -o run --output-format csv -- python3 scripts/prof_gemm_cmp.py $ps 4096 12288 6 $impl > $O/${ps}_${impl}_b.log 2>&1 || echo "FAIL(b) $ps $impl"
echo "$ps $impl done"
done
done
