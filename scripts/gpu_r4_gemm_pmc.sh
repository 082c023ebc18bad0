#!/bin/bash
# Round 4: counter passes on the qkv dgrad (both operands K-major) for v7 SCHED 2 (variant 9), v6 and hipBLASLt.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4pmc
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
for impl in 9 6 blas; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT -d $O/p1_$impl -o run --output-format csv -- python3 scripts/prof_gemm_cmp.py dgrad 4096 12288 6 $impl > $O/p1_$impl.log 2>&1
  rc=$?; echo "p1 $impl rc=$rc"; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUFFER_LOAD_WAVEFRONTS_sum SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA -d $O/p2_$impl -o run --output-format csv -- python3 scripts/prof_gemm_cmp.py dgrad 4096 12288 6 $impl > $O/p2_$impl.log 2>&1
  rc=$?; echo "p2 $impl rc=$rc"; [ $rc -eq 124 -o $rc -eq 137 -o $rc -eq 134 -o $rc -eq 139 ] && exit $rc
done
echo done
