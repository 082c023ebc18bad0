#!/bin/bash
# Counter passes on the native GEMM (o_proj-shaped dgrad: 32768x4096x4096) + group_m sweep.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gprof
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d gpurun_out/gprof/p1 -o run --output-format csv -- python3 scripts/prof_gemm_one.py dgrad 4096 4096 10 > gpurun_out/gprof/p1.log 2>&1
echo "p1 rc=$?"
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES -d gpurun_out/gprof/p2 -o run --output-format csv -- python3 scripts/prof_gemm_one.py dgrad 4096 4096 10 > gpurun_out/gprof/p2.log 2>&1
echo "p2 rc=$?"
for g in 4 8 16 32; do PADDLE2_AMD_GEMM_GROUP_M=$g timeout -k 10 120 python -u scripts/bench_gemm_native.py 2>/dev/null | grep '"o_proj"\|"qkv"' | sed "s/^/g$g /"; done
