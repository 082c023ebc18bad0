#!/bin/bash
# Round 6 (e): PMC counters of the split-dQ backward kernels (bwd main kernel with dS out, dq_gemm_kernel).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $O/p1 -o run --output-format csv -- python3 scripts/prof_flash_bwd_split.py 1 > $O/p1.log 2>&1
r=$?; [ $r -ne 0 ] && { tail -20 $O/p1.log; exit $r; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d $O/p2 -o run --output-format csv -- python3 scripts/prof_flash_bwd_split.py 1 > $O/p2.log 2>&1
r=$?; [ $r -ne 0 ] && { tail -20 $O/p2.log; exit $r; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $O/p3 -o run --output-format csv -- python3 scripts/prof_flash_bwd_split.py 0 > $O/p3.log 2>&1
r=$?; [ $r -ne 0 ] && { tail -20 $O/p3.log; exit $r; }
find $O -name "*kernel_trace.csv" -delete
exit 0
