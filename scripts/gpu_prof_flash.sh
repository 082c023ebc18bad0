#!/bin/bash
# Two PMC passes (each its own run, counters within per-block limits) over the flash fwd/bwd kernels.
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_flash
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA -d $OUT/p1 -o p1 --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/prof_flash.py || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD -d $OUT/p2 -o p2 --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/prof_flash.py || exit $?
find $OUT -name "*.csv" | head
