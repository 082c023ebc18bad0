#!/bin/bash
# Round 6 (ae): PMC counters of the weight gradient (qkv shape, 32768 tokens, beta 0) on v4's spread kernel (variant 5)
# vs the persistent MN-major v7 kernel, and of the TN dgrad / N-major forward for reference.  One counter pass per
# kernel (8 SQ + 1 GRBM counters), --kernel-trace only.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6ae
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
prof() {  # name, env, args
  local n=$1; shift; local e=$1; shift
  env $e timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$n -o run -- python3 scripts/prof_gemm_one.py "$@" > $O/$n.log 2>&1
  local r=$?; echo "$n rc=$r"; [ $r -ne 0 ] && { tail -5 $O/$n.log; exit $r; }
}
prof wgrad_v5 PADDLE2_AMD_GEMM_VARIANT_WGRAD=5 wgrad0 4096 12288 10
prof wgrad_v7mn X=0 wgrad0 4096 12288 10
prof dgrad_tn X=0 dgrad 12288 4096 10
prof fwd_nn X=0 fwd 4096 12288 10
for d in wgrad_v5 wgrad_v7mn dgrad_tn fwd_nn; do rm -f $(find $O/$d -name "*kernel_trace.csv") 2>/dev/null; done
exit 0
