#!/bin/bash
# kernel table of the Llama-2-7B serving run (b64, prompt 1024, 64 new tokens, HIP-graph decode)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pdec
export PYTHONPATH=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/pdec/trace -o run -- \
    python3 $GRAFT_REPO_ROOT/scripts/bench_serving.py --new 32 > $GRAFT_REPO_ROOT/gpurun_out/pdec/run.log 2>&1
rc=$?; tail -2 $GRAFT_REPO_ROOT/gpurun_out/pdec/run.log; exit $rc
