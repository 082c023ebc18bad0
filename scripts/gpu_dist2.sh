#!/bin/bash
# The bench's N>1 code path (stage-3 all-gather / reduce-scatter, barriers, max-over-ranks timing) on ONE GPU:
# two ranks share cuda:0 and talk over gloo (RCCL cannot put two ranks on one device); tiny Llama.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dist2
export PYTHONPATH=$GRAFT_REPO_ROOT
PADDLE_DISTRI_BACKEND=gloo PADDLE2_AMD_DEVICE=gpu:0 timeout -k 10 400 python -u bench.py --gpus 2 --model tiny \
    --seq-len 512 --micro-batch 2 --steps 3 --warmup 1 > gpurun_out/dist2/bench2.log 2>&1
rc=$?; echo "dist2 rc=$rc"; grep '"metric"' gpurun_out/dist2/bench2.log | cut -c1-400; tail -5 gpurun_out/dist2/bench2.log | cut -c1-300
exit $rc
