#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONPATH=$PWD TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u scripts/debug_conv3x3c.py > gpurun_out/dbg_conv3.log 2>&1
echo rc=$?; grep -v amdgpu.ids gpurun_out/dbg_conv3.log | head -80
