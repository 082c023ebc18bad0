#!/bin/bash
# Round-3 kernel profiles of the secondary configs (verdict item 9): ResNet50 bf16 NHWC b256 and GPT-3 13B bf16
# b2 s2048 (stage 3), rocprofv3 kernel trace -> per-step kernel tables; flash GPU tests first.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sec
export PYTHONPATH=$GRAFT_REPO_ROOT TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread -m gpu tests/test_native_allocator.py \
    tests/test_batch_norm_gpu.py > gpurun_out/sec/alloc_tests.log 2>&1
rc=$?; tail -2 gpurun_out/sec/alloc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/bench_resnet50.py --steps 20 --warmup 5 --batch 256 > gpurun_out/sec/resnet.json \
    2> gpurun_out/sec/resnet.err
rc=$?; echo "resnet rc=$rc"; cat gpurun_out/sec/resnet.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/sec/prof_resnet -o run --output-format csv -- \
    python3 scripts/bench_resnet50.py --steps 3 --warmup 2 --batch 256 > gpurun_out/sec/resnet_prof.log 2>&1
rc=$?; echo "resnet rocprof rc=$rc"; tail -1 gpurun_out/sec/resnet_prof.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
python3 scripts/kernel_table.py gpurun_out/sec/prof_resnet/run_kernel_trace.csv > gpurun_out/sec/resnet_kernels.txt
head -30 gpurun_out/sec/resnet_kernels.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/sec/prof_gpt -o run --output-format csv -- \
    python3 bench.py --model gpt3-13b --seq-len 2048 --micro-batch 2 --steps 2 --warmup 1 \
    > gpurun_out/sec/gpt_prof.log 2>&1
rc=$?; echo "gpt rocprof rc=$rc"; grep '"metric"' gpurun_out/sec/gpt_prof.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
python3 scripts/kernel_table.py gpurun_out/sec/prof_gpt/run_kernel_trace.csv > gpurun_out/sec/gpt_kernels.txt
head -30 gpurun_out/sec/gpt_kernels.txt
rm -f gpurun_out/sec/prof_*/run_kernel_trace.csv.gz
