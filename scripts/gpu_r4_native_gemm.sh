#!/bin/bash
# Round 4: GEMM GPU tests (spread TN kernel as the default forward / dgrad / SwiGLU route), isolated bench incl.
# the SwiGLU epilogue, the 1-GPU training bench (native vs hipBLASLt routing), and a kernel trace of the step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4ng
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 900 python3 -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 300 --timeout-method thread > $O/gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 $O/gemm_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u scripts/bench_gemm_v7.py 448 > $O/bench_gemm.jsonl 2> $O/bench_gemm.err || exit $?
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 3 > $O/bench_native.log 2>&1
rc=$?; echo "bench native rc=$rc"; tail -1 $O/bench_native.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
PADDLE2_AMD_GEMM_FWD=blas PADDLE2_AMD_GEMM_DGRAD=blas timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 3 > $O/bench_blas.log 2>&1
rc=$?; echo "bench blas rc=$rc"; tail -1 $O/bench_blas.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 > $O/bench_prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 scripts/kernel_table.py $O/prof/run_kernel_trace.csv > $O/kernels.txt
head -40 $O/kernels.txt
