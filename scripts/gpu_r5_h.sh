#!/bin/bash
# Round 5 (h): the GPT-3 13B fp8 step (b2 s2048): default routing (fp8 schedule 2 is now the kernel default), fp8
# wgrad into the fp32 main-grad slot, the all-native fp8 GEMM on schedules 1 / 2; then kernel tables of the default
# fp8 step and of the default Llama-2-7B bench step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5h
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
B="bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 8 --warmup 3"
for v in "default:" "wmain:PADDLE2_AMD_FP8_WGRAD_MAIN=1" "nat1:PADDLE2_AMD_FP8_GEMM=native PADDLE2_AMD_FP8_SCHED=1" \
         "nat2:PADDLE2_AMD_FP8_GEMM=native PADDLE2_AMD_FP8_SCHED=2"; do
  name=${v%%:*}; envs=${v#*:}
  env $envs timeout -k 10 300 python -u $B > $O/fp8_$name.log 2>&1
  r=$?; echo "$name: $(tail -1 $O/fp8_$name.log | cut -c1-200)"; [ $r -ne 0 ] && { tail -30 $O/fp8_$name.log; exit $r; }
done
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_fp8 -o run --output-format csv -- python3 bench.py --model gpt3-13b --fp8 --seq-len 2048 --micro-batch 2 --steps 3 --warmup 2 > $O/prof_fp8.log 2>&1
r=$?; echo "prof rc=$r"; [ $r -ne 0 ] && { tail -20 $O/prof_fp8.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_fp8 -name "*kernel_trace.csv" | head -1) > $O/kernels_fp8.txt 2>&1; head -45 $O/kernels_fp8.txt
rm -f $(find $O/prof_fp8 -name "*kernel_trace.csv") 2>/dev/null
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $O/prof_7b -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $O/prof_7b.log 2>&1
r=$?; echo "prof 7b rc=$r"; tail -1 $O/prof_7b.log | cut -c1-300; [ $r -ne 0 ] && { tail -20 $O/prof_7b.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_7b -name "*kernel_trace.csv" | head -1) > $O/kernels_7b.txt 2>&1; head -45 $O/kernels_7b.txt
rm -f $(find $O/prof_7b -name "*kernel_trace.csv") 2>/dev/null
exit 0
