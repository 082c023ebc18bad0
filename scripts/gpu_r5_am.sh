#!/bin/bash
# Round 5 (am): kernel trace of the b1 HIP-graph decode (Llama-2-7B): per-kernel time per decode step vs the step.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5am
mkdir -p $O
export TMPDIR=/tmp PYTHONPATH=$PWD
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof_b1 -o run --output-format csv -- python3 scripts/bench_serving.py --batch 1 --prompt 1024 --new 64 > $O/prof_b1.log 2>&1
r=$?; echo "prof rc=$r: $(grep -E 'ms/step|tok/s' $O/prof_b1.log | tail -2 | cut -c1-200)"; [ $r -ne 0 ] && { tail -20 $O/prof_b1.log; exit $r; }
python3 scripts/kernel_table.py $(find $O/prof_b1 -name "*kernel_trace.csv" | head -1) > $O/kernels_b1.txt 2>&1; head -30 $O/kernels_b1.txt
cp $(find $O/prof_b1 -name "*kernel_trace.csv" | head -1) $O/trace_b1.csv
python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/r5am/trace_b1.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# the last 640 kernels ~ the last decode steps; print gaps between consecutive kernels
ks = rows[-2000:]
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(ks, ks[1:])]
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks)
span = int(ks[-1]["End_Timestamp"]) - int(ks[0]["Start_Timestamp"])
gaps_s = sorted(gaps)
print(f"last {len(ks)} kernels: span {span/1e6:.2f} ms, busy {busy/1e6:.2f} ms, gap median {gaps_s[len(gaps)//2]/1e3:.2f} us, "
      f"p90 {gaps_s[int(len(gaps)*0.9)]/1e3:.2f} us, total gaps {sum(g for g in gaps if g > 0)/1e6:.2f} ms")
c = collections.Counter(r["Kernel_Name"][:80] for r in ks)
t = collections.Counter()
for r in ks:
    t[r["Kernel_Name"][:80]] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
for k, v in t.most_common(14):
    print(f"{v/1e6:8.3f} ms {c[k]:5d}x  {k}")
PY
rm -f $(find $O/prof_b1 -name "*kernel_trace.csv") $O/trace_b1.csv 2>/dev/null
exit 0
