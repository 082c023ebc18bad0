"""Per-step kernel table from a rocprofv3 kernel trace: the span between the 2nd and 3rd AdamW launch is one
steady-state step; kernels grouped by (short name, grid, workgroup) with calls, total ms and share."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
opt = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"].lower()]
# step boundaries: first AdamW launch of each optimizer step (launches of one step are consecutive)
starts = [opt[0]] + [b for a, b in zip(opt, opt[1:]) if b - a > 1]
lo, hi = (starts[-2], starts[-1]) if len(starts) >= 2 else (0, len(rows))
step = rows[lo:hi]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
busy = 0.0
for r in step:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    busy += d
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:70]
    key = (name, r.get("Grid_Size", ""), r.get("Workgroup_Size", ""))
    agg[key][0] += 1
    agg[key][1] += d
print(f"step span {(t1 - t0) / 1e6:.1f} ms, kernel busy {busy:.1f} ms, {len(step)} launches")
for (name, g, w), (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
    print(f"{ms:9.2f} ms {100 * ms / busy:5.1f}% {n:5d}x grid {g:>9} wg {w:>4}  {name}")
