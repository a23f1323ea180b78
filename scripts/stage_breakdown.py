"""Per-stage kernel time of one serial bench step from a rocprofv3 kernel trace (bench.py --serial:
every launch on one stream in program order).  A step starts at the store's k_elig_hist; stages
are cut at each analysis' first kernel (the first launch after the previous stage that matches the
stage's opener).  usage: stage_breakdown.py TRACE.csv [TOP] [STAGE,NAMES]  (the names in launch
order: the sharded step runs its drivers as bench.py --shard-groups lists them)"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 12
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_elig_hist" in r["Kernel_Name"]]
a, b = starts[-2], starts[-1]
step = rows[a:b]
# stage openers in serial_step order: store, rq1, rq2_count, rq2_add, rq3, rq4a, rq4b (each analysis
# copies the eligible-project flags first: k_copy_elig)
cuts = [0] + [i for i, r in enumerate(step) if "k_copy_elig" in r["Kernel_Name"]]
names = ["store"] + (sys.argv[3].split(",") if len(sys.argv) > 3 else ["rq1", "rq2_count", "rq2_add", "rq3", "rq4a", "rq4b"])
t0 = int(step[0]["Start_Timestamp"])
print(f"step span {(int(step[-1]['End_Timestamp']) - t0) / 1e3:.1f} us, {len(step)} kernels, cuts {len(cuts)}")
for si, c0 in enumerate(cuts):
    c1 = cuts[si + 1] if si + 1 < len(cuts) else len(step)
    part = step[c0:c1]
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in part)
    span = int(part[-1]["End_Timestamp"]) - int(part[0]["Start_Timestamp"])
    nm = names[si] if si < len(names) else f"stage{si}"
    print(f"== {nm}: {len(part)} kernels, busy {busy / 1e3:.1f} us, span {span / 1e3:.1f} us")
    agg = defaultdict(lambda: [0, 0])
    for r in part:
        k = r["Kernel_Name"].split("(")[0][:90]
        agg[k][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[k][1] += 1
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"   {t / 1e3:9.1f} us {n:4d}x  {k}")
