"""Timeline of one concurrent bench step from a rocprofv3 kernel trace (bench.py without --serial:
store on the engine stream, the analyses' graphs on four streams).  A step runs from one
k_elig_hist (the store's first kernel) to the next; per stream: first start, last end, busy time
and kernel count, relative to the step start - the critical path is the stream that ends last.
usage: step_timeline.py TRACE.csv [STEP_INDEX_FROM_END]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
back = int(sys.argv[2]) if len(sys.argv) > 2 else 2
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_elig_hist" in r["Kernel_Name"]]
a, b = starts[-back - 1], starts[-back]
step = rows[a:b]
t0 = int(step[0]["Start_Timestamp"])
end = max(int(r["End_Timestamp"]) for r in step)
print(f"step span {(end - t0) / 1e3:.1f} us, {len(step)} kernels")
by = defaultdict(list)
for r in step:
    by[(r["Queue_Id"], r["Stream_Id"])].append(r)
for k, rs in sorted(by.items(), key=lambda kv: int(kv[1][0]["Start_Timestamp"])):
    s = (int(rs[0]["Start_Timestamp"]) - t0) / 1e3
    e = (max(int(r["End_Timestamp"]) for r in rs) - t0) / 1e3
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rs) / 1e3
    first = rs[0]["Kernel_Name"].split("(")[0][:50]
    last = rs[-1]["Kernel_Name"].split("(")[0][:50]
    print(f"queue {k[0]:>3} stream {k[1]:>3}: {len(rs):4d} kernels  {s:8.1f} -> {e:8.1f} us  busy {busy:8.1f}  "
          f"first {first} | last {last}")
# STREAM_DUMP=1: every kernel of the stream that ends last (the critical path), with its start /
# end relative to the step and the gap to the previous kernel of that stream
import os  # noqa: E402
if os.environ.get("STREAM_DUMP"):
    last = max(by.items(), key=lambda kv: max(int(r["End_Timestamp"]) for r in kv[1]))
    prev = None
    print(f"-- critical stream {last[0]}")
    for r in last[1]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else 0.0
        prev = e
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} us  gap {gap:6.1f}  {r['Kernel_Name'].split('(')[0][:90]}")
