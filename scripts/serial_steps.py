"""One step of a serial kernel trace (scripts/gpu_r4.sh profs:...): the kernels of the step in
launch order with their durations and the idle gap before each, then the per-kernel totals.
Steps start at the store's prologue kernel; the step printed is the median-length one of the
timed steps.

usage: python scripts/serial_steps.py <run_kernel_trace.csv> [first-kernel substring]"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    mark = sys.argv[2] if len(sys.argv) > 2 else "k_store_prologue"
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
    spans = []
    for a, b in zip(starts, starts[1:]):
        t0 = int(rows[a]["Start_Timestamp"])
        t1 = int(rows[b - 1]["End_Timestamp"])
        spans.append((t1 - t0, a, b))
    spans = spans[2:]  # (warm-up steps)
    spans.sort()
    dur, a, b = spans[len(spans) // 2]
    print(f"{len(spans)} steps; median step {dur / 1000:.1f} us, {b - a} kernels")
    prev = None
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    busy = 0.0
    for r in rows[a:b]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1000 if prev is not None else 0.0
        name = r["Kernel_Name"]
        short = name.split("(")[0][-70:] if "(" in name else name[-70:]
        print(f"{(s - int(rows[a]['Start_Timestamp'])) / 1000:9.1f} {(e - s) / 1000:8.1f} gap {gap:6.1f}  {short}")
        tot[short] += (e - s) / 1000
        cnt[short] += 1
        busy += (e - s) / 1000
        prev = e
    print(f"busy {busy:.1f} us of {dur / 1000:.1f}")
    for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{v:9.1f} us {cnt[k]:3d}x  {k}")


if __name__ == "__main__":
    main()
