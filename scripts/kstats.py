"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time, per step.

    python3 scripts/kstats.py <kernel_stats.csv> [steps|auto] [top]

The step count defaults to ``auto``: the call count of a kernel that runs exactly once per step -
the store build's gather (``k_store_gather``, one launch per fz_store_build, and every step of
bench.py builds the store once; the untimed warm-up, recording and probe-window steps included).
A number given instead is used as is (round 4's summaries passed steps + 3 and so under-counted
the warm-up / probe steps: "1.4/step" for once-per-step kernels)."""
import csv
import sys

STEP_KERNEL = "k_store_gather"

rows = list(csv.DictReader(open(sys.argv[1])))
arg = sys.argv[2] if len(sys.argv) > 2 else "auto"
if arg == "auto":
    once = [r for r in rows if STEP_KERNEL in r["Name"]]
    steps = float(sum(int(r["Calls"]) for r in once)) if once else 1.0
    how = f"{int(steps)} steps = calls of {STEP_KERNEL}" if once else "1 step (no step kernel in the trace)"
else:
    steps = float(arg)
    how = f"{arg} steps (given)"
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{len(rows)} kernels, total {tot / 1e6:.3f} ms, {how}, per step {tot / 1e6 / steps:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) / steps:7.1f}/step "
          f"{float(r['AverageNs']) / 1e3:8.2f} us  {r['Name'][:100]}")
