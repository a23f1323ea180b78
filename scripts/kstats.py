"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time (per-step figures need the
step count of the profiled run: bench.py --steps S --warmup W runs S + W steps plus one setup
build)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{len(rows)} kernels, total {tot / 1e6:.3f} ms, per step {tot / 1e6 / steps:.3f} ms")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step {int(r['Calls']) / steps:7.1f}/step "
          f"{float(r['AverageNs']) / 1e3:8.2f} us  {r['Name'][:100]}")
