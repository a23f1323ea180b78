"""Summarise a one-GPU strong-scaling rehearsal (scripts/gpu_r6.sh STEPS=strong: lines
"<config> shard <r> of <N> <ms_per_step> <rows>") as JSON: per N the slowest shard's step (each shard's fastest of its repeats; T(N), the
per-rank compute of an N-GPU run before any exchange), speedup T(1) / T(N), efficiency speedup / N
and the ratio T(N) / (T(1) / N).

    python3 scripts/strong_summary.py profiles/r06_c5L_strong.txt > profiles/r06_c5L_strong.json"""
import json
import sys
from collections import defaultdict


def main(path):
    shards = defaultdict(dict)
    cfg = None
    for ln in open(path):
        f = ln.split()
        if len(f) < 6 or f[1] != "shard":
            continue
        cfg = f[0]
        v = (float(f[5]), int(f[6]) if len(f) > 6 else None)
        old = shards[int(f[4])].get(int(f[2]))
        shards[int(f[4])][int(f[2])] = v if old is None or v[0] < old[0] else old  # (repeats: the fastest)
    t = {n: max(v[0] for v in d.values()) for n, d in shards.items()}
    out = {"config": cfg, "source": path, "T_ms": {str(n): t[n] for n in sorted(t)},
           "shards_ms": {str(n): [shards[n][r][0] for r in sorted(shards[n])] for n in sorted(shards)},
           "shard_rows": {str(n): [shards[n][r][1] for r in sorted(shards[n])] for n in sorted(shards)}}
    if 1 in t:
        out["speedup"] = {str(n): round(t[1] / t[n], 3) for n in sorted(t)}
        out["efficiency"] = {str(n): round(t[1] / t[n] / n, 3) for n in sorted(t)}
        out["T_over_linear"] = {str(n): round(t[n] / (t[1] / n), 3) for n in sorted(t)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
