"""HBM counter bytes per kernel NAME (template arguments included, so each time-sort length class
is its own row) from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; KB per dispatch).

    python scripts/pmc_by_kernel.py <fetch csv> <write csv> <out.json> [name substring ...]

Raw counter bytes, no width correction (see profiles/r05_pmc_calib.json for the per-width ratios)."""
import csv
import json
import sys


def per_kernel(path):
    out = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        e = out.setdefault(k, [set(), 0.0])
        e[0].add(d)
        e[1] += float(r["Counter_Value"]) * 1024.0
    return {k: (len(v[0]), v[1]) for k, v in out.items()}


def main():
    fcsv, wcsv, dst = sys.argv[1:4]
    subs = sys.argv[4:]
    f, w = per_kernel(fcsv), per_kernel(wcsv)
    rows = []
    for k in sorted(set(f) | set(w)):
        if subs and not any(s in k for s in subs):
            continue
        nf, fb = f.get(k, (0, 0.0))
        nw, wb = w.get(k, (0, 0.0))
        rows.append({"kernel": k[:160], "dispatches": max(nf, nw), "fetch_raw_bytes": fb, "write_bytes": wb})
    rows.sort(key=lambda r: -(r["fetch_raw_bytes"] + r["write_bytes"]))
    for r in rows[:40]:
        print("%5d  fetch(raw) %10.1f MB  write %10.1f MB  %s" % (r["dispatches"], r["fetch_raw_bytes"] / 1e6,
                                                                 r["write_bytes"] / 1e6, r["kernel"][:100]))
    json.dump({"sources": [fcsv, wcsv], "kernels": rows}, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
