"""HBM traffic per launch of one kernel from two rocprofv3 PMC passes (MI355X_MICROARCH.md, HBM
section): FETCH_SIZE and WRITE_SIZE are collected in separate runs (FETCH_SIZE takes 3 of the 4
TCC slots, WRITE_SIZE 2), both in KB per dispatch.  gfx950 correction: FETCH_SIZE reports half the
bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is.

    python scripts/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> \
        <kernel-name substring> <config> <out.json>

bench.py reads <out.json> (profiles/) into roofline.traffic when kernel and config match."""
import csv
import json
import sys


def per_dispatch(path, sub):
    out = []
    for r in csv.DictReader(open(path)):
        if sub in r["Kernel_Name"]:
            out.append(float(r["Counter_Value"]) * 1024.0)
    return out


def main():
    fetch_csv, write_csv, sub, config, out = sys.argv[1:6]
    f = per_dispatch(fetch_csv, sub)
    w = per_dispatch(write_csv, sub)
    if not f or len(f) != len(w):
        raise SystemExit(f"dispatch counts differ or empty: fetch {len(f)}, write {len(w)}")
    fetch = 2.0 * sum(f) / len(f)   # gfx950: FETCH_SIZE = 1/2 of wide streaming-read bytes
    write = sum(w) / len(w)
    res = {"kernel_match": sub, "config": config, "launches": len(f), "fetch_bytes_per_launch": fetch,
           "fetch_raw_bytes_per_launch": fetch / 2.0, "write_bytes_per_launch": write,
           "traffic_bytes_per_launch": fetch + write,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                     "bench.py --steps 2 --warmup 1 --no-cpu-baseline; FETCH_SIZE x2 (gfx950 correction)",
           "sources": [fetch_csv, write_csv]}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
