"""HBM traffic per probed launch of the bench's roofline kernels from two rocprofv3 PMC passes
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are collected in separate runs
(FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2), both in KB per dispatch.  gfx950
correction: FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is
doubled; WRITE_SIZE is taken as is.

    python scripts/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> \
        <config> <out.json>

One probe scope of bench.py (fz_probe) may cover several dispatches (the store's time sort is
four length-class launches per table): its traffic is the sum over the matching dispatches divided
by the number of scopes, counted by a kernel that runs exactly once per scope.  bench.py reads
<out.json> (profiles/*_pmc_traffic.json) into roofline.traffic and the per-kernel table."""
import csv
import json
import sys

# probe name -> (kernel-name substring of its dispatches, substring of a once-per-scope kernel)
KERNELS = {
    "radix_scatter": ("k_onesweep<", "k_onesweep<"),
    "radix_hist": ("k_onesweep_hist", "k_onesweep_hist"),
    "elig_hist": ("k_elig_hist", "k_elig_hist"),
    "filter_compact": ("k_filter_compact", "k_filter_compact"),
    "seg_time_sort": ("k_seg_time_bucket", "k_prefix_offsets"),
    "store_gather": ("k_store_gather", "k_store_gather"),
}


def dispatches(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out.setdefault(int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(out)), []).append(
            (r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    return [(v[0][0], sum(x for _, x in v)) for _, v in sorted(out.items())]


def per_scope(rows, sub, per):
    n = sum(1 for k, _ in rows if per in k)
    tot = sum(b for k, b in rows if sub in k)
    return (tot / n, n) if n else (None, 0)


def main():
    fetch_csv, write_csv, config, out = sys.argv[1:5]
    f, w = dispatches(fetch_csv), dispatches(write_csv)
    res = {"config": config, "kernels": {},
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of "
                     "bench.py; FETCH_SIZE x2 (gfx950 correction); bytes per probe scope",
           "sources": [fetch_csv, write_csv]}
    for probe, (sub, per) in KERNELS.items():
        fb, nf = per_scope(f, sub, per)
        wb, nw = per_scope(w, sub, per)
        if fb is None or wb is None or nf != nw:
            continue
        res["kernels"][probe] = {"kernel_match": sub, "scopes": nf, "fetch_bytes_per_launch": 2.0 * fb,
                                 "fetch_raw_bytes_per_launch": fb, "write_bytes_per_launch": wb,
                                 "traffic_bytes_per_launch": 2.0 * fb + wb}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
