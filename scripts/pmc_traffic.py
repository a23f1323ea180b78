"""HBM traffic per probed launch of the bench's roofline kernels from two rocprofv3 PMC passes
(MI355X_MICROARCH.md, HBM section): FETCH_SIZE and WRITE_SIZE are collected in separate runs
(FETCH_SIZE takes 3 of the 4 TCC slots, WRITE_SIZE 2), both in KB per dispatch.  gfx950
correction: FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so it is
doubled; WRITE_SIZE is taken as is.

    python scripts/pmc_traffic.py <fetch counter_collection.csv> <write counter_collection.csv> \
        <config> <out.json>

The PMC runs are `bench.py --serial` (every launch on one stream, so dispatch order is program
order).  One probe scope of bench.py (fz_probe) may cover several dispatches; each scope below is
found in the dispatch sequence: it opens at an `open` kernel (or at its first matching kernel when
it has none), takes the `match` dispatches that follow, and closes at the first dispatch that
matches neither `match` nor `allow` (or at `close`).  traffic = bytes of the matched dispatches /
number of scopes.  A kernel that several scopes launch (k_seg_time_bucket: the store's time sort
and the long-segment sub-bucket sort) is booked to the scope whose opener precedes it, so no
dispatch is counted twice and traffic / scope time stays a physical rate.  bench.py reads
<out.json> (profiles/*_pmc_traffic.json) into roofline.traffic and the per-kernel table."""
import csv
import json
import sys

SCOPES = {
    # (round 6: the store's three tables share each pass, k_onesweep_tabs)
    "radix_scatter": {"match": ["k_onesweep<", "k_onesweep_tabs<"]},
    "radix_hist": {"match": ["k_onesweep_hist"]},
    "elig_hist": {"match": ["k_elig_hist"]},
    # (the selective filters - tiles of unselected projects skipped - are probed apart)
    "filter_compact": {"match": ["k_filter_compact"], "exclude": ["CovRowsRq3", "PositiveCoverage34", "CovRowsBeforeLimit"]},
    # (template names go on after the predicate: "k_filter_compact<fz::CovRowsRq3, ...>")
    "filter_select": {"match": ["k_filter_compact<fz::CovRowsRq3", "k_filter_compact<fz::PositiveCoverage34",
                                "k_filter_compact<fz::CovRowsBeforeLimit"]},
    # the four length-class launches of the store's time sort (all three tables), between the prefix
    # offsets and the views launch
    "seg_time_sort": {"open": "k_prefix_offsets", "match": ["k_seg_time_bucket"], "allow": ["k_fill"],
                      "close": "k_store_views"},
    "store_gather": {"match": ["k_store_gather"]},
    "big_compact": {"match": ["k_big_compact"]},
    # the long class over the sub-buckets, right after the radix passes of the distribution (fills
    # of its counters between)
    "big_sub_sort": {"open": "k_big_compact", "match": ["k_seg_time_bucket"],
                     "allow": ["k_fill", "k_onesweep", "__amd"]},
    "seg_reduce": {"open": "k_chunk_reduce", "match": ["k_chunk_reduce", "k_seg_fold", "k_seg_sum"],
                   "pre": ["k_tiny_reduce"]},
    "seg_spearman": {"open": "k_spearman_chunks", "match": ["k_spearman_chunks", "k_seg_fold", "k_seg_sum"]},
    "seg_rank_union": {"open": "k_bm_union_chunks<0>", "match": ["k_bm_union_chunks", "k_seg_fold", "k_seg_sum"]},
    "scan_i64": {"match": ["k_scan_lookback"]},
    # RQ2's per-session order statistics by selection: the small-segment launch opens the scope
    # (the size-class lists and the workgroup classes follow)
    "seg_qstats": {"open": "k_qs_micro", "match": ["k_qs_micro", "k_qs_tiny", "k_qs_sort_mid", "k_qs_block", "k_qs_wave"],
                   "allow": ["k_fill"]},
    "describe_select": {"match": ["k_describe_sel"]},
    "spearman_shapiro": {"match": ["k_spearman_index_small"]},
    "ragged_transpose": {"match": ["k_rt_move"]},
    # seg_sort_f64's bucket path: value bucket classes, then the merge sort of flagged segments
    "seg_value_sort": {"open": "k_seg_val_bucket<256, 1024>",
                       "match": ["k_seg_val_bucket", "k_tile_sort", "k_merge_round", "k_merge_splits",
                                 "k_tile_count", "k_tile_fill", "k_scan"],
                       "allow": ["k_fill"]},
}


def dispatches(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out.setdefault(int(r.get("Dispatch_Id") or r.get("Correlation_Id") or len(out)), []).append(
            (r["Kernel_Name"], float(r["Counter_Value"]) * 1024.0))
    return [(v[0][0], sum(x for _, x in v)) for _, v in sorted(out.items())]


def scopes(rows, spec):
    """(scopes found, bytes of their dispatches) for one scope spec over the dispatch sequence."""
    match, allow = spec["match"], spec.get("allow", []) + ["__amd_rocclr"]
    opener, closer, pre = spec.get("open"), spec.get("close"), spec.get("pre", [])
    has = lambda k, subs: any(s in k for s in subs)  # noqa: E731
    n, tot, inside, pend = 0, 0.0, False, 0.0
    excl = spec.get("exclude", [])
    for k, b in rows:
        if excl and has(k, excl):
            continue
        if opener is None:  # every matching dispatch is one probed launch
            if has(k, match):
                n += 1
                tot += b
            continue
        if opener in k:
            n += 1
            inside = True
            tot += pend + (b if has(k, match) else 0.0)
            pend = 0.0
            continue
        if inside:
            if closer and closer in k:
                inside = False
            elif has(k, match):
                tot += b
                continue
            elif has(k, allow):
                continue
            else:
                inside = False
        pend = b if has(k, pre) else 0.0
    return n, tot


def main():
    fetch_csv, write_csv, config, out = sys.argv[1:5]
    f, w = dispatches(fetch_csv), dispatches(write_csv)
    res = {"config": config, "kernels": {},
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs of bench.py --serial; "
                     "FETCH_SIZE x2 (gfx950 correction); bytes per probe scope, scopes found in dispatch order "
                     "(scripts/pmc_traffic.py SCOPES)",
           "sources": [fetch_csv, write_csv]}
    for probe, spec in SCOPES.items():
        nf, fb = scopes(f, spec)
        nw, wb = scopes(w, spec)
        if nf == 0 or nf != nw:
            continue
        res["kernels"][probe] = {"scope": spec, "scopes": nf, "fetch_bytes_per_launch": 2.0 * fb / nf,
                                 "fetch_raw_bytes_per_launch": fb / nf, "write_bytes_per_launch": wb / nw,
                                 "traffic_bytes_per_launch": (2.0 * fb / nf) + wb / nw}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
