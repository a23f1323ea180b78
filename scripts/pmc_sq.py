"""Shader-sequencer counters per kernel family from one rocprofv3 --pmc pass (at most 8 SQ_
counters per run, MI355X_MICROARCH.md): where a family's wave cycles go.

    python scripts/pmc_sq.py <counter_collection.csv> <out.json>

SQ_WAVE_CYCLES, SQ_WAIT_ANY (parked on s_waitcnt / barriers), SQ_WAIT_INST_ANY (issue stalls) and
SQ_ACTIVE_INST_ANY are disjoint parts of the wave cycles (all in quad-cycles); SQ_ACTIVE_INST_VALU
over the wave cycles is the VALU-issue share.  A memory/latency-bound kernel shows WAIT_ANY
dominating; a compute-bound one ACTIVE_INST_VALU."""
import csv
import json
import sys

FAMILIES = {
    "seg_reduce": ["k_chunk_reduce", "k_seg_fold", "k_seg_sum", "k_tiny_reduce"],
    "seg_spearman": ["k_spearman_chunks", "k_spearman_index_small"],
    "seg_value_sort": ["k_seg_val_bucket", "k_seg_sort_"],
    "seg_qstats": ["k_qs_micro", "k_qs_tiny", "k_qs_block"],
    "describe_select": ["k_describe_sel"],
    "two_sample_small": ["k_two_sample_small"],
    "ragged_transpose": ["k_rt_move"],
    "radix_scatter": ["k_onesweep<"],
    "filter_compact": ["k_filter_compact"],
    "seg_time_sort": ["k_seg_time_bucket"],
    "bm": ["k_bm_"],
}


def main():
    path, out = sys.argv[1:3]
    acc, per = {}, {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        # every kernel on its own too (name up to its argument list, template arguments cut at 60)
        kk = k.split("(")[0][:90]
        b = per.setdefault(kk, {"dispatches": set()})
        b["dispatches"].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        b[r["Counter_Name"]] = b.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        fam = next((f for f, subs in FAMILIES.items() if any(s in k for s in subs)), None)
        if fam is None:
            continue
        a = acc.setdefault(fam, {"dispatches": set()})
        a["dispatches"].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        a[r["Counter_Name"]] = a.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    res = {}
    kernels = {}
    for kk, a in sorted(per.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0.0))[:40]:
        d = {k: v for k, v in a.items() if k != "dispatches"}
        d["dispatches"] = len(a["dispatches"])
        wc = d.get("SQ_WAVE_CYCLES", 0.0)
        if wc > 0:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
                if k in d:
                    d[k + "_share"] = round(d[k] / wc, 4)
        kernels[kk] = d
    for fam, a in acc.items():
        d = {k: v for k, v in a.items() if k != "dispatches"}
        d["dispatches"] = len(a["dispatches"])
        wc = d.get("SQ_WAVE_CYCLES", 0.0)
        if wc > 0:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_SCA"):
                if k in d:
                    d[k + "_share"] = round(d[k] / wc, 4)
        res[fam] = d
    json.dump({"source": path, "families": res, "kernels": kernels}, open(out, "w"), indent=1)
    for fam, d in sorted(res.items()):
        print(fam, {k: v for k, v in d.items() if k.endswith("_share") or k == "dispatches"})
    print("-- kernels by wave cycles")
    for kk, d in kernels.items():
        print(f"{d.get('SQ_WAVE_CYCLES', 0):14.0f} n={d['dispatches']:5d} wait={d.get('SQ_WAIT_ANY_share', 0):.2f} "
              f"valu={d.get('SQ_ACTIVE_INST_VALU_share', 0):.2f} lds={d.get('SQ_ACTIVE_INST_LDS_share', 0):.2f} {kk}")


if __name__ == "__main__":
    main()
