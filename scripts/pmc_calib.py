"""Counter / byte ratios of scripts/pmc_calib.hip's kernels (one known byte count per access width).

    python scripts/pmc_calib.py <fetch counter_collection.csv> <write counter_collection.csv> \
        <pmc_calib stdout> <out.json>

FETCH_SIZE and WRITE_SIZE are in KB per dispatch; the ratio printed is counter bytes / moved bytes
(no correction applied): 0.5 for a read means the guide's x2 gfx950 correction holds for that width,
1.0 means the counter is exact for it."""
import csv
import json
import sys


def per_kernel(path):
    out = {}
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        out.setdefault(k, 0.0)
        out[k] += float(r["Counter_Value"]) * 1024.0
    return out


def main():
    fcsv, wcsv, log, dst = sys.argv[1:5]
    moved = {}
    for line in open(log):
        p = line.split()
        if len(p) == 2 and p[0].startswith("k_"):
            moved[p[0]] = int(p[1])
    f, w = per_kernel(fcsv), per_kernel(wcsv)
    res = {"method": "scripts/pmc_calib.hip: one dispatch per access width over 1 GiB (past the Infinity Cache, "
                     "a 1 GiB write between dispatches); counter bytes / moved bytes, uncorrected", "kernels": {}}
    for name, nb in moved.items():
        key = name.replace("<", "<").strip()
        fk = [k for k in f if k.startswith("void " + key) or k.startswith(key)]
        wk = [k for k in w if k.startswith("void " + key) or k.startswith(key)]
        fb = sum(f[k] for k in fk)
        wb = sum(w[k] for k in wk)
        res["kernels"][name] = {"bytes": nb, "fetch_ratio": round(fb / nb, 4), "write_ratio": round(wb / nb, 4)}
        print("%-16s fetch %.4f  write %.4f" % (name, fb / nb, wb / nb))
    json.dump(res, open(dst, "w"), indent=1)


if __name__ == "__main__":
    main()
