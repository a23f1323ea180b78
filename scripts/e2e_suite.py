"""End-to-end drop-in suite on one GPU ("report compute-only and end-to-end"):
the six scripts of run_all_analysis.sh over a synthetic table saved as a columnar directory -
load (memory-mapped columns), upload to HBM, store build, then per script compute + render + write
(stdout to a file, CSVs under data/result_data) with the figures drawn in side processes beside the
next scripts, joined at the end.  Prints one JSON line; the reference's suite took 379 s on the
config-2 table in the build container (single-threaded Python + SQLite + figures).

usage: python scripts/e2e_suite.py [--config c2] [--no-figures] [--out DIR]"""
import argparse
import contextlib
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c2")
    ap.add_argument("--no-figures", action="store_true")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import tse_amd.synth as synth
    from tse_amd import engine as E
    from tse_amd import store
    from tse_amd.rq import scripts

    work = args.out or tempfile.mkdtemp(prefix="fz_e2e_")
    col = os.path.join(work, "data", "columnar")
    t = synth.generate(synth.config(args.config))
    store.save_columnar(t, col)
    rows = t.n_rows
    del t
    times = {}
    t0 = time.perf_counter()
    tab = scripts.load_tables(col)
    times["load_s"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    eng = E.Engine(0)
    eng.upload(tab)
    eng.build_store()
    import torch
    torch.cuda.synchronize()
    times["engine_upload_store_s"] = time.perf_counter() - t1
    pending = []
    per = {}
    with open(os.path.join(work, "stdout.txt"), "w") as out, contextlib.redirect_stdout(out):
        errors = {}
        for name in scripts.SCRIPTS:
            ts = time.perf_counter()
            try:
                scripts.run(name, eng, tab, cwd=work, figures=not args.no_figures, pending=pending)
            except Exception as e:  # noqa: BLE001 - the reference script raises the same on such a table
                # (e.g. rq1_detection_rate.py's percentage of linked issues on a table without
                # issues: ZeroDivisionError, exit status 1) - record it and go on, as run_all does
                errors[name] = type(e).__name__
            per[name] = round(time.perf_counter() - ts, 3)
    tf = time.perf_counter()
    for p in pending:
        p.join()
    times["figures_tail_s"] = time.perf_counter() - tf
    eng.close()
    total = time.perf_counter() - t0
    nfiles = sum(len(f) for _, _, f in os.walk(os.path.join(work, "data", "result_data")))
    print(json.dumps({"config": args.config, "rows": rows, "figures": not args.no_figures,
                      "total_s": round(total, 3), "rows_per_s": round(rows / total, 1),
                      **{k: round(v, 3) for k, v in times.items()}, "scripts_s": per,
                      "files_written": nfiles, "script_errors": errors, "reference_suite_s": 379.0,
                      "speedup_vs_reference": round(379.0 / total, 1)}), flush=True)


if __name__ == "__main__":
    main()
