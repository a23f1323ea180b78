"""Build the reference-held known-answer fixtures under tests/golden/shipped/ (run in the build
container only; /root/reference does not exist on the GPU box).

The reference ships its real-data OUTPUTS (data/result_data/**) but not its inputs.  This script
turns some of them into test vectors (SURVEY.md 4, 8(c) inventory items 2-6):

* rq1_detection_rate_stats.csv, rq4_g1_g2_detection_trend.csv, rq4_gc_introduction_iteration.csv
  and detected_coverage_changes.csv are copied verbatim: they are the inputs of the finishing
  statistics (rq1_detection_rate.py:243-268, rq4a_bug.py:156-207,698-780,246-299,
  rq3_diff_coverage_at_detection.py:25-66,321-335) whose printed results the tests check.
* data/result_data/rq3/change_analysis/<project>.csv (854 files, 270,347 rows) are inverted into
  the session tables that produce them through rq2_coverage_and_added.py:73-238: per project the
  Coverage builds that end / start each pair of consecutive (modules, revisions) runs, and the
  total_coverage rows on the dates the pairs join on.  The tests regenerate the files from those
  tables (GPU path and CPU oracle) and require them byte for byte.  The revisions text (two 40-hex
  hashes per cell, a pure pass-through column that only decides where runs start) is replaced by
  a stable id "{r<k>}" in both the tables and the expected files, which keeps the fixture small.

Output: shipped/*.csv (copies), shipped/change_analysis.npz (tables), shipped/change_analysis.json
(project names, modules pool, per-file row count and sha256 of the expected bytes),
shipped/rq3_detected_stdout.txt: what the reference's own print_summary_statistics
(rq3_diff_coverage_at_detection.py:25-66) and its Anderson-Darling prints (:329-333) write for the
shipped detected sample - the UNMODIFIED reference module is loaded with runpy (not as __main__,
so main() does not run) under the same stubs as tests/golden/make_goldens.py.
"""
import csv
import datetime as dt
import hashlib
import io
import json
import os
import shutil
import sys

import numpy as np

REF = "/root/reference/data/result_data"
HERE = os.path.dirname(os.path.abspath(__file__))
EPOCH = dt.datetime(1970, 1, 1)
DAY = 86_400_000_000


def us(s):
    d = dt.datetime.strptime(s, "%Y-%m-%d %H:%M:%S.%f" if "." in s else "%Y-%m-%d %H:%M:%S")
    x = d - EPOCH
    return (x.days * 86400 + x.seconds) * 1_000_000 + x.microseconds


def copy_csvs():
    for rel in ("rq1/rq1_detection_rate_stats.csv", "rq4/bug/rq4_g1_g2_detection_trend.csv",
                "rq4/bug/rq4_gc_introduction_iteration.csv", "rq3/detected_coverage_changes.csv"):
        shutil.copyfile(os.path.join(REF, rel), os.path.join(HERE, os.path.basename(rel)))


def invert_change_analysis():
    src = os.path.join(REF, "rq3", "change_analysis")
    names = sorted((f[:-4] for f in os.listdir(src) if f.endswith(".csv")), key=lambda s: s.encode())
    rev_id, mod_id, mods = {}, {}, []
    b_proj, b_time, b_mod, b_rev = [], [], [], []
    c_proj, c_day, c_cvd, c_tot, c_cvd_ok, c_tot_ok = [], [], [], [], [], []
    files = {}
    limit = us("2025-01-08 00:00:00")

    def rid(s):
        return rev_id.setdefault(s, len(rev_id))

    def mid(s):
        if s not in mod_id:
            mod_id[s] = len(mods)
            mods.append(s)
        return mod_id[s]

    for p, name in enumerate(names):
        with open(os.path.join(src, name + ".csv"), newline="") as f:
            rows = list(csv.reader(f))
        header, rows = rows[0], rows[1:]
        assert rows, name
        # builds: end of run 0, then for each pair k: start of run k+1 and (if later) its end
        builds = [(us(rows[0][1]), rows[0][2], rows[0][3])]
        for k, r in enumerate(rows):
            start = (us(r[4]), r[5], r[6])
            end = (us(rows[k + 1][1]), rows[k + 1][2], rows[k + 1][3]) if k + 1 < len(rows) else start
            assert (start[1], start[2]) == (end[1], end[2]), (name, k)
            assert builds[-1][0] < start[0] <= end[0] < limit, (name, k)
            builds.append(start)
            if end[0] != start[0]:
                builds.append(end)
        for t, m, rv in builds:
            b_proj.append(p)
            b_time.append(t)
            b_mod.append(mid(m))
            b_rev.append(rid(rv))
        # coverage rows on the joined dates (both cells nan -> no row on that date)
        cov = {}
        for r in rows:
            for ts, cv, tt in ((r[1], r[7], r[8]), (r[4], r[9], r[10])):
                day = us(ts) // DAY * DAY
                assert cov.setdefault(day, (cv, tt)) == (cv, tt), (name, ts)
        for day in sorted(cov):
            cv, tt = cov[day]
            if cv == "nan" and tt == "nan":
                continue
            c_proj.append(p)
            c_day.append(day)
            c_cvd.append(0 if cv == "nan" else int(float(cv)))
            c_tot.append(0 if tt == "nan" else int(float(tt)))
            c_cvd_ok.append(cv != "nan")
            c_tot_ok.append(tt != "nan")
        # expected bytes: the shipped file with each revisions cell mapped to its id
        buf = io.StringIO(newline="")
        w = csv.writer(buf)
        w.writerow(header)
        for r in rows:
            r = list(r)
            r[3] = "{r%d}" % rid(r[3])
            r[6] = "{r%d}" % rid(r[6])
            w.writerow(r)
        data = buf.getvalue().encode()
        files[name] = {"rows": len(rows), "sha256": hashlib.sha256(data).hexdigest()}
    assert min(b_time) > us("2001-01-01 00:00:00")  # the fixture loader's filler days are in 2000
    np.savez_compressed(
        os.path.join(HERE, "change_analysis.npz"),
        b_project=np.asarray(b_proj, np.uint32), b_time=np.asarray(b_time, np.int64),
        b_modules=np.asarray(b_mod, np.int32), b_revisions=np.asarray(b_rev, np.int32),
        c_project=np.asarray(c_proj, np.uint32), c_date=np.asarray(c_day, np.int64),
        c_covered=np.asarray(c_cvd, np.int64), c_total=np.asarray(c_tot, np.int64),
        c_covered_valid=np.asarray(c_cvd_ok, bool), c_total_valid=np.asarray(c_tot_ok, bool))
    with open(os.path.join(HERE, "change_analysis.json"), "w") as f:
        json.dump({"source": "data/result_data/rq3/change_analysis/*.csv (reference)",
                   "projects": names, "modules_pool": mods, "n_revisions": len(rev_id),
                   "files": files}, f, indent=0)
    print(f"{len(names)} projects, {len(b_time)} builds, {len(c_day)} coverage rows, "
          f"{sum(v['rows'] for v in files.values())} change rows")


RQ3_SNIPPET = r'''
import csv, sys, runpy, matplotlib
matplotlib.use("Agg")
sys.path.insert(0, "fake")
from scipy import stats
g = runpy.run_path("program/research_questions/rq3_diff_coverage_at_detection.py", run_name="kat")
rows = list(csv.reader(open(sys.argv[1], newline="")))[1:]
pct = [float(r[0]) for r in rows]
tot = [int(r[2]) for r in rows]
g["print_summary_statistics"](pct, "Detected")
g["print_summary_statistics"](tot, "Detected Total")
r = stats.anderson(pct, dist="norm")
print("Detected")
print("Test statistic (A\u00b2):", r.statistic)
print("Critical values:", r.critical_values)
print("Significance levels (%):", r.significance_level)
'''


def reference_rq3_summary():
    import subprocess
    import tempfile
    sys.path.insert(0, os.path.dirname(HERE))
    import make_goldens as mg
    with tempfile.TemporaryDirectory() as work:
        os.symlink("/root/reference/program", os.path.join(work, "program"))
        os.makedirs(os.path.join(work, "fake", "psycopg2"))
        with open(os.path.join(work, "fake", "dbFile.py"), "w") as f:
            f.write(mg.FAKE_DB)
        with open(os.path.join(work, "fake", "seaborn.py"), "w") as f:
            f.write(mg.SEABORN_STUB)
        for name in ("__init__.py", "extras.py"):
            with open(os.path.join(work, "fake", "psycopg2", name), "w") as f:
                f.write("def connect(*a, **k):\n    raise RuntimeError('no database')\n"
                        "def execute_values(*a, **k):\n    raise RuntimeError('no database')\n")
        with open(os.path.join(work, "kat.py"), "w") as f:
            f.write(RQ3_SNIPPET)
        env = dict(os.environ, MPLBACKEND="Agg", PYTHONDONTWRITEBYTECODE="1")
        out = subprocess.run([sys.executable, "-B", "kat.py", os.path.join(HERE, "detected_coverage_changes.csv")],
                             cwd=work, env=env, capture_output=True, text=True, check=True)
    with open(os.path.join(HERE, "rq3_detected_stdout.txt"), "w") as f:
        f.write(out.stdout)


if __name__ == "__main__":
    if not os.path.isdir(REF):
        sys.exit("the reference checkout is needed to (re)build these fixtures")
    copy_csvs()
    invert_change_analysis()
    reference_rq3_summary()
