"""Generate golden fixtures by running the UNMODIFIED reference scripts (this container only).

Recipe: the reference's six ``rq*.py`` scripts are executed with
``runpy`` from a scratch working directory whose ``program/`` is a symlink to
``/root/reference/program``.  ``dbFile.DB`` is replaced by a fake backed by sqlite3
(``PARSE_DECLTYPES`` so TIMESTAMP columns come back as ``datetime``), ``psycopg2`` and
``seaborn`` are stubbed, and ``savefig``/``show`` are no-ops (figures are not parity
targets).  Inputs are the deterministic synthetic tables of ``tse_amd.synth`` (the
fixture records their sha256 fingerprint); outputs - every CSV the scripts write plus
stdout/stderr - are copied into ``tests/golden/<case>/``.  Nothing from the reference is
copied into the repository: only its outputs on our inputs.

Usage:  python tests/golden/make_goldens.py [tiny medium ...]
"""
from __future__ import annotations

import gzip
import json
import os
import shutil
import sqlite3
import subprocess
import sys
import tempfile
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

import tse_amd.synth as synth  # noqa: E402
sys.path.insert(0, os.path.dirname(HERE))
import null_edges  # noqa: E402
from tse_amd.schema import CODE_NULL, TS_NULL, us_to_dt  # noqa: E402

REFERENCE = "/root/reference"
SCRIPTS = ["rq1_detection_rate", "rq2_coverage_count", "rq2_coverage_and_added",
           "rq3_diff_coverage_at_detection", "rq4a_bug", "rq4b_coverage"]

FAKE_DB = '''
import os, sqlite3
class DB:
    def __init__(self, database=None, user=None, password=None, host=None, port=None):
        self.connection = None
        self.cursor = None
    def connect(self):
        self.connection = sqlite3.connect(os.environ["FAKE_DB"], detect_types=sqlite3.PARSE_DECLTYPES)
        self.cursor = self.connection.cursor()
    def executeQuery(self, queryType, query):
        if queryType.lower() == "select":
            self.cursor.execute(query)
            return self.cursor.fetchall()
        self.cursor.execute(query)
        self.connection.commit()
    def closeConnection(self):
        self.connection.close()
'''

SEABORN_STUB = '''
import matplotlib.pyplot as plt
def set_theme(*a, **k): pass
def set_style(*a, **k): pass
def despine(*a, **k): pass
def color_palette(*a, **k): return [(0.1 * i, 0.5, 0.5) for i in range(10)]
def histplot(*a, **k): return plt.gca()
def boxplot(*a, **k): return plt.gca()
def violinplot(*a, **k): return plt.gca()
'''

RUNNER = '''
import sys, runpy, matplotlib
matplotlib.use("Agg")
import matplotlib.pyplot as plt, matplotlib.figure
plt.savefig = lambda *a, **k: None
plt.show = lambda *a, **k: None
matplotlib.figure.Figure.savefig = lambda *a, **k: None
sys.path.insert(0, "fake")
runpy.run_path("program/research_questions/%s.py", run_name="__main__")
'''


def _ts(us):
    return None if us == TS_NULL else us_to_dt(us).strftime("%Y-%m-%d %H:%M:%S.%f")


def write_sqlite(t, path):
    con = sqlite3.connect(path)
    cur = con.cursor()
    cur.executescript('''
        CREATE TABLE total_coverage(project TEXT, date TIMESTAMP, coverage REAL, covered_line INTEGER, total_line INTEGER);
        CREATE TABLE buildlog_data(name TEXT, project TEXT, build_type TEXT, result TEXT, timecreated TIMESTAMP, modules TEXT, revisions TEXT);
        CREATE TABLE issues(number INTEGER, project TEXT, rts TIMESTAMP, status TEXT, new_id INTEGER, severity TEXT, crash_type TEXT);
        CREATE TABLE project_info(project TEXT, first_commit_datetime TIMESTAMP);
    ''')
    P = t.projects
    cur.executemany("INSERT INTO total_coverage VALUES (?,?,?,?,?)", [
        (P[p], _ts(d), float(c) if cv else None, int(a) if av else None, int(b) if bv else None)
        for p, d, c, cv, a, av, b, bv in zip(t.c_project.tolist(), t.c_date.tolist(), t.c_coverage.tolist(),
                                             t.c_coverage_valid.tolist(), t.c_covered.tolist(),
                                             t.c_covered_valid.tolist(), t.c_total.tolist(), t.c_total_valid.tolist())])
    cur.executemany("INSERT INTO buildlog_data VALUES (?,?,?,?,?,?,?)", [
        (n, P[p], t.build_types[bt], None if r == CODE_NULL else t.results[r], _ts(tm),
         None if m < 0 else t.modules_pool[m], None if v < 0 else t.revisions_pool[v])
        for n, p, bt, r, tm, m, v in zip(t.b_name.tolist(), t.b_project.tolist(), t.b_type.tolist(),
                                         t.b_result.tolist(), t.b_time.tolist(), t.b_modules.tolist(),
                                         t.b_revisions.tolist())])
    cur.executemany("INSERT INTO issues VALUES (?,?,?,?,?,?,?)", [
        (n, P[p], _ts(r), t.statuses[s], nid, "High", "Heap-buffer-overflow")
        for n, p, r, s, nid in zip(t.i_number.tolist(), t.i_project.tolist(), t.i_rts.tolist(),
                                   t.i_status.tolist(), t.i_new_id.tolist())])
    cur.executemany("INSERT INTO project_info VALUES (?,?)", [
        (P[p], _ts(f)) for p, f in zip(t.pi_project.tolist(), t.pi_first_commit.tolist())])
    cur.executescript('''
        CREATE INDEX ix_b ON buildlog_data(project, build_type, timecreated);
        CREATE INDEX ix_c ON total_coverage(project, date);
        CREATE INDEX ix_i ON issues(project, rts);
    ''')
    con.commit()
    con.close()


def prune_change_analysis(out_dir, keep=6):
    """Per-project change_analysis/<p>.csv files are row subsets of the combined file: keep a
    few verbatim and a sha256 manifest of all of them (names + exact bytes are still checked)."""
    import hashlib
    d = os.path.join(out_dir, "result_data", "rq3", "change_analysis")
    if not os.path.isdir(d):
        return
    man = {}
    for k, fn in enumerate(sorted(os.listdir(d))):
        path = os.path.join(d, fn)
        if fn.endswith(".gz"):
            with gzip.open(path, "rb") as f:
                data = f.read()
            name = fn[:-3]
        else:
            with open(path, "rb") as f:
                data = f.read()
            name = fn
        man[name] = hashlib.sha256(data).hexdigest()
        if k >= keep:
            os.remove(path)
    with open(os.path.join(out_dir, "result_data", "rq3", "change_analysis_manifest.json"), "w") as f:
        json.dump(man, f, indent=0, sort_keys=True)


def run_case(case: str, out_root: str):
    base, edge = null_edges.split(case)
    cfg = synth.config(base)
    t = synth.generate(cfg)
    scripts = SCRIPTS
    if edge:  # NULL line-count edges (tests/null_edges.py): one changed row, two scripts
        t = null_edges.apply(t, edge)
        scripts = null_edges.SCRIPTS
    work = tempfile.mkdtemp(prefix=f"fzgold_{case}_")
    os.symlink(os.path.join(REFERENCE, "program"), os.path.join(work, "program"))
    for d in ("fake", "stubs/psycopg2", "data/processed_data/csv"):
        os.makedirs(os.path.join(work, d), exist_ok=True)
    with open(os.path.join(work, "fake/dbFile.py"), "w") as f:
        f.write(FAKE_DB)
    with open(os.path.join(work, "stubs/psycopg2/__init__.py"), "w") as f:
        f.write("def connect(*a, **k):\n    raise RuntimeError('psycopg2 stub')\n")
    with open(os.path.join(work, "stubs/psycopg2/extras.py"), "w") as f:
        f.write("def execute_values(*a, **k):\n    raise RuntimeError('psycopg2 stub')\n")
    with open(os.path.join(work, "stubs/seaborn.py"), "w") as f:
        f.write(SEABORN_STUB)
    with open(os.path.join(work, "data/processed_data/csv/project_corpus_analysis.csv"), "w") as f:
        f.write(t.corpus_csv)
    db = os.path.join(work, "fake.db")
    write_sqlite(t, db)

    out_dir = os.path.join(out_root, case)
    shutil.rmtree(out_dir, ignore_errors=True)
    os.makedirs(out_dir)
    meta = {"case": case, "config": {k: (list(v) if isinstance(v, tuple) else v) for k, v in cfg.__dict__.items()},
            "fingerprint": null_edges.fingerprint(t) if edge else synth.table_fingerprint(t), "scripts": {}}
    env = dict(os.environ, FAKE_DB=db, MPLBACKEND="Agg", PYTHONDONTWRITEBYTECODE="1",
               PYTHONPATH=os.path.join(work, "stubs"), PYTHONHASHSEED="0")
    for s in scripts:
        t0 = time.time()
        proc = subprocess.run([sys.executable, "-B", "-c", RUNNER % s], cwd=work, env=env,
                              capture_output=True, text=True)
        dt = time.time() - t0
        sd = os.path.join(out_dir, s)
        os.makedirs(sd)
        with open(os.path.join(sd, "stdout.txt"), "w") as f:
            f.write(proc.stdout.replace(work, "<WORK>"))
        # stderr: keep logging lines, drop tqdm progress bars
        err = [ln for ln in proc.stderr.splitlines() if "it/s]" not in ln and "s/it]" not in ln and "%|" not in ln]
        with open(os.path.join(sd, "stderr.txt"), "w") as f:
            f.write(("\n".join(err) + "\n").replace(work, "<WORK>"))
        meta["scripts"][s] = {"returncode": proc.returncode, "seconds": round(dt, 2)}
        print(f"[{case}] {s}: rc={proc.returncode} {dt:.1f}s", flush=True)
    # collect every CSV output
    res = os.path.join(work, "data/result_data")
    for root, _, files in os.walk(res):
        for fn in files:
            if fn.endswith(".csv"):
                src = os.path.join(root, fn)
                rel = os.path.relpath(src, res)
                dst = os.path.join(out_dir, "result_data", rel)
                os.makedirs(os.path.dirname(dst), exist_ok=True)
                if os.path.getsize(src) > 64 * 1024:   # keep the fixture tree small
                    with open(src, "rb") as fi, gzip.open(dst + ".gz", "wb", compresslevel=9) as fo:
                        shutil.copyfileobj(fi, fo)
                else:
                    shutil.copy(src, dst)
    prune_change_analysis(out_dir)
    with open(os.path.join(out_dir, "meta.json"), "w") as f:
        json.dump(meta, f, indent=1)
    shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    if not os.path.isdir(REFERENCE):
        sys.exit("the reference is not present: goldens can only be regenerated in the build container")
    cases = sys.argv[1:] or ["tiny", "medium"]
    if cases == ["edges"]:
        cases = ["tiny+" + e for e in null_edges.EDGES]
    for c in cases:
        run_case(c, HERE)
