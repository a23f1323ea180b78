"""Drop-in runners for the six reference scripts (``program/research_questions/*.py``).

``run(name, ...)`` does what ``python3 program/research_questions/<name>.py`` does in the
reference (``run_all_analysis.sh:13-46``): compute the analysis - here on the GPU through
``libfz`` - then print the same stdout lines, emit the same log records (RQ4 scripts use
``logging.basicConfig(level=INFO, format='%(asctime)s [%(levelname)s] %(message)s')``,
``rq4a_bug.py:23-28``) and write the same files under ``<cwd>/data/result_data``.

Figures (PDF) are host-side matplotlib in the reference and not part of the hot path; the
renderer records what each figure would contain (``Rendered.figures``) but this runner does not
draw them (``compute`` mode of SURVEY.md 7).
"""
from __future__ import annotations

import logging
import os
import sys
from typing import Optional

from .. import engine as E
from ..schema import Tables
from . import compute, render

SCRIPTS = ["rq1_detection_rate", "rq2_coverage_and_added", "rq2_coverage_count",
           "rq3_diff_coverage_at_detection", "rq4a_bug", "rq4b_coverage"]   # run_all_analysis.sh order


def data_source() -> str:
    """Where the drop-ins read the session tables: $FZ_DATA (a columnar directory written by
    ``store.save_columnar``, a directory of PostgreSQL CSV exports, or the plain-format dump
    ``data/database/backup_clean.sql`` itself), default data/columnar."""
    return os.environ.get("FZ_DATA", os.path.join("data", "columnar"))


def load_tables(path: Optional[str] = None) -> Tables:
    from .. import store
    path = path or data_source()
    if os.path.isfile(path):
        return store.from_pg_dump(path)
    if os.path.exists(os.path.join(path, "meta.json")):
        return store.load_columnar(path)
    if os.path.exists(os.path.join(path, "buildlog_data.csv")):
        return store.from_csv_dir(path)
    raise FileNotFoundError(f"no session tables at {path!r} (set FZ_DATA to a columnar or CSV-export directory or a pg_dump .sql file)")


def analyse(name: str, eng: E.Engine, t: Tables, cwd: str) -> render.Rendered:
    if name == "rq1_detection_rate":
        return render.rq1(compute.rq1(eng), t)
    if name == "rq2_coverage_count":
        return render.rq2_count(compute.rq2_count(eng), t)
    if name == "rq2_coverage_and_added":
        return render.rq2_add(compute.rq2_add(eng), t)
    if name == "rq3_diff_coverage_at_detection":
        return render.rq3(compute.rq3(eng), t)
    if name == "rq4a_bug":
        return render.rq4a(compute.rq4a(eng), t, cwd=cwd)
    if name == "rq4b_coverage":
        b = compute.rq4b_buffers(eng)
        compute.rq4b_launch(eng, b)
        n_elig = int(b.host("eligible", eng.tables.fz.n_projects).sum())
        return render.rq4b(compute.rq4b_collect(eng, b), t, n_eligible=n_elig, cwd=cwd)
    raise ValueError(f"unknown script {name!r}")


def emit(r: render.Rendered, cwd: str, out=None) -> None:
    """Write files (relative keys under cwd), stdout lines and log records like the reference."""
    out = out or sys.stdout
    for path, data in r.files.items():
        full = path if os.path.isabs(path) else os.path.join(cwd, path)
        os.makedirs(os.path.dirname(full), exist_ok=True)
        with open(full, "wb") as f:
            f.write(data)
    for line in r.preamble_stderr:
        print(line, file=sys.stderr)
    if r.log:
        log = logging.getLogger("fz.rq")
        if not logging.getLogger().handlers:
            logging.basicConfig(level=logging.INFO, format="%(asctime)s [%(levelname)s] %(message)s")
        for lvl, msg in r.log:
            log.log(getattr(logging, lvl), msg)
    out.write(r.text())
    out.flush()


def run(name: str, eng: Optional[E.Engine] = None, t: Optional[Tables] = None, cwd: Optional[str] = None):
    cwd = cwd or os.getcwd()
    t = t if t is not None else load_tables()
    own = eng is None
    if own:
        eng = E.Engine(0)
    if eng.tables is None or eng.tables.host is not t:
        eng.upload(t)
        eng.build_store()
    r = analyse(name, eng, t, cwd)
    emit(r, cwd)
    if own:
        eng.close()
    return r


def main_all(argv=None) -> int:
    """run_all_analysis.sh: the six scripts in order, one engine, tables loaded once."""
    t = load_tables()
    eng = E.Engine(0)
    eng.upload(t)
    eng.build_store()
    for k, name in enumerate(SCRIPTS, 1):
        print(f"\n[{k}/6] Running {name} ...")
        run(name, eng, t)
    eng.close()
    return 0


if __name__ == "__main__":
    sys.exit(main_all())
