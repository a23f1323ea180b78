"""Drop-in runners for the six reference scripts (``program/research_questions/*.py``).

``run(name, ...)`` does what ``python3 program/research_questions/<name>.py`` does in the
reference (``run_all_analysis.sh:13-46``): compute the analysis - here on the GPU through
``libfz`` - then print the same stdout lines, emit the same log records (RQ4 scripts use
``logging.basicConfig(level=INFO, format='%(asctime)s [%(levelname)s] %(message)s')``,
``rq4a_bug.py:23-28``) and write the same files under ``<cwd>/data/result_data``.

Figures (PDF) are host-side matplotlib in the reference and not part of the hot path: the runner
hands each script's figure data to a side process (``rq/figures.py``) after the tables and stdout
are written, at the reference's paths.  ``FZ_FIGURES=0`` skips them (the ``compute`` mode of
SURVEY.md 7).
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


DUMP = os.path.join("data", "database", "backup_clean.sql")   # README.md:14-15 (restored into PG there)
COLUMNAR = os.path.join("data", "columnar")


def data_source() -> str:
    """Where the drop-ins read the session tables: $FZ_DATA (a columnar directory written by
    ``store.save_columnar``, a directory of PostgreSQL CSV exports, or the plain-format dump
    itself); else ./data/columnar; else the reference's dump ./data/database/backup_clean.sql."""
    env = os.environ.get("FZ_DATA")
    if env:
        return env
    if not os.path.exists(os.path.join(COLUMNAR, "meta.json")) and os.path.isfile(DUMP):
        return DUMP
    return COLUMNAR


def load_tables(path: Optional[str] = None) -> Tables:
    from .. import store
    path = path or data_source()
    if os.path.isfile(path):
        t = store.from_pg_dump(path)
        if path == DUMP and not os.environ.get("FZ_DATA"):
            store.save_columnar(t, COLUMNAR)  # the next scripts map the columns instead of re-parsing
        return t
    if os.path.exists(os.path.join(path, "meta.json")):
        return store.load_columnar(path)
    if os.path.exists(os.path.join(path, "buildlog_data.csv")):
        return store.from_csv_dir(path)
    raise FileNotFoundError(f"no session tables at {path!r} (set FZ_DATA to a columnar or CSV-export directory or a pg_dump .sql file)")


def analyse(name: str, eng: E.Engine, t: Tables, cwd: str) -> render.Rendered:
    return analyse_result(name, eng, t, cwd)[1]


def analyse_result(name: str, eng: E.Engine, t: Tables, cwd: str):
    """(result object, rendered output) of one script."""
    if name == "rq1_detection_rate":
        r = compute.rq1(eng)
        return r, render.rq1(r, t)
    if name == "rq2_coverage_count":
        r = compute.rq2_count(eng)
        return r, render.rq2_count(r, t)
    if name == "rq2_coverage_and_added":
        r = compute.rq2_add(eng)
        return r, render.rq2_add(r, t)
    if name == "rq3_diff_coverage_at_detection":
        r = compute.rq3(eng)
        return r, render.rq3(r, t)
    if name == "rq4a_bug":
        r = compute.rq4a(eng)
        return r, render.rq4a(r, t, cwd=cwd)
    if name == "rq4b_coverage":
        b = compute.rq4b_buffers(eng)
        compute.rq4b_launch(eng, b)
        n_elig = int(b.host("eligible", eng.tables.fz.n_projects).sum())
        r = compute.rq4b_collect(eng, b)
        return r, render.rq4b(r, t, n_eligible=n_elig, cwd=cwd)
    raise ValueError(f"unknown script {name!r}")


def figures_enabled() -> bool:
    return os.environ.get("FZ_FIGURES", "1") not in ("0", "", "no", "false")


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


def run(name: str, eng: Optional[E.Engine] = None, t: Optional[Tables] = None, cwd: Optional[str] = None,
        figures: Optional[bool] = None, pending: Optional[list] = None):
    """One drop-in script.  Figures are drawn by a side process started after the outputs are
    written; it is joined before returning unless the caller collects it in `pending`."""
    cwd = cwd or os.getcwd()
    t = t if t is not None else load_tables()
    own = eng is None
    if own:
        eng = E.Engine(0)
    if eng.tables is None or eng.tables.host is not t:
        eng.upload(t)
        eng.build_store()
    res, r = analyse_result(name, eng, t, cwd)
    emit(r, cwd)
    if own:
        eng.close()
    if figures if figures is not None else figures_enabled():
        from . import figures as F
        procs = F.draw_in_side_process([F.spec(name, res, t)], cwd, workers=F.figure_workers())
        if pending is not None:
            pending.extend(procs)
        else:
            for proc in procs:
                proc.join()
    return r


def main_one(name: str) -> int:
    """`python3 program/research_questions/<name>.py`: one script, argument-less (the tables from
    data_source(), outputs under the working directory)."""
    run(name)
    return 0


def main_all(argv=None) -> int:
    """run_all_analysis.sh: the six scripts in order, one engine, tables loaded once; the figure
    processes run beside the next scripts and are joined at the end."""
    t = load_tables()
    eng = E.Engine(0)
    eng.upload(t)
    eng.build_store()
    pending = []
    for k, name in enumerate(SCRIPTS, 1):
        print(f"\n[{k}/6] Running {name} ...")
        run(name, eng, t, pending=pending)
    eng.close()
    for p in pending:
        p.join()
    return 0 if all(p.exitcode == 0 for p in pending) else 1


if __name__ == "__main__":
    sys.exit(main_all())
