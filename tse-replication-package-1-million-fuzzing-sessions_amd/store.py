"""Columnar loader: the replacement for restoring ``data/database/backup_clean.sql`` into PostgreSQL
and fetching rows through ``program/__module/dbFile.py``.

Two on-disk forms feed ``schema.Tables`` (which ``engine.Engine.upload`` streams to HBM):

* a **columnar directory** (the engine's native format): one ``.npy`` per typed column plus
  ``meta.json`` holding the text pools (project names, modules, revisions, build names), the code
  vocabularies and the corpus CSV text.  ``save_columnar`` / ``load_columnar``; numpy ``.npy`` files
  are memory-mapped on load (no pickle: ``allow_pickle=False``).
* a **CSV export directory** as written by PostgreSQL ``\\copy <table> TO '<table>.csv' CSV HEADER``
  for ``buildlog_data``, ``total_coverage``, ``issues`` and ``project_info`` (column names as in
  ``queries1.py:18-55,120-129,289-295``), plus ``project_corpus_analysis.csv``
  (``user_corpus.py:225-233``).  ``from_csv_dir`` dictionary-encodes ``project`` in byte order,
  maps ``build_type`` / ``result`` / ``status`` to the schema codes, parses timestamps to int64
  microseconds (naive), and keeps NULLs as validity bits / ``TS_NULL``.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional

import numpy as np

from .schema import (BUILD_TYPES, CODE_NULL, RESULTS, STATUSES, TS_NULL, Tables)

_NUMERIC = ["b_project", "b_type", "b_result", "b_time", "b_modules", "b_revisions",
            "c_project", "c_date", "c_coverage", "c_coverage_valid", "c_covered", "c_covered_valid",
            "c_total", "c_total_valid", "i_number", "i_project", "i_rts", "i_status", "i_new_id",
            "pi_project", "pi_first_commit"]


def save_columnar(t: Tables, path: str) -> None:
    os.makedirs(path, exist_ok=True)
    for name in _NUMERIC:
        np.save(os.path.join(path, name + ".npy"), np.ascontiguousarray(getattr(t, name)), allow_pickle=False)
    meta = {"projects": t.projects, "modules_pool": t.modules_pool, "revisions_pool": t.revisions_pool,
            "b_name": [None if x is None else str(x) for x in t.b_name.tolist()],
            "build_types": t.build_types, "results": t.results, "statuses": t.statuses,
            "corpus_csv": t.corpus_csv}
    with open(os.path.join(path, "meta.json"), "w") as f:
        json.dump(meta, f)


def load_columnar(path: str, mmap: bool = True) -> Tables:
    with open(os.path.join(path, "meta.json")) as f:
        meta = json.load(f)
    cols = {name: np.load(os.path.join(path, name + ".npy"), mmap_mode="r" if mmap else None, allow_pickle=False)
            for name in _NUMERIC}
    names = np.empty(len(meta["b_name"]), dtype=object)
    names[:] = meta["b_name"]
    return Tables(projects=meta["projects"], modules_pool=meta["modules_pool"],
                  revisions_pool=meta["revisions_pool"], b_name=names, build_types=meta["build_types"],
                  results=meta["results"], statuses=meta["statuses"], corpus_csv=meta["corpus_csv"],
                  **{k: np.asarray(v) for k, v in cols.items()})


# ---------------------------------------------------------------------------------- CSV ingest
def _ts(series) -> np.ndarray:
    """Naive timestamps (text) -> int64 microseconds; NULL -> TS_NULL."""
    import pandas as pd
    dt = pd.to_datetime(series, errors="coerce", format="mixed")
    out = np.full(len(series), TS_NULL, dtype=np.int64)
    ok = dt.notna().to_numpy()
    if ok.any():
        v = dt[ok]
        if getattr(v.dt, "tz", None) is not None:
            v = v.dt.tz_localize(None)
        out[ok] = v.astype("datetime64[us]").astype(np.int64).to_numpy()
    return out


def _codes(series, vocab: List[str]) -> np.ndarray:
    """Text -> codes into vocab (extended in place with unseen strings); NULL -> CODE_NULL."""
    out = np.full(len(series), CODE_NULL, dtype=np.uint8)
    index = {s: i for i, s in enumerate(vocab)}
    for k, s in enumerate(series.tolist()):
        if s is None or (isinstance(s, float) and np.isnan(s)):
            continue
        if s not in index:
            index[s] = len(vocab)
            vocab.append(s)
        if index[s] >= CODE_NULL:
            raise ValueError("more than 254 distinct codes")
        out[k] = index[s]
    return out


def _pool(series):
    """Text column -> (int32 ids, pool); NULL -> -1."""
    pool: List[Optional[str]] = []
    index: Dict[str, int] = {}
    ids = np.full(len(series), -1, dtype=np.int32)
    for k, s in enumerate(series.tolist()):
        if s is None or (isinstance(s, float) and np.isnan(s)):
            continue
        if s not in index:
            index[s] = len(pool)
            pool.append(s)
        ids[k] = index[s]
    return ids, pool


def _nullable_int(series):
    import pandas as pd
    v = pd.to_numeric(series, errors="coerce")
    ok = v.notna().to_numpy()
    out = np.zeros(len(series), dtype=np.int64)
    out[ok] = v[ok].astype(np.int64).to_numpy()
    return out, ok


def from_csv_dir(path: str, corpus_csv: Optional[str] = None) -> Tables:
    """Ingest PostgreSQL CSV exports (see module docstring) into columnar ``Tables``."""
    import pandas as pd
    rd = lambda name: pd.read_csv(os.path.join(path, name + ".csv"), dtype=str, keep_default_na=False,  # noqa: E731
                                  na_values=[""])
    b, c, i = rd("buildlog_data"), rd("total_coverage"), rd("issues")
    pi = rd("project_info") if os.path.exists(os.path.join(path, "project_info.csv")) else None
    names = set(b["project"].dropna()) | set(c["project"].dropna()) | set(i["project"].dropna())
    if pi is not None:
        names |= set(pi["project"].dropna())
    projects = sorted(names, key=lambda s: s.encode())  # byte order == ORDER BY under C collation
    pid = {n: k for k, n in enumerate(projects)}
    enc = lambda s: np.array([pid[x] for x in s.tolist()], dtype=np.uint32)  # noqa: E731
    build_types, results, statuses = list(BUILD_TYPES), list(RESULTS), list(STATUSES)
    b_mod, mod_pool = _pool(b["modules"])
    b_rev, rev_pool = _pool(b["revisions"])
    # correctly rounded text -> double (pandas' fast parser is not round-trip exact)
    cov = pd.Series([float(x) if isinstance(x, str) else np.nan for x in c["coverage"].tolist()])
    cvd, cvd_ok = _nullable_int(c["covered_line"])
    tot, tot_ok = _nullable_int(c["total_line"])
    names_arr = np.empty(len(b), dtype=object)
    names_arr[:] = [None if isinstance(x, float) else x for x in b["name"].tolist()]
    if corpus_csv is None:
        cp = os.path.join(path, "project_corpus_analysis.csv")
        corpus_csv = open(cp).read() if os.path.exists(cp) else ""
    return Tables(
        projects=projects,
        b_project=enc(b["project"]), b_type=_codes(b["build_type"], build_types),
        b_result=_codes(b["result"], results), b_time=_ts(b["timecreated"]), b_modules=b_mod,
        b_revisions=b_rev, b_name=names_arr, modules_pool=mod_pool, revisions_pool=rev_pool,
        c_project=enc(c["project"]), c_date=_ts(c["date"]),
        c_coverage=np.nan_to_num(cov.to_numpy(dtype=np.float64), nan=0.0), c_coverage_valid=cov.notna().to_numpy(),
        c_covered=cvd, c_covered_valid=cvd_ok, c_total=tot, c_total_valid=tot_ok,
        i_number=pd.to_numeric(i["number"]).to_numpy(dtype=np.int64), i_project=enc(i["project"]),
        i_rts=_ts(i["rts"]), i_status=_codes(i["status"], statuses),
        i_new_id=_nullable_int(i["new_id"])[0] if "new_id" in i else np.zeros(len(i), np.int64),
        pi_project=enc(pi["project"]) if pi is not None else np.zeros(0, np.uint32),
        pi_first_commit=_ts(pi["first_commit_datetime"]) if pi is not None else np.zeros(0, np.int64),
        build_types=build_types, results=results, statuses=statuses, corpus_csv=corpus_csv)


def to_csv_dir(t: Tables, path: str) -> None:
    """Write ``Tables`` as PostgreSQL-style CSV exports (used by tests and to seed a database)."""
    import csv
    from .schema import us_to_dt
    os.makedirs(path, exist_ok=True)

    def ts(v):
        return "" if v == TS_NULL else str(us_to_dt(v))

    def code(vocab, v):
        return "" if v == CODE_NULL else vocab[v]

    def pool(p, k):
        return "" if k < 0 or p[k] is None else p[k]

    with open(os.path.join(path, "buildlog_data.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["name", "project", "build_type", "result", "timecreated", "modules", "revisions"])
        for k in range(len(t.b_project)):
            w.writerow([t.b_name[k] or "", t.projects[t.b_project[k]], code(t.build_types, t.b_type[k]),
                        code(t.results, t.b_result[k]), ts(t.b_time[k]), pool(t.modules_pool, t.b_modules[k]),
                        pool(t.revisions_pool, t.b_revisions[k])])
    with open(os.path.join(path, "total_coverage.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["project", "date", "coverage", "covered_line", "total_line"])
        for k in range(len(t.c_project)):
            w.writerow([t.projects[t.c_project[k]], ts(t.c_date[k]),
                        repr(float(t.c_coverage[k])) if t.c_coverage_valid[k] else "",
                        int(t.c_covered[k]) if t.c_covered_valid[k] else "",
                        int(t.c_total[k]) if t.c_total_valid[k] else ""])
    with open(os.path.join(path, "issues.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["number", "project", "rts", "status", "new_id"])
        for k in range(len(t.i_project)):
            w.writerow([int(t.i_number[k]), t.projects[t.i_project[k]], ts(t.i_rts[k]),
                        code(t.statuses, t.i_status[k]), int(t.i_new_id[k])])
    with open(os.path.join(path, "project_info.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["project", "first_commit_datetime"])
        for k in range(len(t.pi_project)):
            w.writerow([t.projects[t.pi_project[k]], ts(t.pi_first_commit[k])])
    with open(os.path.join(path, "project_corpus_analysis.csv"), "w") as f:
        f.write(t.corpus_csv)
