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
* the **plain-format dump** ``data/database/backup_clean.sql`` (README.md:14-15) read directly from
  its ``COPY ... FROM stdin`` blocks by ``from_pg_dump`` (no PostgreSQL restore needed).
"""
from __future__ import annotations

import csv
import io
import json
import os
import re
from typing import Dict, List, Optional

import numpy as np

from .schema import (BUILD_TYPES, CODE_NULL, RESULTS, STATUSES, TS_NULL, Tables)

_NUMERIC = ["b_project", "b_type", "b_result", "b_time", "b_modules", "b_revisions",
            "c_project", "c_date", "c_coverage", "c_coverage_valid", "c_covered", "c_covered_valid",
            "c_total", "c_total_valid", "i_number", "i_project", "i_rts", "i_status", "i_new_id",
            "pi_project", "pi_first_commit"]


_DERIVED = {"b_group": Tables.group_key, "b_rev_canon": Tables.rev_canon}  # persisted encodings


def save_columnar(t: Tables, path: str) -> None:
    os.makedirs(path, exist_ok=True)
    for name in _NUMERIC:
        np.save(os.path.join(path, name + ".npy"), np.ascontiguousarray(getattr(t, name)), allow_pickle=False)
    for name, fn in _DERIVED.items():  # the loader's dictionary encodings, computed once here
        np.save(os.path.join(path, name + ".npy"), np.ascontiguousarray(fn(t)), allow_pickle=False)
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
    t = Tables(projects=meta["projects"], modules_pool=meta["modules_pool"],
               revisions_pool=meta["revisions_pool"], b_name=names, build_types=meta["build_types"],
               results=meta["results"], statuses=meta["statuses"], corpus_csv=meta["corpus_csv"],
               **{k: np.asarray(v) for k, v in cols.items()})
    keys = {"b_group": ("group_key", (t.b_modules, t.b_revisions, t.modules_pool, t.revisions_pool)),
            "b_rev_canon": ("rev_canon", (t.b_revisions, t.revisions_pool))}
    for name, (entry, inputs) in keys.items():  # persisted encodings (older directories: computed on use)
        f = os.path.join(path, name + ".npy")
        if os.path.exists(f):
            t.derived[entry] = (tuple(inputs), np.load(f, mmap_mode="r" if mmap else None, allow_pickle=False))
    return t


# ---------------------------------------------------------------------------------- CSV ingest
# a UTC offset after the time of day ('+00', '+02', '-05:30') as a timestamptz column dumps it
_TZ_SUFFIX = re.compile(r"^(.*\d{2}:\d{2}(?::\d{2}(?:\.\d+)?)?)[+-]\d{2}(?::?\d{2})?$")


def _ts(series) -> np.ndarray:
    """Timestamps (text) -> int64 microseconds of the printed wall-clock time; NULL -> TS_NULL.

    The analyses compare naive values (the reference's columns are `timestamp without time zone`,
    SURVEY.md 8(c)); a timestamptz dump prints each value with the server's offset, which differs
    between rows under daylight saving ('+01' / '+02'), so the offset is dropped before parsing."""
    import pandas as pd
    text = series.astype(object).where(series.notna(), None)
    text = text.map(lambda x: _TZ_SUFFIX.sub(r"\1", x) if isinstance(x, str) else x)
    dt = pd.to_datetime(text, errors="coerce", format="mixed")
    out = np.full(len(series), TS_NULL, dtype=np.int64)
    ok = dt.notna().to_numpy()
    if ok.any():
        out[ok] = dt[ok].astype("datetime64[us]").astype(np.int64).to_numpy()
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


def from_csv_dir(path: str, corpus_csv: Optional[str] = None, project_order=None) -> Tables:
    """Ingest PostgreSQL CSV exports (see module docstring) into columnar ``Tables``.
    ``project_order``: see ``_from_frames``."""
    import pandas as pd
    rd = lambda name: pd.read_csv(os.path.join(path, name + ".csv"), dtype=str, keep_default_na=False,  # noqa: E731
                                  na_values=[""])
    pi = rd("project_info") if os.path.exists(os.path.join(path, "project_info.csv")) else None
    if corpus_csv is None:
        cp = os.path.join(path, "project_corpus_analysis.csv")
        corpus_csv = open(cp).read() if os.path.exists(cp) else ""
    return _from_frames(rd("buildlog_data"), rd("total_coverage"), rd("issues"), pi, corpus_csv, project_order)


def _from_frames(b, c, i, pi, corpus_csv: str, project_order=None) -> Tables:
    """Text frames (one ``str``/NULL cell per value) -> columnar ``Tables``; shared by the CSV-export
    and the pg_dump ingest.

    Project ids follow ``ORDER BY project`` (the order of every per-project CSV row, and which project
    RQ3 treats as the last one, rq3:245-257).  Default: byte order, i.e. PostgreSQL under the C
    collation (and SQLite's BINARY).  A database with a locale collation (e.g. en_US.UTF-8 orders
    '-', '_' and case differently) is matched by passing ``project_order``: either the list of
    project names in the server's order (e.g. ``SELECT DISTINCT project ... ORDER BY project``) or
    a sort-key function over names (e.g. ``locale.strxfrm``)."""
    import pandas as pd
    names = set(b["project"].dropna()) | set(c["project"].dropna()) | set(i["project"].dropna())
    if pi is not None:
        names |= set(pi["project"].dropna())
    if project_order is None:
        projects = sorted(names, key=lambda s: s.encode())  # byte order == ORDER BY under C collation
    elif callable(project_order):
        projects = sorted(names, key=project_order)
    else:
        rank = {n: k for k, n in enumerate(project_order)}
        missing = names - set(rank)
        if missing:
            raise ValueError(f"project_order misses {len(missing)} project(s), e.g. {sorted(missing)[:3]}")
        projects = sorted(names, key=rank.__getitem__)
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


# ---------------------------------------------------------------------------------- pg_dump ingest
# The reference's data ships as a plain-format PostgreSQL dump (``data/database/backup_clean.sql``,
# README.md:14-15) that ``psql`` restores before any script runs.  Each table's rows sit in a
# ``COPY <table> (<columns>) FROM stdin;`` block of PostgreSQL's text COPY format: one row per line,
# tab-separated fields, ``\N`` = NULL, backslash escapes for \\ \b \f \n \r \t \v, octal \NNN and
# hex \xHH, terminated by a ``\.`` line.  ``from_pg_dump`` streams the dump once, keeps only the four
# tables the analyses read (other tables and all DDL are skipped) and feeds the same converter as
# the CSV-export ingest, so no database server is needed.
_DUMP_TABLES = ("buildlog_data", "total_coverage", "issues", "project_info")
_COPY_RE = re.compile(r'^COPY\s+(?:"?[\w$]+"?\.)?"?(\w+)"?\s*\(([^)]*)\)\s+FROM\s+stdin;\s*$')
_ESC_RE = re.compile(r"\\(x[0-9A-Fa-f]{1,2}|[0-7]{1,3}|.)")
_ESC_CHARS = {"b": "\b", "f": "\f", "n": "\n", "r": "\r", "t": "\t", "v": "\v"}


def _copy_unescape(field: str) -> str:
    def rep(m):
        e = m.group(1)
        if e[0] == "x":
            return chr(int(e[1:], 16))
        if e[0] in "01234567":
            return chr(int(e, 8) & 0xFF)
        return _ESC_CHARS.get(e, e)
    return _ESC_RE.sub(rep, field)


def _copy_escape(v) -> str:
    if v is None:
        return "\\N"
    s = str(v)
    return (s.replace("\\", "\\\\").replace("\t", "\\t").replace("\n", "\\n").replace("\r", "\\r")
            .replace("\b", "\\b").replace("\f", "\\f").replace("\v", "\\v"))


def _dump_corpus(path: str) -> str:
    base = os.path.dirname(os.path.abspath(path))
    for cp in (os.path.join(base, "project_corpus_analysis.csv"),
               os.path.join(base, "..", "processed_data", "csv", "project_corpus_analysis.csv")):
        if os.path.exists(cp):
            return open(cp).read()
    return ""


def from_pg_dump(path: str, corpus_csv: Optional[str] = None, project_order=None, native: Optional[bool] = None,
                 threads: Optional[int] = None) -> Tables:
    """Ingest a plain-format ``pg_dump`` file (see above) into columnar ``Tables``.

    ``corpus_csv``: text of ``project_corpus_analysis.csv`` (``rq4a_bug.py:34``); default: that
    file next to the dump or under ``../processed_data/csv/`` as in the reference's data layout.
    ``project_order``: see ``_from_frames`` (the database's collation).
    The native parser (csrc/fz_ingest.cpp, ``lib/libfzingest.so``: worker threads over the COPY
    blocks) is used when built (``native=None``; $FZ_INGEST=python forces this module's pandas
    path); a dump holding a cell it does not recognise (an unusual timestamp or number format) goes
    through the pandas path, which is the reference for every cell."""
    if corpus_csv is None:
        corpus_csv = _dump_corpus(path)
    if native is None:
        native = os.environ.get("FZ_INGEST", "native") != "python" and os.path.exists(_INGEST_LIB)
    if native:
        try:
            t = _from_pg_dump_native(path, corpus_csv, project_order, threads)
        except ValueError:  # a malformed dump: the pandas path reports it (same messages as ever)
            t = None
        if t is not None:
            return t
    return _from_pg_dump_pandas(path, corpus_csv, project_order)


_INGEST_LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libfzingest.so")
_ingest = None


def _ingest_lib():
    global _ingest
    if _ingest is None:
        import ctypes as C
        lib = C.CDLL(_INGEST_LIB)
        P, I64 = C.c_void_p, C.c_int64
        for name, res, args in (("fz_ingest_pg_dump", C.c_int, [C.c_char_p, C.c_int, C.POINTER(P)]),
                                ("fz_ingest_last_error", C.c_char_p, []), ("fz_ingest_free", None, [P]),
                                ("fz_ingest_rows", I64, [P, C.c_int]), ("fz_ingest_has", C.c_int, [P, C.c_int]),
                                ("fz_ingest_count", I64, [P, C.c_int]),
                                ("fz_ingest_strings", I64, [P, C.c_int, P, P]),
                                ("fz_ingest_column", C.c_int, [P, C.c_int, P])):
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
        _ingest = lib
    return _ingest


def _from_pg_dump_native(path, corpus_csv, project_order, threads):
    """libfzingest's columns as ``Tables`` (None when a cell needs the pandas parser)."""
    import ctypes as C
    lib = _ingest_lib()
    h = C.c_void_p()
    nthreads = threads or max(1, min(32, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity")
                                     else os.cpu_count() or 1))
    if lib.fz_ingest_pg_dump(path.encode(), nthreads, C.byref(h)) != 0:
        raise ValueError(f"{path}: {lib.fz_ingest_last_error().decode(errors='replace')}")
    try:
        if lib.fz_ingest_count(h, -3) > 0:
            return None

        def strings(which, n=None):
            n = lib.fz_ingest_count(h, which) if n is None else n
            total = lib.fz_ingest_strings(h, which, None, None)
            blob = np.empty(max(total, 1), np.uint8)
            offs = np.empty(n + 1, np.int64)
            lib.fz_ingest_strings(h, which, blob.ctypes.data_as(C.c_void_p), offs.ctypes.data_as(C.c_void_p))
            raw = blob[:total].tobytes()
            return raw, offs

        def str_list(which):
            raw, offs = strings(which)
            o = offs.tolist()
            return [raw[o[k]:o[k + 1]].decode("utf-8") for k in range(len(o) - 1)]

        def col(code, n, dtype):
            a = np.empty(n, dtype)
            if n:
                lib.fz_ingest_column(h, code, a.ctypes.data_as(C.c_void_p))
            return a

        nb, nc, ni, npi = (lib.fz_ingest_rows(h, k) for k in range(4))
        projects = str_list(-1)
        vocab = [str_list(k) for k in range(5)]
        raw, offs = strings(-2, nb)
        nnull = col(6, nb, np.uint8).astype(bool)
        names = np.empty(nb, dtype=object)
        if raw.isascii():
            text, o = raw.decode("ascii"), offs.tolist()
            names[:] = [None if nnull[k] else text[o[k]:o[k + 1]] for k in range(nb)]
        else:
            o = offs.tolist()
            names[:] = [None if nnull[k] else raw[o[k]:o[k + 1]].decode("utf-8") for k in range(nb)]
        t = Tables(
            projects=projects,
            b_project=col(0, nb, np.uint32), b_type=col(1, nb, np.uint8), b_result=col(2, nb, np.uint8),
            b_time=col(3, nb, np.int64), b_modules=col(4, nb, np.int32), b_revisions=col(5, nb, np.int32),
            b_name=names, modules_pool=vocab[2], revisions_pool=vocab[3],
            c_project=col(7, nc, np.uint32), c_date=col(8, nc, np.int64), c_coverage=col(9, nc, np.float64),
            c_coverage_valid=col(10, nc, np.uint8).astype(bool), c_covered=col(11, nc, np.int64),
            c_covered_valid=col(12, nc, np.uint8).astype(bool), c_total=col(13, nc, np.int64),
            c_total_valid=col(14, nc, np.uint8).astype(bool),
            i_number=col(15, ni, np.int64), i_project=col(16, ni, np.uint32), i_rts=col(17, ni, np.int64),
            i_status=col(18, ni, np.uint8), i_new_id=col(19, ni, np.int64),
            pi_project=col(20, npi, np.uint32), pi_first_commit=col(21, npi, np.int64),
            build_types=vocab[0], results=vocab[1], statuses=vocab[4], corpus_csv=corpus_csv)
    finally:
        lib.fz_ingest_free(h)
    if project_order is not None:  # the database's collation: re-number the byte-ordered ids
        if callable(project_order):
            order = sorted(projects, key=project_order)
        else:
            rank = {n: k for k, n in enumerate(project_order)}
            missing = set(projects) - set(rank)
            if missing:
                raise ValueError(f"project_order misses {len(missing)} project(s), e.g. {sorted(missing)[:3]}")
            order = sorted(projects, key=rank.__getitem__)
        pid = {n: k for k, n in enumerate(order)}
        remap = np.array([pid[n] for n in projects], dtype=np.uint32)
        import dataclasses
        t = dataclasses.replace(t, projects=order, b_project=remap[t.b_project], c_project=remap[t.c_project],
                                i_project=remap[t.i_project], pi_project=remap[t.pi_project])
    return t


def _from_pg_dump_pandas(path: str, corpus_csv: str, project_order=None) -> Tables:
    """The dump through pandas' C tokenizer and this module's text converters (the reference
    parser of every cell; see from_pg_dump)."""
    import pandas as pd
    blocks: Dict[str, List[str]] = {}
    cols: Dict[str, List[str]] = {}
    with open(path, encoding="utf-8", newline="\n") as f:
        it = iter(f)
        for line in it:
            if not line.startswith("COPY "):
                continue
            m = _COPY_RE.match(line.rstrip("\n"))
            if m is None:
                continue
            name = m.group(1)
            keep = name in _DUMP_TABLES
            if keep:
                cols[name] = [c.strip().strip('"') for c in m.group(2).split(",")]
                out = blocks.setdefault(name, [])
                tabs = len(cols[name]) - 1
            for row in it:
                if row == "\\.\n" or row == "\\.":
                    break
                if keep:
                    if row.count("\t") != tabs:
                        raise ValueError(f"{path}: COPY {name}: {row.count(chr(9)) + 1} fields, expected {tabs + 1}")
                    out.append(row if row.endswith("\n") else row + "\n")
            else:
                raise ValueError(f"{path}: COPY {name} block not terminated by \\.")
    for need in _DUMP_TABLES[:3]:
        if need not in blocks:
            raise ValueError(f"{path}: no COPY block for table {need!r}")

    def frame(name):
        # the C tokenizer splits the block (tabs are always escaped inside fields, so no quoting);
        # only cells holding a backslash go through the escape decoder
        if not blocks[name]:
            return pd.DataFrame({c: pd.Series([], dtype=object) for c in cols[name]})
        text = "".join(blocks[name])
        df = pd.read_csv(io.StringIO(text), sep="\t", header=None, names=cols[name], dtype=str,
                         quoting=csv.QUOTE_NONE, keep_default_na=False, na_values=["\\N"],
                         skip_blank_lines=False, engine="c")
        if "\\" not in text.replace("\\N", ""):
            return df
        for c in df.columns:
            col = df[c]
            esc = col.str.contains("\\", regex=False, na=False)
            if esc.any():
                df.loc[esc, c] = col[esc].map(_copy_unescape)
        return df

    pi = frame("project_info") if "project_info" in blocks else None
    return _from_frames(frame("buildlog_data"), frame("total_coverage"), frame("issues"), pi, corpus_csv,
                        project_order)


def to_pg_dump(t: Tables, path: str) -> None:
    """Write ``Tables`` as a plain-format dump (DDL + one COPY block per table) that ``psql`` can
    restore and ``from_pg_dump`` reads back; used by tests and to seed a database."""
    from .schema import us_to_dt

    def ts(v):
        return None if v == TS_NULL else str(us_to_dt(v))

    def code(vocab, v):
        return None if v == CODE_NULL else vocab[v]

    def pool(p, k):
        return None if k < 0 else p[k]

    def block(f, name, ddl, header, it):
        f.write(f"CREATE TABLE public.{name} (\n    " + ",\n    ".join(ddl) + "\n);\n\n")
        f.write(f"COPY public.{name} ({', '.join(header)}) FROM stdin;\n")
        for r in it:
            f.write("\t".join(_copy_escape(v) for v in r) + "\n")
        f.write("\\.\n\n")

    P = t.projects
    with open(path, "w", encoding="utf-8", newline="\n") as f:
        f.write("--\n-- PostgreSQL database dump\n--\n\nSET client_encoding = 'UTF8';\n"
                "SET standard_conforming_strings = on;\n\n")
        block(f, "buildlog_data",
              ["name text", "project text", "build_type text", "result text",
               "timecreated timestamp without time zone", "modules text", "revisions text"],
              ["name", "project", "build_type", "result", "timecreated", "modules", "revisions"],
              ((t.b_name[k], P[t.b_project[k]], code(t.build_types, t.b_type[k]),
                code(t.results, t.b_result[k]), ts(t.b_time[k]), pool(t.modules_pool, t.b_modules[k]),
                pool(t.revisions_pool, t.b_revisions[k])) for k in range(len(t.b_project))))
        block(f, "total_coverage",
              ["project text", "date timestamp without time zone", "coverage double precision",
               "covered_line integer", "total_line integer"],
              ["project", "date", "coverage", "covered_line", "total_line"],
              ((P[t.c_project[k]], ts(t.c_date[k]),
                repr(float(t.c_coverage[k])) if t.c_coverage_valid[k] else None,
                int(t.c_covered[k]) if t.c_covered_valid[k] else None,
                int(t.c_total[k]) if t.c_total_valid[k] else None) for k in range(len(t.c_project))))
        block(f, "issues",
              ["number bigint", "project text", "rts timestamp without time zone", "status text",
               "new_id bigint"],
              ["number", "project", "rts", "status", "new_id"],
              ((int(t.i_number[k]), P[t.i_project[k]], ts(t.i_rts[k]), code(t.statuses, t.i_status[k]),
                int(t.i_new_id[k])) for k in range(len(t.i_project))))
        block(f, "project_info", ["project text", "first_commit_datetime timestamp without time zone"],
              ["project", "first_commit_datetime"],
              ((P[t.pi_project[k]], ts(t.pi_first_commit[k])) for k in range(len(t.pi_project))))
        f.write("--\n-- PostgreSQL database dump complete\n--\n")
