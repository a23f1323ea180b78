"""CPU tests of the columnar loader (store.py): the native columnar directory and the PostgreSQL
CSV-export ingest both reproduce the tables - checked through the oracle's RQ outputs, which must
not change (a loader bug would move counts or orders)."""
import numpy as np
import pytest

import goldens
from gpu_common import assert_same
from oracle import rq_oracle as orc
from tse_amd import store, synth


def test_columnar_roundtrip(tmp_path):
    t = goldens.tables("tiny")
    store.save_columnar(t, str(tmp_path / "col"))
    t2 = store.load_columnar(str(tmp_path / "col"))
    assert synth.table_fingerprint(t2) == synth.table_fingerprint(t)


@pytest.mark.parametrize("fn", [orc.rq1, orc.rq2_count, orc.rq2_add, orc.rq3, orc.rq4a, orc.rq4b])
def test_csv_export_ingest_preserves_results(tmp_path_factory, fn):
    t = goldens.tables("tiny")
    d = tmp_path_factory.getbasetemp() / "csvdir"
    if not (d / "issues.csv").exists():
        store.to_csv_dir(t, str(d))
    t2 = store.from_csv_dir(str(d))
    assert t2.projects == t.projects
    assert np.array_equal(t2.b_time, t.b_time) and np.array_equal(t2.c_date, t.c_date)
    assert np.array_equal(t2.c_coverage, t.c_coverage)
    assert np.array_equal(t2.group_key() == t2.group_key()[0], t.group_key() == t.group_key()[0])
    assert_same(fn(t2), fn(t))


def test_copy_text_escapes_roundtrip():
    s = "a\\b\tc\nd\re\x08f\x0cg\x0bh"
    enc = store._copy_escape(s)
    assert "\t" not in enc and "\n" not in enc
    assert store._copy_unescape(enc) == s
    assert store._copy_escape(None) == "\\N"
    assert store._copy_unescape("\\101\\x42\\q") == "ABq"      # octal, hex, any other escaped char


@pytest.mark.parametrize("fn", [orc.rq1, orc.rq2_count, orc.rq2_add, orc.rq3, orc.rq4a, orc.rq4b])
def test_pg_dump_ingest_preserves_results(tmp_path_factory, fn):
    """A plain-format dump (COPY text blocks, \\N NULLs, escapes in build names, unrelated tables
    in between) reproduces the tables and every oracle result."""
    t = goldens.tables("tiny")
    d = tmp_path_factory.getbasetemp() / "dump"
    sql = d / "backup_clean.sql"
    if not sql.exists():
        d.mkdir(exist_ok=True)
        t.b_name = t.b_name.copy()
        t.b_name[0] = "odd\tname\\with\nescapes"
        store.to_pg_dump(t, str(sql))
        txt = sql.read_text()
        # an unrelated table (skipped) and a quoted COPY header, as pg_dump writes for some names
        txt = txt.replace("CREATE TABLE public.issues",
                          'COPY public."crash_log" (id, body) FROM stdin;\n1\tx\\ty\n2\t\\N\n\\.\n\n'
                          "CREATE TABLE public.issues")
        sql.write_text(txt)
        (d / "project_corpus_analysis.csv").write_text(t.corpus_csv)
    t2 = store.from_pg_dump(str(sql))
    assert t2.projects == t.projects
    assert t2.b_name[0] == "odd\tname\\with\nescapes"
    assert np.array_equal(t2.b_time, t.b_time) and np.array_equal(t2.c_date, t.c_date)
    assert np.array_equal(t2.c_coverage, t.c_coverage)
    assert np.array_equal(t2.c_covered_valid, t.c_covered_valid) and np.array_equal(t2.i_rts, t.i_rts)
    assert t2.corpus_csv == t.corpus_csv
    assert_same(fn(t2), fn(t))


def test_pg_dump_errors(tmp_path):
    p = tmp_path / "bad.sql"
    p.write_text("COPY public.issues (number, project) FROM stdin;\n1\tx\n")
    with pytest.raises(ValueError, match="not terminated"):
        store.from_pg_dump(str(p))
    p.write_text("COPY public.issues (number, project) FROM stdin;\n1\tx\textra\n\\.\n")
    with pytest.raises(ValueError, match="fields"):
        store.from_pg_dump(str(p))
    p.write_text("SELECT 1;\n")
    with pytest.raises(ValueError, match="no COPY block"):
        store.from_pg_dump(str(p))


def test_pg_dump_empty_block_and_utc_offsets(tmp_path):
    """An empty COPY block (no rows) and timestamptz text ('+00' suffix, as a UTC server dumps it)
    load as an empty table and as naive wall-clock microseconds."""
    p = tmp_path / "d.sql"
    p.write_text(
        "COPY public.buildlog_data (name, project, build_type, result, timecreated, modules, revisions) FROM stdin;\n"
        "b1\tp\tFuzzing\tFinish\t2020-01-02 03:04:05.000006+00\t{m}\t{r}\n\\.\n"
        "COPY public.total_coverage (project, date, coverage, covered_line, total_line) FROM stdin;\n"
        "p\t2020-01-02 00:00:00+00\t12.5\t10\t80\np\t2020-01-03 00:00:00+00\t\\N\t\\N\t\\N\n\\.\n"
        "COPY public.issues (number, project, rts, status, new_id) FROM stdin;\n\\.\n"
        "COPY public.project_info (project, first_commit_datetime) FROM stdin;\n\\.\n")
    t = store.from_pg_dump(str(p), corpus_csv="")
    assert t.projects == ["p"] and len(t.i_number) == 0 and len(t.pi_project) == 0
    assert int(t.b_time[0]) == int(np.datetime64("2020-01-02T03:04:05.000006", "us").astype(np.int64))
    assert t.c_coverage_valid.tolist() == [True, False] and t.c_covered_valid.tolist() == [True, False]
    assert t.c_coverage[0] == 12.5 and t.modules_pool == ["{m}"]


def test_pg_dump_mixed_utc_offsets(tmp_path):
    """timestamptz text dumped under a daylight-saving server TimeZone carries different offsets in
    one column ('+01' in winter, '+02' in summer, also '+05:30'): every value keeps its printed
    wall-clock time (the analyses compare naive values)."""
    p = tmp_path / "d.sql"
    p.write_text(
        "COPY public.buildlog_data (name, project, build_type, result, timecreated, modules, revisions) FROM stdin;\n"
        "b1\tp\tFuzzing\tFinish\t2020-01-02 03:04:05.25+01\t{m}\t{r}\n"
        "b2\tp\tFuzzing\tFinish\t2020-07-02 03:04:05+02\t{m}\t{r}\n"
        "b3\tp\tCoverage\tFinish\t2020-07-03 10:00:00+05:30\t{m}\t{r}\n\\.\n"
        "COPY public.total_coverage (project, date, coverage, covered_line, total_line) FROM stdin;\n"
        "p\t2020-01-02 00:00:00+01\t12.5\t10\t80\np\t2020-07-03 00:00:00+02\t\\N\t\\N\t\\N\n\\.\n"
        "COPY public.issues (number, project, rts, status, new_id) FROM stdin;\n"
        "7\tp\t2020-03-29 02:30:00-07\tFixed\t1\n\\.\n")
    t = store.from_pg_dump(str(p), corpus_csv="")
    us = lambda s: int(np.datetime64(s, "us").astype(np.int64))  # noqa: E731
    assert t.b_time.tolist() == [us("2020-01-02T03:04:05.25"), us("2020-07-02T03:04:05"), us("2020-07-03T10:00:00")]
    assert t.c_date.tolist() == [us("2020-01-02T00:00:00"), us("2020-07-03T00:00:00")]
    assert t.i_rts.tolist() == [us("2020-03-29T02:30:00")]


def test_project_order_override(tmp_path):
    """ORDER BY project under a locale collation: the caller's order (a name list or a sort key)
    replaces byte order for the project ids."""
    p = tmp_path / "d.sql"
    p.write_text(
        "COPY public.buildlog_data (name, project, build_type, result, timecreated, modules, revisions) FROM stdin;\n"
        "b1\tlib-b\tFuzzing\tFinish\t2020-01-02 03:04:05\t{m}\t{r}\n"
        "b2\tlib_a\tFuzzing\tFinish\t2020-01-02 03:04:05\t{m}\t{r}\n"
        "b3\tLibC\tFuzzing\tFinish\t2020-01-02 03:04:05\t{m}\t{r}\n\\.\n"
        "COPY public.total_coverage (project, date, coverage, covered_line, total_line) FROM stdin;\n\\.\n"
        "COPY public.issues (number, project, rts, status, new_id) FROM stdin;\n\\.\n")
    assert store.from_pg_dump(str(p), corpus_csv="").projects == ["LibC", "lib-b", "lib_a"]   # bytes
    t = store.from_pg_dump(str(p), corpus_csv="", project_order=["lib_a", "lib-b", "LibC"])
    assert t.projects == ["lib_a", "lib-b", "LibC"] and t.b_project.tolist() == [1, 0, 2]
    t = store.from_pg_dump(str(p), corpus_csv="", project_order=lambda s: s.lower().replace("-", "").replace("_", ""))
    assert t.projects == ["lib_a", "lib-b", "LibC"]
    with pytest.raises(ValueError, match="misses"):
        store.from_pg_dump(str(p), corpus_csv="", project_order=["lib_a"])
