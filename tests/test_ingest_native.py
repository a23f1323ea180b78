"""The native dump ingest (csrc/fz_ingest.cpp, libfzingest.so) against the
pandas path of store.from_pg_dump, which is the reference parser of every cell: identical Tables
(every column, dictionary order, vocabularies, names) on dumps with NULLs, COPY escapes, non-ASCII
text, UTC offsets, date-only and fractional timestamps, empty strings and a project order of the
database's collation; a cell the native parser does not recognise sends the whole dump through the
pandas path."""
import dataclasses
import os
import re

import numpy as np
import pytest

from tse_amd import store
import tse_amd.synth as synth

pytestmark = pytest.mark.skipif(not os.path.exists(store._INGEST_LIB), reason="libfzingest.so not built")


def _same(a, b):
    for f in dataclasses.fields(a):
        if f.name == "derived":
            continue
        x, y = getattr(a, f.name), getattr(b, f.name)
        if isinstance(x, np.ndarray):
            assert x.dtype == y.dtype, f.name
            if x.dtype == object:
                assert list(x) == list(y), f.name
            else:
                assert np.array_equal(x, y), f.name
        else:
            assert x == y, f.name


def _awkward(t):
    """A medium table with the text the dump format has to carry."""
    t = dataclasses.replace(t, projects=list(t.projects))
    t.projects[1] = "with\ttab\\and\\nnewline"
    t.projects[2] = "ünïcödé-☃"
    t.projects[3] = ""
    mods = list(t.modules_pool)
    mods[0] = "{mod\\ule,\"two\"}"
    names = t.b_name.copy()
    names[::7] = None
    names[1] = "tab\there"
    names[2] = ""
    return dataclasses.replace(t, modules_pool=mods, b_name=names)


@pytest.mark.parametrize("case", ["tiny", "medium"])
def test_native_matches_pandas(case, tmp_path):
    t = _awkward(synth.generate(synth.config(case)))
    path = str(tmp_path / "dump.sql")
    store.to_pg_dump(t, path)
    # timestamp spellings a server prints: '+00' offsets (timestamptz), 'T' separators, dates only
    text = open(path, encoding="utf-8").read()
    text = re.sub(r"(\d{4}-\d\d-\d\d \d\d:\d\d:\d\d(?:\.\d+)?)\t", lambda m: m.group(1) + "+00\t", text, count=50)
    text = re.sub(r"\t(\d{4}-\d\d-\d\d) 00:00:00\t", r"\t\1\t", text)
    text = re.sub(r"\t(\d{4}-\d\d-\d\d) (\d\d:\d\d:\d\d\.\d+)\t", r"\t\1T\2\t", text, count=30)
    open(path, "w", encoding="utf-8").write(text)
    a = store.from_pg_dump(path, native=True, threads=3)
    b = store.from_pg_dump(path, native=False)
    _same(a, b)
    assert store._from_pg_dump_native(path, "", None, 2) is not None  # no fallback happened


def test_project_order(tmp_path):
    t = synth.generate(synth.config("tiny"))
    path = str(tmp_path / "dump.sql")
    store.to_pg_dump(t, path)
    order = sorted(t.projects, key=lambda s: s[::-1])
    _same(store.from_pg_dump(path, project_order=order, native=True),
          store.from_pg_dump(path, project_order=order, native=False))
    key = lambda s: s.lower().replace("-", "")  # noqa: E731
    _same(store.from_pg_dump(path, project_order=key, native=True),
          store.from_pg_dump(path, project_order=key, native=False))


def test_unrecognised_cell_falls_back(tmp_path):
    t = synth.generate(synth.config("tiny"))
    path = str(tmp_path / "dump.sql")
    store.to_pg_dump(t, path)
    text = open(path, encoding="utf-8").read()
    text = re.sub(r"\t(\d{4})-(\d\d)-(\d\d) ", r"\t\2/\3/\1 ", text, count=1)  # an MDY timestamp
    open(path, "w", encoding="utf-8").write(text)
    assert store._from_pg_dump_native(path, "", None, 2) is None
    _same(store.from_pg_dump(path), store.from_pg_dump(path, native=False))


def test_errors(tmp_path):
    p = tmp_path / "bad.sql"
    p.write_text("COPY public.buildlog_data (name, project) FROM stdin;\nx\ty\n")
    with pytest.raises(ValueError, match="not terminated"):
        store._from_pg_dump_native(str(p), "", None, 2)
    with pytest.raises(ValueError, match="not terminated"):  # reported by the pandas path
        store.from_pg_dump(str(p), native=True)
