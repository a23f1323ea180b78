"""The native CSV writers (csrc/fz_write.cpp via tse_amd/rq/writer.py) against Python's own
formatting: repr(float) on random bit patterns and the layout boundaries of CPython's
format_float_short, coverage_by_session_index.csv rows (rq2_coverage_count.py:347-352) and the
change-point tables (rq2_coverage_and_added.py:221-238) against csv.writer byte for byte.  The
golden and shipped-output tests render through the same writer (test_oracle_golden.py,
test_shipped_kat.py)."""
import io
import csv
import math
import struct

import numpy as np
import pytest

from tse_amd.rq import render, writer

pytestmark = pytest.mark.skipif(writer.lib() is None, reason="libfzwrite.so not built")


def _csv(rows):
    b = io.StringIO(newline="")
    csv.writer(b).writerows(rows)
    return b.getvalue().encode()


EDGE = [0.0, -0.0, 1.0, -1.0, 0.1, 0.2, 0.30000000000000004, 1e16, 1e15, 9999999999999998.0, 1e17, 1.5e16,
        1e-4, 1e-5, 0.0001, 0.00012345, 1.2345e-5, 123456789.0, 2.0 ** 53, 2.0 ** 53 + 2, 1e22, 1e23, 5e-324,
        2.2250738585072014e-308, 1.7976931348623157e308, math.inf, -math.inf, math.nan, 100.0, 99.99999999999999,
        33.333333333333336, 66.66666666666667, 1e100, 1.0000000000000002, 4.35, 0.5, 12.0, 1234.5678]


def test_repr_edges():
    for v in EDGE:
        assert writer.repr_float(v) == repr(v), v


def test_repr_random_bits():
    rng = np.random.default_rng(1)
    bits = rng.integers(0, 2 ** 63, 200_000, dtype=np.int64).astype(np.uint64)
    bits |= (rng.integers(0, 2, len(bits)).astype(np.uint64) << np.uint64(63))
    vals = bits.view(np.float64)
    for v in vals.tolist():
        assert writer.repr_float(v) == repr(v), struct.pack("<d", v).hex()


def test_repr_percentages_and_integers():
    rng = np.random.default_rng(2)
    cov = rng.integers(0, 200_000, 100_000)
    tot = rng.integers(1, 200_000, 100_000)
    for v in (cov / tot * 100.0).tolist() + [float(x) for x in rng.integers(-2 ** 53, 2 ** 53, 20_000).tolist()]:
        assert writer.repr_float(v) == repr(v)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_float_rows_match_csv_writer(seed):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, 40, 3000)
    lens[:5] = 0
    vals = np.concatenate([rng.uniform(0, 100, int(lens.sum())) * rng.choice([1.0, 1e-7, 1e18], int(lens.sum()))])
    vals[rng.random(len(vals)) < 0.01] = np.nan
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    got = writer.float_rows(vals, offs)
    v = vals.tolist()
    assert got == _csv([v[offs[i]:offs[i + 1]] for i in range(len(lens))])


def test_float_rows_empty():
    assert writer.float_rows(np.zeros(0), np.zeros(1, np.int64)) == b""
    assert writer.float_rows(np.zeros(0), np.zeros(3, np.int64)) == b"\r\n\r\n"


def test_change_rows_match_python_render(monkeypatch):
    """render.rq2_add through the native writer == through csv.writer, on a table with NULL cells,
    float-upcast projects, missing coverage rows and None modules / revisions."""
    from oracle import rq_oracle as orc
    from tse_amd import synth
    t = synth.generate(synth.config("tiny"))
    r = orc.rq2_add(t)
    assert len(r.row_project) > 0
    rng = np.random.default_rng(5)
    k = len(r.row_project)
    r.row_cov_i = np.where(rng.random(k) < 0.1, -1, r.row_cov_i)
    r.diff_total = np.where(rng.random(k) < 0.1, np.nan, r.diff_total)
    r.covered_is_float = rng.random(len(r.covered_is_float)) < 0.5
    t.b_modules = np.where(rng.random(len(t.b_modules)) < 0.05, -1, t.b_modules).astype(t.b_modules.dtype)
    t.derived.clear()
    native = render.rq2_add(r, t)
    monkeypatch.setenv("FZ_WRITER", "python")
    py = render.rq2_add(r, t)
    assert native.stdout == py.stdout
    assert native.files.keys() == py.files.keys()
    for p in py.files:
        assert native.files[p] == py.files[p], p
