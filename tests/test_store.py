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
