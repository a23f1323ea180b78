"""GPU parity for RQ4 (rq4a_bug.py, rq4b_coverage.py): corpus groups, G1/G2 iteration tables, G4
windows, per-session quartiles + Brunner-Munzel, coverage deltas, initial-coverage tests."""
import pytest

import goldens
from gpu_common import assert_same
from oracle import rq_oracle as orc
from tse_amd.rq import compute, render

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", goldens.CASES)
def test_rq4a(engine_for, case):
    eng = engine_for(case)
    t = goldens.tables(case)
    ours = compute.rq4a(eng)
    ref = orc.rq4a(t)
    assert_same(ours, ref)
    r = render.rq4a(ours, t)
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq4a_bug"), rtol=1e-9)
    assert not errs, "\n".join(errs)
    rel = "rq4/bug/rq4_g1_g2_detection_trend.csv"
    assert r.files["data/result_data/" + rel] == goldens.file_bytes(case, rel)


@pytest.mark.parametrize("case", goldens.CASES)
def test_rq4b(engine_for, case):
    eng = engine_for(case)
    t = goldens.tables(case)
    ours = compute.rq4b(eng)
    ref = orc.rq4b(t)
    assert_same(ours, ref)
    r = render.rq4b(ours, t, n_eligible=len(orc.eligible_projects(t)))
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq4b_coverage"), rtol=1e-9)
    assert not errs, "\n".join(errs)
