"""GPU parity for RQ1 (rq1_detection_rate.py:101-269): HIP path through libfz vs the CPU oracle
(field by field) and, rendered, vs the reference's own outputs (golden fixtures)."""
import pytest

import goldens
from gpu_common import assert_same
from oracle import rq_oracle as orc
from tse_amd.rq import compute, render

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", goldens.CASES)
def test_rq1_matches_oracle_and_golden(engine_for, case):
    eng = engine_for(case)
    t = goldens.tables(case)
    ours = compute.rq1(eng)
    ref = orc.rq1(t)
    assert_same(ours, ref)
    r = render.rq1(ours, t)
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq1_detection_rate"))
    assert not errs, "\n".join(errs)
    for rel in ("rq1/rq1_detection_rate_stats.csv", "rq1/rq1_raw_issues_for_analysis.csv"):
        assert r.files["data/result_data/" + rel] == goldens.file_bytes(case, rel), rel


def test_rq1_threshold_edge(engine_for):
    """TEST_MODE-style threshold 1 (rq1_detection_rate.py:233): every iteration kept."""
    eng = engine_for("tiny")
    t = goldens.tables("tiny")
    assert_same(compute.rq1(eng, threshold=1), orc.rq1(t, threshold=1))
    # a threshold no iteration reaches: no late-stage block
    ours = compute.rq1(eng, threshold=10**9)
    assert ours.late is None
    assert_same(ours, orc.rq1(t, threshold=10**9))
