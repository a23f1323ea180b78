"""GPU parity for RQ3 (rq3_diff_coverage_at_detection.py:202-360): detections, non-detected changes,
summary tables, Anderson-Darling, Levene and Brunner-Munzel vs the CPU oracle and the golden output."""
import pytest

import goldens
from gpu_common import assert_same
from oracle import rq_oracle as orc
from tse_amd.rq import compute, render

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", goldens.CASES)
def test_rq3(engine_for, case):
    eng = engine_for(case)
    t = goldens.tables(case)
    ours = compute.rq3(eng)
    assert_same(ours, orc.rq3(t))
    r = render.rq3(ours, t)
    errs = goldens.compare_lines(r.text(), goldens.text(case, "rq3_diff_coverage_at_detection"), rtol=1e-9)
    assert not errs, "\n".join(errs)
    for rel in ("rq3/detected_coverage_changes.csv", "rq3/non_detected_coverage_changes.csv"):
        assert r.files["data/result_data/" + rel] == goldens.file_bytes(case, rel), rel
