"""GPU: NULL line counts reaching the reference's arithmetic (tests/null_edges.py).  The HIP path
counts the pairs / rows the reference would have crashed on (counts[FZ_RQ3_NULL_TOTAL],
counts[FZ_RQ2C_NULL_LINES]) and the host raises the same TypeError; where the reference ran, the
outputs equal its goldens and the oracle.  The sharded RQ3 drops the NULL pairs of the globally last
project's flush with its rows (parallel.rq3_sharded)."""
import ctypes as C

import pytest

import goldens
from gpu_common import assert_same
from oracle import rq_oracle as orc
from test_null_edges import CASES, run_expecting_reference
from tse_amd import engine as E
from tse_amd.rq import compute

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case,script", CASES)
def test_gpu_matches_reference_on_null_edges(engine_for, case, script):
    eng = engine_for(case)
    t = goldens.tables(case)
    fn = (lambda: compute.rq2_count(eng)) if script == "rq2_coverage_count" else (lambda: compute.rq3(eng))
    run_expecting_reference(case, script, fn, t)
    if goldens.returncode(case, script) == 0:
        assert_same(fn(), orc.rq2_count(t) if script == "rq2_coverage_count" else orc.rq3(t))


@pytest.mark.parametrize("case", ["tiny+null_total_last", "tiny+null_total_mid"])
def test_gpu_rq3_flush_last_counts(engine_for, case):
    """fz_rq3_ex(FZ_RQ3_FLUSH_LAST): NULL pairs counted, those of the last project's flush apart;
    the one-rank sharded driver then raises exactly when the reference does."""
    eng = engine_for(case)
    t = goldens.tables(case)
    ref = orc.rq3(t, flush_last=True, on_null="count")
    b = compute.rq3_buffers(eng)
    E._check(eng.lib, eng.lib.fz_rq3_ex(eng.ctx, E.FZ_RQ3_FLUSH_LAST | E.FZ_RQ3_SKIP_STATS, C.byref(b.out)))
    cnt = b.host("counts")
    assert int(cnt[E.RQ3_NULL_TOTAL]) == ref.n_null_total and int(cnt[E.RQ3_NULL_LAST]) == ref.n_null_last
    total = cnt.copy()
    total[E.RQ3_NULL_TOTAL] -= total[E.RQ3_NULL_LAST]
    assert (total[E.RQ3_NULL_TOTAL] > 0) == (goldens.returncode(case, "rq3_diff_coverage_at_detection") != 0)
