"""NULL line counts reaching the reference's arithmetic (tests/null_edges.py): the CPU oracle, rendered,
matches what the UNMODIFIED reference did on each edge table (tests/golden/tiny+<edge>/, written
by tests/golden/make_goldens.py edges) - the same TypeError where the reference crashed
(rq3_diff_coverage_at_detection.py:253,297 `None > 0`; rq2_coverage_count.py:301 `float(None)`),
the same stdout and CSV bytes where it ran.  test_gpu_null_edges.py holds the HIP path to the same."""
import pytest

import goldens
import null_edges
from oracle import rq_oracle as orc
from tse_amd.rq import render

CASES = [(f"tiny+{e}", s) for e in null_edges.EDGES for s in null_edges.SCRIPTS]


def reference_error(case, script):
    """The exception line the reference printed last on stderr, e.g. 'TypeError: ...'."""
    lines = [ln for ln in goldens.text(case, script, "stderr").splitlines() if ln.strip()]
    return lines[-1]


def check_rendered(case, script, result, t):
    if script == "rq2_coverage_count":
        r = render.rq2_count(result, t)
        files = ["rq2/coverage_by_session_index.csv"]
    else:
        r = render.rq3(result, t)
        files = ["rq3/detected_coverage_changes.csv", "rq3/non_detected_coverage_changes.csv"]
    errs = goldens.compare_lines(r.text(), goldens.text(case, script), rtol=1e-9)
    assert not errs, "\n".join(errs)
    for rel in files:
        assert r.files["data/result_data/" + rel] == goldens.file_bytes(case, rel), rel


def run_expecting_reference(case, script, fn, t):
    """fn() -> result; raises exactly where the reference raised, else renders its outputs."""
    if goldens.returncode(case, script) != 0:
        kind, _, msg = reference_error(case, script).partition(": ")
        assert kind == "TypeError"
        with pytest.raises(TypeError) as ei:
            fn()
        assert str(ei.value) == msg
        return
    check_rendered(case, script, fn(), t)


@pytest.mark.parametrize("case,script", CASES)
def test_oracle_matches_reference_on_null_edges(case, script):
    t = goldens.tables(case)
    fn = (lambda: orc.rq2_count(t)) if script == "rq2_coverage_count" else (lambda: orc.rq3(t))
    run_expecting_reference(case, script, fn, t)


def test_edges_exercise_both_outcomes():
    rc = {(c, s): goldens.returncode(c, s) for c, s in CASES}
    assert rc[("tiny+null_total_mid", "rq3_diff_coverage_at_detection")] != 0
    assert rc[("tiny+null_total_last", "rq3_diff_coverage_at_detection")] == 0   # never flushed (rq3:245-257)
    assert rc[("tiny+covered_null_zero", "rq2_coverage_count")] == 0             # x[1] != 0 skips it
    assert rc[("tiny+covered_null", "rq2_coverage_count")] != 0


def test_oracle_shard_counts_null_pairs():
    """on_null='count' (shards): the last project's flush reports its NULL pairs separately, so the
    sharded driver can drop them with that project's rows (parallel.rq3_sharded)."""
    t = goldens.tables("tiny+null_total_last")
    r = orc.rq3(t, flush_last=True, on_null="count")
    assert r.n_null_total > 0 and r.n_null_total == r.n_null_last
    t = goldens.tables("tiny+null_total_mid")
    r = orc.rq3(t, flush_last=True, on_null="count")
    assert r.n_null_total > r.n_null_last
