"""GPU path on the reference's SHIPPED real-data vectors (tests/golden/shipped/): the finishing
entry points and the full store + rq2_add pipeline through libfz reproduce what the reference
printed or wrote for the real dataset.  Same vectors as tests/test_shipped_kat.py (CPU oracle)."""
import numpy as np
import pytest
from scipy import stats

import shipped
from gpu_common import assert_same
from oracle import rq_oracle as orc
from tse_amd import engine as E
from tse_amd.rq import common, compute, render

pytestmark = pytest.mark.gpu


def test_rq1_finish_shipped(engine):
    """fz_rq1_finish on the 2,341 shipped iterations prints rq1_detection_rate.py:401-407."""
    it, idt = shipped.rq1_tables()
    counts, late = engine.rq1_finish(it, idt, 100)
    assert counts[E.RQ1_KEPT_ITERS] == 2341 and counts[E.RQ1_FIRST_DOWN] == 27 and counts[E.RQ1_LATE] == 2314
    d = compute._describe(E.describe_from_doubles(late), with_min_nonzero=True)
    assert render.rq1_late_lines(d) == ["\n" + shipped.RQ1_LATE_BLOCK[0]] + shipped.RQ1_LATE_BLOCK[1:]
    ref = orc.rq1_finish(it, idt, 100)
    for f in ("count", "n_zero", "min", "max", "q1", "q3", "median", "mean", "min_nonzero"):
        assert_same(getattr(d, f), getattr(ref, f), f"late.{f}")


def test_rq4a_finish_shipped(engine):
    """fz_rq4a_finish on the shipped G1/G2 trend table (1,600 iterations) and the 86 shipped
    introduction iterations prints rq4a_bug.py:698-747 and :281-285 as the reference did."""
    g1t, g1d, g2t, g2d = shipped.rq4a_tables()
    intro = np.array([k for _, k in shipped.intro_rows()], np.int64)
    counts, sc = engine.rq4a_finish(g1t, g1d, g2t, g2d, intro, np.zeros(30, np.int64))
    assert counts[E.RQ4A_ROWS] == 1600 and counts[E.RQ4A_AFTER_G1] > 0 and counts[E.RQ4A_AFTER_G2] > 0
    after = {"g1": (float(sc[E.RQ4A_AFTER_G1_MEDIAN]), float(sc[E.RQ4A_AFTER_G1_IQR])),
             "g2": (float(sc[E.RQ4A_AFTER_G2_MEDIAN]), float(sc[E.RQ4A_AFTER_G2_IQR]))}
    rows = common.rq4a_rows(g1t, g1d, g2t, g2d)
    assert render.rq4a_trend_lines(rows, after) == shipped.RQ4A_MAIN_LINES
    istats = (float(sc[E.RQ4A_INTRO_MEAN]), float(sc[E.RQ4A_INTRO_MEDIAN]), int(sc[E.RQ4A_INTRO_MIN]),
              int(sc[E.RQ4A_INTRO_MAX]))
    assert render.rq4a_intro_lines(int((intro > 0).sum()), istats)[:3] == shipped.RQ4A_INTRO_LINES
    steps = {s: [0, 0] for s in list(range(-7, 0)) + list(range(1, 8))}
    ref_after, ref_istats, _ = orc.rq4a_finish(g1t, g1d, g2t, g2d, intro.tolist(), steps)
    assert_same(after, ref_after, "after")
    assert_same(istats, ref_istats, "intro_stats")


def test_rq3_stats_shipped(engine):
    """fz_rq3_stats on the shipped detected sample (5,465 changes): the summary tables are the
    reference's own printout, the Anderson-Darling statistic / critical values match scipy."""
    pct, cov, tot = shipped.detected_changes()
    desc, tests = engine.rq3_stats(pct, tot, pct[:64])
    o = render.Rendered()
    render._summary(o, compute._describe(E.describe_from_doubles(desc[0])), "Detected")
    render._summary(o, compute._describe(E.describe_from_doubles(desc[2])), "Detected Total")
    gold = open(shipped.DIR + "/rq3_detected_stdout.txt").read()
    assert gold.startswith(o.text())
    r = stats.anderson(list(pct), dist="norm")
    assert abs(tests[E.RQ3_AD_DET] - r.statistic) <= 1e-9 * abs(r.statistic)
    assert np.array_equal(tests[E.RQ3_AD_DET + 1:E.RQ3_AD_DET + 6], r.critical_values)
    ref = orc.rq3_stats(pct, tot, pct[:64])
    assert_same(compute._describe(E.describe_from_doubles(desc[0])), ref["desc_detected"], "desc_detected")
    assert_same(compute._describe(E.describe_from_doubles(desc[2])), ref["desc_det_total"], "desc_det_total")


def test_change_analysis_shipped(engine):
    """The store + fz_rq2_add on the tables inverted from the 854 shipped change_analysis files
    (358,540 builds, 661k coverage rows in heap order) regenerates every file byte for byte."""
    t = shipped.change_analysis_tables()
    engine.upload(t)
    engine.build_store()
    r = compute.rq2_add(engine)
    assert len(r.row_project) == 270347
    errs = shipped.check_change_files(render.rq2_add(r, t).files)
    assert not errs, "\n".join(errs)
    assert_same(r, orc.rq2_add(t), "rq2_add")


@pytest.mark.parametrize("nd", [1, 2, 3])
def test_rq3_stats_tiny_samples(engine, nd):
    """fz_rq3_stats with one to three detected changes (a shard's gathered sample can be that small):
    every statistic as scipy computes it - Anderson-Darling with N = 1 is NaN with scipy's own
    (negative) critical values, no error - checked against the oracle (scipy 1.15.3)."""
    rng = np.random.default_rng(nd)
    det = rng.normal(0, 1, size=nd)
    tot = rng.integers(-5, 5, size=nd)
    non = rng.normal(0.2, 2, size=40)
    desc, tests = engine.rq3_stats(det, tot, non)
    ref = orc.rq3_stats(det, tot, non)
    assert_same(compute._describe(E.describe_from_doubles(desc[0])), ref["desc_detected"], "desc_detected")
    ad = (float(tests[E.RQ3_AD_DET]), tests[E.RQ3_AD_DET + 1:E.RQ3_AD_DET + 6])
    assert_same(ad, ref["anderson_det"], "anderson_det")
    assert_same((float(tests[E.RQ3_LEVENE_W]), float(tests[E.RQ3_LEVENE_P])), ref["levene"], "levene")
    assert_same((float(tests[E.RQ3_BM_STAT]), float(tests[E.RQ3_BM_P])), ref["brunnermunzel"], "brunnermunzel")
