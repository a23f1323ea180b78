"""Known-answer tests from the reference's SHIPPED real-data outputs (SURVEY.md 4 item 3, 8(c)
inventory 2-6), on the CPU: the oracle and the host renderer reproduce what the reference printed
or wrote for the real 1-million-session dataset.  The GPU path runs the same vectors in
tests/test_gpu_shipped.py."""
import numpy as np
import pytest
from scipy import stats

import shipped
from oracle import rq_oracle as orc
from tse_amd.rq import common, render


def test_rq1_late_block_oracle():
    """rq1_detection_rate.py:243-268 on the shipped stats CSV prints rq1:401-407 exactly."""
    it, idt = shipped.rq1_tables()
    keys, rates, first_down, late = common.rq1_rates(it, idt, 100)
    assert len(keys) == 2341 and first_down == 27 and len(late) == 2314
    lines = render.rq1_late_lines(orc.rq1_finish(it, idt, 100))
    assert lines[0] == "\n" + shipped.RQ1_LATE_BLOCK[0]
    assert lines[1:] == shipped.RQ1_LATE_BLOCK[1:]


def test_rq4a_trend_csv_bytes():
    """rq4a_bug.py:186-204: the rate columns are repr(det / total * 100) - regenerating the CSV from
    the shipped counts gives the shipped bytes (1,600 rows)."""
    rows = common.rq4a_rows(*shipped.rq4a_tables())
    assert len(rows) == 1600
    assert render.csv_bytes(rows, render._TREND_HDR) == shipped.raw_bytes("rq4_g1_g2_detection_trend.csv")


def test_rq4a_main_lines_oracle():
    g1t, g1d, g2t, g2d = shipped.rq4a_tables()
    intro = [k for _, k in shipped.intro_rows()]
    steps = {s: [0, 0] for s in list(range(-7, 0)) + list(range(1, 8))}
    after, istats, _ = orc.rq4a_finish(g1t, g1d, g2t, g2d, intro, steps)
    rows = common.rq4a_rows(g1t, g1d, g2t, g2d)
    assert render.rq4a_trend_lines(rows, after) == shipped.RQ4A_MAIN_LINES
    n_pos = sum(k > 0 for k in intro)
    assert render.rq4a_intro_lines(n_pos, istats)[:3] == shipped.RQ4A_INTRO_LINES


def test_rq3_detected_summary_oracle():
    """rq3_diff_coverage_at_detection.py:25-66, :329-333 on the shipped detected sample: the
    renderer's tables are the reference's own printout (tests/golden/shipped/rq3_detected_stdout.txt,
    produced by the unmodified reference function) and the Anderson-Darling numbers match."""
    pct, cov, tot = shipped.detected_changes()
    r = orc.rq3_stats(pct, tot, pct[:10])
    o = render.Rendered()
    render._summary(o, r["desc_detected"], "Detected")
    render._summary(o, r["desc_det_total"], "Detected Total")
    gold_text = open(shipped.DIR + "/rq3_detected_stdout.txt").read()
    assert gold_text.startswith(o.text())
    gold = gold_text.split("\n")
    stat_line = [g for g in gold if g.startswith("Test statistic")][0]
    assert float(stat_line.split(":")[1]) == r["anderson_det"][0]
    assert "Critical values: " + str(np.asarray(r["anderson_det"][1])) in gold


def test_change_analysis_files_oracle():
    """rq2_coverage_and_added.py:73-238 on the tables inverted from the 854 shipped per-project
    change_analysis files regenerates every file byte for byte (270,347 rows: the fp64 op order of
    :189-200, pandas' float upcast of the covered/total columns, csv float repr, nan cells)."""
    t = shipped.change_analysis_tables()
    r = orc.rq2_add(t)
    assert len(r.row_project) == sum(v["rows"] for v in shipped.change_analysis_expected().values())
    errs = shipped.check_change_files(render.rq2_add(r, t).files)
    assert not errs, "\n".join(errs)


def test_change_analysis_fixture_shape():
    t = shipped.change_analysis_tables()
    assert len(t.projects) == 854
    # every project is eligible only through its fillers: 365 rows with coverage > 0 before the limit
    assert len(orc.eligible_projects(t)) == 854
    # the NULL row makes every project's covered/total columns float-typed (as in all shipped files)
    assert (~t.c_covered_valid).sum() >= 854
