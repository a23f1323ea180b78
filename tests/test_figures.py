"""The reference's figures, drawn off the critical path from each script's
result object (tse_amd/rq/figures.py): every PDF the reference writes for these inputs appears at
its path (rq1_detection_rate.py:320, rq2_coverage_count.py:326-482, rq3:177-358, rq4a_bug.py:241,
rq4b_coverage.py:635,1117) and is a PDF.  The figure data come from the oracle here (CPU); the GPU
drop-in run (test_gpu_scripts.py) draws them from libfz results through the same code.  PDF bytes
are not a parity target (matplotlib embeds versions and dates)."""
import os

import pytest

import goldens
from oracle import rq_oracle as orc
from tse_amd.rq import figures as F
from tse_amd.rq import render

CASES = {
    "rq1_detection_rate": (orc.rq1, render.rq1),
    "rq2_coverage_count": (orc.rq2_count, render.rq2_count),
    "rq3_diff_coverage_at_detection": (orc.rq3, render.rq3),
    "rq4a_bug": (orc.rq4a, None),
    "rq4b_coverage": (orc.rq4b, None),
}
EXPECTED = {
    "rq1_detection_rate": ["rq1/rq1_detection_rate.pdf"],
    "rq2_coverage_count": ["rq2/all_project_corr_hist.pdf", "rq2/average_median_lineplot.pdf"],
    "rq3_diff_coverage_at_detection": ["rq3/coverage_diff_boxplot.pdf", "rq3/coverage_diff_histograms.pdf",
                                       "rq3/detected.pdf", "rq3/non_detected.pdf"],
    "rq4a_bug": ["rq4/bug/rq4_g1_g2_detection_trend.pdf"],
    "rq4b_coverage": [],
}


@pytest.mark.parametrize("name", list(CASES))
def test_figures_drawn(name, tmp_path):
    t = goldens.tables("medium")
    fn, rend = CASES[name]
    r = fn(t)
    paths = F.draw(F.spec(name, r, t), str(tmp_path))
    base = tmp_path / "data" / "result_data"
    rel = {os.path.relpath(p, base) for p in paths}
    for want in EXPECTED[name]:
        assert want in rel, (name, sorted(rel))
    if rend is not None:  # every figure the renderer announces is drawn at that path
        for path, _ in rend(r, t).figures:
            assert os.path.relpath(path, "data/result_data") in rel, path
    for p in paths:
        with open(p, "rb") as f:
            assert f.read(5) == b"%PDF-", p


def test_side_processes(tmp_path):
    """Several drawing processes: RQ2's per-project figures dealt over them, the rest in one."""
    t = goldens.tables("medium")
    r2 = orc.rq2_count(t)
    specs = [F.spec("rq1_detection_rate", orc.rq1(t), t), F.spec("rq2_coverage_count", r2, t)]
    procs = F.draw_in_side_process(specs, str(tmp_path), workers=3)
    assert len(procs) >= 2
    for p in procs:
        p.join(300)
        assert p.exitcode == 0
    base = tmp_path / "data" / "result_data"
    assert (base / "rq1" / "rq1_detection_rate.pdf").exists()
    want = {os.path.basename(p) for p, _ in render.rq2_count(r2, t).figures}
    assert want and want <= set(os.listdir(base / "rq2" / "projects"))
