"""CPU checks of the synthetic workloads and of the parity checker."""
import math

import numpy as np
import pytest

import tse_amd.synth as synth
from tse_amd.schema import LIMIT_US
from gpu_common import TAIL, assert_same
from oracle import rq_oracle as orc


def test_config4_shape():
    t = synth.generate(synth.config("c4", n_projects=4, lengths=(100_000, 3_000)))
    counts = np.bincount(t.c_project)
    assert counts.tolist() == [100_000, 3_000, 100_000, 3_000]
    assert t.c_date.max() < LIMIT_US                      # every row inside the analysis window
    v = t.c_coverage[t.c_coverage_valid & (t.c_total > 0)]
    assert len(np.unique(v)) <= 256                       # heavy ties: 256 coverage levels
    # odd projects follow a monotone trend: strongly rank-correlated with time
    rows = np.nonzero((t.c_project == 1) & t.c_coverage_valid & (t.c_total > 0))[0]
    rows = rows[np.argsort(t.c_date[rows])]
    rho, _, _, _ = orc.series_tests(t.c_covered[rows] / t.c_total[rows] * 100)
    assert rho > 0.9


def test_existing_configs_unchanged():
    # the config-4 options are off by default: the golden-case tables keep their fingerprints
    a = synth.generate(synth.config("tiny"))
    b = synth.generate(synth.config("tiny", step_us=synth.US_PER_DAY, tie_levels=None, trend_mix=False))
    assert synth.table_fingerprint(a) == synth.table_fingerprint(b)


def test_series_tests_match_scipy():
    from scipy import stats
    x = np.random.default_rng(0).normal(size=1000)
    r = stats.spearmanr(range(1000), x)
    w = stats.shapiro(x)
    assert orc.series_tests(x) == (float(r[0]), float(r[1]), float(w[0]), float(w[1]))
    assert all(math.isnan(v) for v in orc.series_tests([1.0]))


def test_tail_pvalues_compared_in_log_space():
    assert_same(1.10474276682699e-101, 1.1047427655087815e-101)   # 1.2e-9 rel, 5e-12 rel in -ln p
    with pytest.raises(AssertionError):
        assert_same(1.0e-101, 1.1e-101)
    with pytest.raises(AssertionError):
        assert_same(0.5 * TAIL * 10, 0.5 * TAIL * 10 * (1 + 1e-8))  # above the tail: plain 1e-9 rel
