"""The multi-core C++ CPU baseline (oracle/cpu/fz_cpu.cpp, bench.py's cpu_baseline leg) computes
what the oracle computes: every output of the six analyses on both golden cases, integers exactly,
floating point within 1e-9 relative (it sums in long double / a different order than numpy).
Run with 1 and 4 threads: the result must not depend on the thread count."""
import numpy as np
import pytest

import goldens
from oracle import cpu_baseline as cb
from oracle import rq_oracle as orc
from tse_amd.schema import LIMIT_US, RQ3_LIMIT_US

RTOL = 1e-9


@pytest.fixture(scope="module", params=goldens.CASES)
def case(request):
    t = goldens.tables(request.param)
    host = cb.HostTables(t)
    return t, host


def _f(a, b, what):
    a = np.asarray(a, np.float64).ravel()
    b = np.asarray(b, np.float64).ravel()
    assert a.shape == b.shape, f"{what}: shape {a.shape} vs {b.shape}"
    np.testing.assert_allclose(a, b, rtol=RTOL, atol=1e-12, equal_nan=True, err_msg=what)


def _i(a, b, what):
    a = np.asarray(a, np.int64).ravel()
    b = np.asarray(b, np.int64).ravel()
    assert a.shape == b.shape, f"{what}: shape {a.shape} vs {b.shape}"
    assert np.array_equal(a, b), what


def _desc(d, rq3=True):
    if d is None:
        return []
    if rq3:
        return [d.count, d.n_pos, d.n_zero, d.n_neg, d.mean, d.median, d.std, d.min, d.max, d.q1, d.q3]
    return [d.count, d.n_zero, d.min, d.max, d.q1, d.q3, d.median, d.mean,
            np.nan if d.min_nonzero is None else d.min_nonzero]


def test_limits_match_schema():
    lib = cb.load()
    assert lib.fzcpu_limit_us(0) == LIMIT_US and lib.fzcpu_limit_us(1) == RQ3_LIMIT_US


@pytest.mark.parametrize("threads", [1, 4])
def test_cpu_baseline_matches_oracle(case, threads):
    t, host = case
    out, secs = cb.run(host, threads=threads)
    assert set(secs) == set(cb.TIMES)
    check_port(out, {"rq1": orc.rq1(t), "rq2_count": orc.rq2_count(t), "rq2_add": orc.rq2_add(t), "rq3": orc.rq3(t),
                     "rq4a": orc.rq4a(t), "rq4b": orc.rq4b(t)})


def check_port(out, res):
    """Every output of the C++ port (out) against result objects of the six analyses (res: the
    oracle's, or the GPU engine's - rq/results.py dataclasses, the same fields)."""
    # RQ1
    r = res["rq1"]
    _i(out["rq1_counts"], [r.n_issues_lim, r.n_issues_lim_projects, r.n_fixed_lim, r.n_fixed_lim_projects,
                           len(r.eligible), r.n_without_matching, r.n_target, r.n_target_projects,
                           r.total_fuzz_builds, len(r.matched_issue), r.n_matched_projects], "rq1 counts")
    _i(out["rq1_iter_total"], r.iter_total, "rq1 iter_total")
    _i(out["rq1_iter_detected"], r.iter_detected, "rq1 iter_detected")
    _i(out["rq1_matched_issue"], r.matched_issue, "rq1 matched_issue")
    _i(out["rq1_matched_build"], r.matched_build, "rq1 matched_build")
    _f(out["rq1_late"], _desc(r.late, rq3=False), "rq1 late")
    # RQ2 count
    r = res["rq2_count"]
    _i(out["rq2c_raw_n"], r.raw_n, "rq2c raw_n")
    _i(out["rq2c_n_trend"], r.n_trend, "rq2c n_trend")
    _f(out["rq2c_sw_w"], r.sw_w, "rq2c sw_w")
    _f(out["rq2c_sw_p"], r.sw_p, "rq2c sw_p")
    _f(out["rq2c_corr"], r.corr, "rq2c corr")
    _i(out["rq2c_session_offsets"], r.session_offsets, "rq2c session offsets")
    _f(out["rq2c_session_values"], r.session_values, "rq2c session values")
    sp = r.spearman_median or (np.nan, np.nan)
    _f(out["rq2c_scalars"], [r.corr_mean, r.corr_median, sp[0], sp[1],
                             np.nan if r.shapiro_median_p is None else r.shapiro_median_p], "rq2c scalars")
    _f(out["rq2c_average"], r.average_trend, "rq2c average")
    _f(out["rq2c_median"], r.median_trend, "rq2c median")
    _f(out["rq2c_pct"], r.dist_percentiles, "rq2c percentiles")
    _f(out["rq2c_dist_mean"], r.dist_mean, "rq2c dist mean")
    # RQ2 add
    r = res["rq2_add"]
    rows = np.stack([r.row_project, r.row_first_build, r.row_end_build, r.row_start_build, r.row_cov_i,
                     r.row_cov_i1], axis=1) if len(r.row_project) else np.zeros((0, 6), np.int64)
    _i(out["rq2a_rows"], rows, "rq2a rows")
    _f(out["rq2a_diff_total"], r.diff_total, "rq2a diff_total")
    _f(out["rq2a_diff_coverage"], r.diff_coverage, "rq2a diff_coverage")
    _i(out["rq2a_flags"], np.stack([r.covered_is_float, r.total_is_float], axis=1), "rq2a flags")
    # RQ3
    r = res["rq3"]
    _i(out["rq3_counts"], [r.n_all_issues, len(r.det_pct), len(r.non_pct)], "rq3 counts")
    _f(out["rq3_det_pct"], r.det_pct, "rq3 det_pct")
    _f(out["rq3_non_pct"], r.non_pct, "rq3 non_pct")
    _i(out["rq3_det_cols"], np.stack([r.det_cov, r.det_tot, r.det_project, r.det_issue], axis=1), "rq3 det cols")
    _i(out["rq3_non_cols"], np.stack([r.non_cov, r.non_tot], axis=1), "rq3 non cols")
    _f(out["rq3_describe"], _desc(r.desc_detected) + _desc(r.desc_non) + _desc(r.desc_det_total), "rq3 describe")
    tests = []
    if r.anderson_det is not None:
        tests = [r.anderson_det[0], *r.anderson_det[1], r.anderson_non[0], *r.anderson_non[1], *r.levene,
                 *r.brunnermunzel]
    _f(out["rq3_tests"], tests, "rq3 tests")
    # RQ4a
    r = res["rq4a"]
    _i(out["rq4a_g1_total"], r.g1_total, "rq4a g1_total")
    _i(out["rq4a_g1_det"], r.g1_det, "rq4a g1_det")
    _i(out["rq4a_g2_total"], r.g2_total, "rq4a g2_total")
    _i(out["rq4a_g2_det"], r.g2_det, "rq4a g2_det")
    _i(out["rq4a_intro"], [x for pk in r.intro for x in pk], "rq4a intro")
    _i(out["rq4a_steps"], [v for s in list(range(-7, 0)) + list(range(1, 8)) for v in r.g4_steps[s]], "rq4a steps")
    _i(out["rq4a_transition"], list(r.g4_transition) + [int(r.has_g4_transition)], "rq4a transition")
    after = [x for k in ("g1", "g2") for x in (r.after[k] or (np.nan, np.nan))]
    intro = list(r.intro_stats) if r.intro_stats else [np.nan] * 4
    _f(out["rq4a_scalars"], after + intro + list(r.g4_overall), "rq4a scalars")
    # RQ4b
    r = res["rq4b"]
    _i(out["rq4b_c2"], r.c2, "rq4b c2")
    _i(out["rq4b_c1"], r.c1, "rq4b c1")
    _f(out["rq4b_g2_q"], r.g2_q, "rq4b g2 quartiles")
    _f(out["rq4b_g1_q"], r.g1_q, "rq4b g1 quartiles")
    _f(out["rq4b_p_bm"], r.p_bm, "rq4b p_bm")
    _i(out["rq4b_last"], [r.last_valid_idx], "rq4b last")
    _f(out["rq4b_spearman6"], [x for pr in (r.spearman6 or []) for x in pr], "rq4b spearman6")
    _f(out["rq4b_pre"], np.concatenate(r.pre_cov), "rq4b pre")
    _f(out["rq4b_post"], np.concatenate(r.post_cov), "rq4b post")
    _f(out["rq4b_medians"], list(r.pre_median) + list(r.post_median), "rq4b medians")
    _f(out["rq4b_init_g2"], r.init_g2, "rq4b init g2")
    _f(out["rq4b_init_g1"], r.init_g1, "rq4b init g1")
    tests = [] if r.mwu_p is None else [r.mwu_p, r.cliff, *r.bm, *r.levene]
    _f(out["rq4b_tests"], tests, "rq4b tests")
