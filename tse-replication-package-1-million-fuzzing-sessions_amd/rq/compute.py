"""GPU compute path: each function runs one reference script's analysis through ``libfz`` and
returns the same result object the CPU oracle produces (``tse_amd.rq.results``).

Only O(iterations) / O(projects) bookkeeping happens here on the host (unpacking counts,
building Python lists for the renderer); every per-row computation is a HIP kernel.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import engine as E
from .results import Describe, RQ1Result, RQ2AddResult, RQ2CountResult, RQ3Result, RQ4aResult, RQ4bResult


def _describe(d: E.FzDescribe, with_min_nonzero=False) -> Describe:
    return Describe(count=int(d.count), n_pos=int(d.n_pos), n_zero=int(d.n_zero), n_neg=int(d.n_neg),
                    mean=float(d.mean), median=float(d.median), std=float(d.std), min=float(d.min),
                    max=float(d.max), q1=float(d.q1), q3=float(d.q3),
                    min_nonzero=(float(d.min_nonzero) if (with_min_nonzero and d.has_nonzero) else None))


class RQ1Buffers:
    """Device outputs of fz_rq1, allocated once per store (re-used across bench steps)."""

    def __init__(self, eng: E.Engine, max_iter: int = 0):
        torch = eng.torch
        fz = eng.tables.fz
        # max_iter: the iteration axis agreed across shards (parallel.agree_max), >= the local one
        M = max(int(eng.stats.max_fuzz_per_project), int(max_iter), 1)
        self.counts = eng.zeros(E.FZ_RQ1_NCOUNTS, torch.int64)
        self.eligible = eng.zeros(fz.n_projects, torch.uint8)
        self.iter_total = eng.zeros(M, torch.int64)
        self.iter_detected = eng.zeros(M, torch.int64)
        self.matched_issue = eng.zeros(fz.n_issues, torch.int64)
        self.matched_build = eng.zeros(fz.n_issues, torch.int64)
        self.late = eng.zeros(E.DESCRIBE_DOUBLES, torch.float64)
        self.out = E.FzRq1Out(*[C.c_void_p(b.data_ptr()) for b in (
            self.counts, self.eligible, self.iter_total, self.iter_detected, self.matched_issue,
            self.matched_build, self.late)])


def rq1_launch(eng: E.Engine, bufs: RQ1Buffers, threshold: int = 100):
    """Enqueue RQ1 on the engine stream (no host synchronisation)."""
    E._check(eng.lib, eng.lib.fz_rq1(eng.ctx, threshold, C.byref(bufs.out)))


def rq1_collect(eng: E.Engine, bufs: RQ1Buffers, threshold: int = 100) -> RQ1Result:
    cnt = bufs.counts.cpu().numpy()
    n_match = int(cnt[E.RQ1_MATCHED])
    M = int(cnt[E.RQ1_MAX_ITER])
    return rq1_result(cnt, bufs.iter_total[:M].cpu().numpy(), bufs.iter_detected[:M].cpu().numpy(),
                      bufs.late.cpu().numpy(), bufs.matched_issue[:n_match].cpu().numpy(),
                      bufs.matched_build[:n_match].cpu().numpy(),
                      np.nonzero(bufs.eligible.cpu().numpy()[:eng.tables.fz.n_projects])[0], threshold)


def rq1_result(cnt, iter_total, iter_detected, late_doubles, matched_issue, matched_build, eligible,
               threshold: int = 100) -> RQ1Result:
    """RQ1Result from fz_rq1's counters and arrays (host copies; also the sharded recombination)."""
    late = None
    if cnt[E.RQ1_LATE] > 0:
        d = _describe(E.describe_from_doubles(late_doubles), with_min_nonzero=True)
        # rq1_detection_rate.py:256-268 reports only these numbers (no sign split, no std)
        late = Describe(count=d.count, n_zero=d.n_zero, min=d.min, max=d.max, q1=d.q1, q3=d.q3,
                        median=d.median, mean=d.mean, min_nonzero=d.min_nonzero)
    elig = np.asarray(eligible)
    return RQ1Result(
        n_issues_lim=int(cnt[E.RQ1_ISSUES_LIM]), n_issues_lim_projects=int(cnt[E.RQ1_ISSUES_LIM_PROJECTS]),
        n_fixed_lim=int(cnt[E.RQ1_FIXED_LIM]), n_fixed_lim_projects=int(cnt[E.RQ1_FIXED_LIM_PROJECTS]),
        eligible=elig, n_without_matching=int(cnt[E.RQ1_WITHOUT_MATCHING]),
        n_target=int(cnt[E.RQ1_TARGET]), n_target_projects=int(cnt[E.RQ1_TARGET_PROJECTS]),
        total_fuzz_builds=int(cnt[E.RQ1_TOTAL_FUZZ]),
        matched_issue=np.asarray(matched_issue), matched_build=np.asarray(matched_build),
        n_matched_projects=int(cnt[E.RQ1_MATCHED_PROJECTS]),
        iter_total=np.asarray(iter_total), iter_detected=np.asarray(iter_detected),
        min_project_threshold=threshold, late=late)


def rq1(eng: E.Engine, threshold: int = 100) -> RQ1Result:
    """rq1_detection_rate.collect_and_analyze_data (rq1_detection_rate.py:101-269) on the GPU."""
    bufs = RQ1Buffers(eng)
    rq1_launch(eng, bufs, threshold)
    return rq1_collect(eng, bufs, threshold)


class OutBuffers:
    """Device buffers for one fz_* output struct: spec = [(field, n, torch dtype)] in struct order."""

    def __init__(self, eng: E.Engine, struct_cls, spec, null=()):
        self.names = [n for n, _, _ in spec]
        for name, n, dt in spec:
            setattr(self, name, eng.zeros(n, dt))
        self.out = struct_cls(*[None if n in null else C.c_void_p(getattr(self, n).data_ptr()) for n in self.names])

    def host(self, name, n=None):
        a = getattr(self, name)
        return (a if n is None else a[:n]).cpu().numpy()


# ------------------------------------------------------------------------------------ RQ2 count
def rq2_count_buffers(eng: E.Engine) -> OutBuffers:
    torch = eng.torch
    fz, st = eng.tables.fz, eng.stats
    P, M, NC = fz.n_projects, max(int(st.max_cov_per_project), 1), fz.n_cov
    f64, i64, u8 = torch.float64, torch.int64, torch.uint8
    return OutBuffers(eng, E.FzRq2CountOut, [
        ("counts", E.FZ_RQ2C_NCOUNTS, i64), ("scalars", E.FZ_RQ2C_NSCALARS, f64), ("eligible", P, u8),
        ("raw_n", P, i64), ("n_trend", P, i64), ("sw_w", P, f64), ("sw_p", P, f64), ("corr", P, f64),
        ("session_offsets", M + 2, i64), ("session_values", NC, f64), ("average_trend", M, f64),
        ("median_trend", M, f64), ("dist_percentiles", 5 * M, f64), ("dist_mean", M, f64)])


def rq2_count_launch(eng: E.Engine, b: OutBuffers):
    E._check(eng.lib, eng.lib.fz_rq2_count(eng.ctx, C.byref(b.out)))


def rq2_count_collect(eng: E.Engine, b: OutBuffers) -> RQ2CountResult:
    P = eng.tables.fz.n_projects
    cnt = b.host("counts")
    sc = b.host("scalars")
    ns, K, nv = int(cnt[E.RQ2C_SESSIONS]), int(cnt[E.RQ2C_GE100]), int(cnt[E.RQ2C_VALUES])
    return rq2_count_result(
        {k: b.host(k, P) for k in ("eligible", "raw_n", "n_trend", "sw_w", "sw_p", "corr")},
        b.host("session_offsets", ns + 1), b.host("session_values", nv), K, b.host("average_trend", K),
        b.host("median_trend", K), b.host("dist_percentiles", 5 * K), b.host("dist_mean", K),
        (float(sc[E.RQ2C_SP_RHO]), float(sc[E.RQ2C_SP_P]), float(sc[E.RQ2C_SW_MEDIAN_P])),
        (float(sc[E.RQ2C_CORR_MEAN]), float(sc[E.RQ2C_CORR_MEDIAN])), null_lines=int(cnt[E.RQ2C_NULL_LINES]))


def rq2_count_result(proj, session_offsets, session_values, K, average, median, pct_flat, dist_mean, tests,
                     corr_mm, null_lines: int = 0) -> RQ2CountResult:
    """RQ2CountResult from per-project columns (full project axis), the session-major values and the
    per-session / median-trend statistics (host copies; also the sharded recombination).  Raises
    TypeError as the reference does (rq2_coverage_count.py:300-303: ``float(None)``) when a fetched
    row with a non-zero or NULL total_line has a NULL line count (counts[FZ_RQ2C_NULL_LINES])."""
    if null_lines:
        raise TypeError("float() argument must be a string or a real number, not 'NoneType'")
    elig = np.nonzero(np.asarray(proj["eligible"]))[0]
    raw_n = np.asarray(proj["raw_n"])[elig]
    corr = np.asarray(proj["corr"])[elig][raw_n > 0]
    pct = np.asarray(pct_flat)[:5 * K].reshape(K, 5).T.copy() if K else np.zeros((5, 0))
    return RQ2CountResult(
        eligible=elig, raw_n=raw_n, n_trend=np.asarray(proj["n_trend"])[elig], sw_w=np.asarray(proj["sw_w"])[elig],
        sw_p=np.asarray(proj["sw_p"])[elig], corr=corr, session_offsets=np.asarray(session_offsets),
        session_values=np.asarray(session_values), corr_mean=float(corr_mm[0]), corr_median=float(corr_mm[1]),
        ge100=np.arange(K, dtype=np.int64), average_trend=np.asarray(average)[:K], median_trend=np.asarray(median)[:K],
        spearman_median=(float(tests[0]), float(tests[1])) if K > 1 else None,
        shapiro_median_p=float(tests[2]) if K >= 3 else None, dist_percentiles=pct, dist_mean=np.asarray(dist_mean)[:K])


def rq2_count(eng: E.Engine) -> RQ2CountResult:
    """rq2_coverage_count.main's analysis (rq2_coverage_count.py:244-483) on the GPU."""
    b = rq2_count_buffers(eng)
    rq2_count_launch(eng, b)
    return rq2_count_collect(eng, b)


# -------------------------------------------------------------------------------------- RQ2 add
def rq2_add_buffers(eng: E.Engine) -> OutBuffers:
    torch = eng.torch
    fz, st = eng.tables.fz, eng.stats
    P, NB = fz.n_projects, max(int(st.n_coverage_builds), 1)
    f64, i64, u8 = torch.float64, torch.int64, torch.uint8
    return OutBuffers(eng, E.FzRq2AddOut, [
        ("counts", E.FZ_RQ2A_NCOUNTS, i64), ("eligible", P, u8), ("row_project", NB, i64),
        ("row_first_build", NB, i64), ("row_end_build", NB, i64), ("row_start_build", NB, i64),
        ("row_cov_i", NB, i64), ("row_cov_i1", NB, i64), ("diff_total", NB, f64), ("diff_coverage", NB, f64),
        ("covered_is_float", P, u8), ("total_is_float", P, u8)])


def rq2_add_launch(eng: E.Engine, b: OutBuffers):
    E._check(eng.lib, eng.lib.fz_rq2_add(eng.ctx, C.byref(b.out)))


def rq2_add_collect(eng: E.Engine, b: OutBuffers) -> RQ2AddResult:
    P = eng.tables.fz.n_projects
    n = int(b.host("counts")[E.RQ2A_ROWS])
    return RQ2AddResult(
        projects=np.nonzero(b.host("eligible", P))[0], row_project=b.host("row_project", n),
        row_first_build=b.host("row_first_build", n), row_end_build=b.host("row_end_build", n),
        row_start_build=b.host("row_start_build", n), row_cov_i=b.host("row_cov_i", n),
        row_cov_i1=b.host("row_cov_i1", n), diff_total=b.host("diff_total", n),
        diff_coverage=b.host("diff_coverage", n), covered_is_float=b.host("covered_is_float", P).astype(bool),
        total_is_float=b.host("total_is_float", P).astype(bool))


def rq2_add(eng: E.Engine) -> RQ2AddResult:
    """rq2_coverage_and_added.analyze_coverage_change (rq2_coverage_and_added.py:73-238) on the GPU."""
    b = rq2_add_buffers(eng)
    rq2_add_launch(eng, b)
    return rq2_add_collect(eng, b)


# ------------------------------------------------------------------------------------------ RQ3
def rq3_buffers(eng: E.Engine) -> OutBuffers:
    torch = eng.torch
    fz = eng.tables.fz
    P, NI, NC = fz.n_projects, fz.n_issues, fz.n_cov
    f64, i64, u8 = torch.float64, torch.int64, torch.uint8
    return OutBuffers(eng, E.FzRq3Out, [
        ("counts", E.FZ_RQ3_NCOUNTS, i64), ("eligible", P, u8), ("det_pct", NI, f64), ("det_cov", NI, i64),
        ("det_tot", NI, i64), ("det_project", NI, i64), ("det_issue", NI, i64), ("non_pct", NC, f64),
        ("non_cov", NC, i64), ("non_tot", NC, i64), ("describe", 3 * E.DESCRIBE_DOUBLES, f64),
        ("tests", E.FZ_RQ3_NTESTS, f64)])


def rq3_launch(eng: E.Engine, b: OutBuffers):
    E._check(eng.lib, eng.lib.fz_rq3(eng.ctx, C.byref(b.out)))


def rq3_main_launch(eng: E.Engine, b: OutBuffers):
    """fz_rq3_ex without the statistics (the samples and counts only)."""
    E._check(eng.lib, eng.lib.fz_rq3_ex(eng.ctx, E.FZ_RQ3_SKIP_STATS, C.byref(b.out)))


def rq3_stats_launch(eng: E.Engine, b: OutBuffers):
    """fz_rq3_stats_dn over the samples of a preceding rq3_main_launch (device lengths: may run on
    another stream ordered after it)."""
    fz = eng.tables.fz
    P = lambda t, k=0: C.c_void_p(t.data_ptr() + 8 * k)  # noqa: E731
    E._check(eng.lib, eng.lib.fz_rq3_stats_dn(eng.ctx, P(b.det_pct), P(b.det_tot), fz.n_issues,
                                              P(b.counts, E.RQ3_DETECTED), P(b.non_pct), fz.n_cov,
                                              P(b.counts, E.RQ3_NON_DETECTED), P(b.describe), P(b.tests)))


RQ3_COLUMNS = ("det_pct", "det_cov", "det_tot", "det_project", "det_issue", "non_pct", "non_cov", "non_tot")


def rq3_collect(eng: E.Engine, b: OutBuffers) -> RQ3Result:
    cnt = b.host("counts")
    nd, nn = int(cnt[E.RQ3_DETECTED]), int(cnt[E.RQ3_NON_DETECTED])
    cols = {k: b.host(k, nd if k.startswith("det") else nn) for k in RQ3_COLUMNS}
    return rq3_result(cnt, cols, b.host("describe"), b.host("tests"))


def rq3_result(cnt, cols, describe_doubles, tests) -> RQ3Result:
    """RQ3Result from fz_rq3's counters, columns and statistics (also the sharded recombination).
    Raises TypeError as the reference does (rq3:253,297: ``None > 0``) when a coverage pair it
    examines has a NULL total_line (counts[FZ_RQ3_NULL_TOTAL])."""
    if int(cnt[E.RQ3_NULL_TOTAL]) > int(cnt[E.RQ3_NULL_LAST]):
        raise TypeError("'>' not supported between instances of 'NoneType' and 'int'")
    nd, nn = len(cols["det_pct"]), len(cols["non_pct"])
    desc = np.asarray(describe_doubles).reshape(3, E.DESCRIBE_DOUBLES)
    ts = np.asarray(tests)
    both = nd > 0 and nn > 0
    return RQ3Result(
        n_all_issues=int(cnt[E.RQ3_ISSUES]), **{k: np.asarray(cols[k]) for k in RQ3_COLUMNS},
        desc_detected=_describe(E.describe_from_doubles(desc[0])) if nd else None,
        desc_non=_describe(E.describe_from_doubles(desc[1])) if nn else None,
        desc_det_total=_describe(E.describe_from_doubles(desc[2])) if nd else None,
        anderson_det=(float(ts[E.RQ3_AD_DET]), ts[E.RQ3_AD_DET + 1:E.RQ3_AD_DET + 6].copy()) if both else None,
        anderson_non=(float(ts[E.RQ3_AD_NON]), ts[E.RQ3_AD_NON + 1:E.RQ3_AD_NON + 6].copy()) if both else None,
        levene=(float(ts[E.RQ3_LEVENE_W]), float(ts[E.RQ3_LEVENE_P])) if both else None,
        brunnermunzel=(float(ts[E.RQ3_BM_STAT]), float(ts[E.RQ3_BM_P])) if both else None,
        n_non_last=int(cnt[E.RQ3_NON_LAST]), n_null_total=int(cnt[E.RQ3_NULL_TOTAL]),
        n_null_last=int(cnt[E.RQ3_NULL_LAST]))


def rq3(eng: E.Engine) -> RQ3Result:
    """rq3_diff_coverage_at_detection.main's analysis (rq3_diff_coverage_at_detection.py:202-360)."""
    b = rq3_buffers(eng)
    rq3_launch(eng, b)
    return rq3_collect(eng, b)


def _groups(member, P):
    return {f"group{k + 1}": np.nonzero(member[:P] & (1 << k))[0].tolist() for k in range(4)}


# ----------------------------------------------------------------------------------------- RQ4a
def rq4a_buffers(eng: E.Engine, max_iter: int = 0) -> OutBuffers:
    torch = eng.torch
    fz, st = eng.tables.fz, eng.stats
    P, M = fz.n_projects, max(int(st.max_fuzz_per_project), int(max_iter), 1)
    f64, i64, u8 = torch.float64, torch.int64, torch.uint8
    return OutBuffers(eng, E.FzRq4aOut, [
        ("counts", E.FZ_RQ4A_NCOUNTS, i64), ("scalars", E.FZ_RQ4A_NSCALARS, f64), ("eligible", P, u8),
        ("member", P, u8), ("g1_total", M, i64), ("g1_det", M, i64), ("g2_total", M, i64), ("g2_det", M, i64),
        ("intro", P, i64), ("g4_steps", 30, i64), ("g4_transition", 4, i64)])


def rq4a_launch(eng: E.Engine, b: OutBuffers):
    E._check(eng.lib, eng.lib.fz_rq4a(eng.ctx, C.byref(eng.groups), C.byref(b.out)))


def rq4a_collect(eng: E.Engine, b: OutBuffers) -> RQ4aResult:
    P = eng.tables.fz.n_projects
    mx = int(b.host("counts")[E.RQ4A_MAX_ITER])
    return rq4a_result(b.host("counts"), b.host("scalars"), b.host("member", P),
                       [b.host(k, mx) for k in ("g1_total", "g1_det", "g2_total", "g2_det")], b.host("intro", P),
                       b.host("g4_steps"), b.host("g4_transition"))


def rq4a_result(cnt, sc, member, tables, intro_a, steps_flat, transition) -> RQ4aResult:
    """RQ4aResult from fz_rq4a's outputs (host copies; also the sharded recombination)."""
    P = len(member)
    groups = _groups(np.asarray(member), P)
    steps = np.asarray(steps_flat).reshape(15, 2)
    after = {}
    for key, n, med, iqr in (("g1", E.RQ4A_AFTER_G1, E.RQ4A_AFTER_G1_MEDIAN, E.RQ4A_AFTER_G1_IQR),
                             ("g2", E.RQ4A_AFTER_G2, E.RQ4A_AFTER_G2_MEDIAN, E.RQ4A_AFTER_G2_IQR)):
        after[key] = (float(sc[med]), float(sc[iqr])) if cnt[n] > 0 else None
    g1t, g1d, g2t, g2d = (np.asarray(x) for x in tables)
    return RQ4aResult(
        groups=groups, g1_total=g1t, g1_det=g1d, g2_total=g2t, g2_det=g2d, after=after,
        intro=[(p, int(intro_a[p])) for p in groups["group4"] if intro_a[p] >= 0],
        intro_stats=((float(sc[E.RQ4A_INTRO_MEAN]), float(sc[E.RQ4A_INTRO_MEDIAN]), int(sc[E.RQ4A_INTRO_MIN]),
                      int(sc[E.RQ4A_INTRO_MAX])) if cnt[E.RQ4A_INTRO_POS] > 0 else None),
        g4_steps={s: (int(steps[s + 7, 0]), int(steps[s + 7, 1])) for s in list(range(-7, 0)) + list(range(1, 8))},
        g4_transition=tuple(int(x) for x in transition),
        g4_overall=(float(sc[E.RQ4A_PRE_RATE]), float(sc[E.RQ4A_POST_RATE])), n_g4_analyzed=int(steps[6, 0]),
        has_g4_transition=bool(cnt[E.RQ4A_HAS_WINDOW]))


def rq4a(eng: E.Engine) -> RQ4aResult:
    """rq4a_bug.main's analysis (rq4a_bug.py:653-884) on the GPU."""
    b = rq4a_buffers(eng)
    rq4a_launch(eng, b)
    return rq4a_collect(eng, b)


# ----------------------------------------------------------------------------------------- RQ4b
def rq4b_buffers(eng: E.Engine, shard: bool = False) -> OutBuffers:
    """shard=False leaves the shard-only outputs (trend series, delta projects) NULL."""
    torch = eng.torch
    fz, st = eng.tables.fz, eng.stats
    P, M = fz.n_projects, max(int(st.max_cov_per_project), 1)
    PP = max(P, 1)
    f64, i64, u8 = torch.float64, torch.int64, torch.uint8
    return OutBuffers(eng, E.FzRq4bOut, [
        ("counts", E.FZ_RQ4B_NCOUNTS, i64), ("eligible", P, u8), ("member", P, u8), ("c2", M, i64), ("c1", M, i64),
        ("g2_q", 3 * M, f64), ("g1_q", 3 * M, f64), ("p_bm", M, f64), ("spearman6", 12, f64),
        ("pre_cov", 7 * PP, f64), ("post_cov", 7 * PP, f64), ("pre_median", 7, f64), ("post_median", 7, f64),
        ("init_g2", P, f64), ("init_g1", P, f64), ("tests", E.FZ_RQ4B_NTESTS, f64),
        ("trend_values", fz.n_cov if shard else 0, f64), ("trend_offsets", max(2 * M, P) + 1 if shard else 0, i64),
        ("delta_order", P if shard else 0, i64)], null=() if shard else ("trend_values", "trend_offsets",
                                                                         "delta_order"))


def rq4b_launch(eng: E.Engine, b: OutBuffers):
    E._check(eng.lib, eng.lib.fz_rq4b(eng.ctx, C.byref(eng.groups), C.byref(b.out)))


def rq4b_collect(eng: E.Engine, b: OutBuffers) -> RQ4bResult:
    cnt, ts = b.host("counts"), b.host("tests")
    ms, nd = int(cnt[E.RQ4B_SESSIONS]), int(cnt[E.RQ4B_DELTA_PROJECTS])
    n2, n1 = int(cnt[E.RQ4B_INIT_G2]), int(cnt[E.RQ4B_INIT_G1])
    pre, post = b.host("pre_cov"), b.host("post_cov")
    return rq4b_result(cnt, b.host("c2", ms), b.host("c1", ms), b.host("g2_q", 3 * ms), b.host("g1_q", 3 * ms),
                       b.host("p_bm", ms), b.host("spearman6"), [pre[i * nd:(i + 1) * nd].copy() for i in range(7)],
                       [post[i * nd:(i + 1) * nd].copy() for i in range(7)], b.host("pre_median"),
                       b.host("post_median"), b.host("init_g2", n2), b.host("init_g1", n1), ts)


def rq4b_result(cnt, c2, c1, g2_q, g1_q, p_bm, sp6, pre_cov, post_cov, pre_median, post_median, init_g2, init_g1,
                tests) -> RQ4bResult:
    """RQ4bResult from fz_rq4b's outputs (host copies; also the sharded recombination)."""
    ms, last = len(c2), int(cnt[E.RQ4B_LAST])
    both = len(init_g2) > 0 and len(init_g1) > 0
    return RQ4bResult(
        group_counts=tuple(int(cnt[k]) for k in (E.RQ4B_G1, E.RQ4B_G2, E.RQ4B_G3, E.RQ4B_G4)), n_sessions=ms,
        c2=np.asarray(c2), c1=np.asarray(c1), g2_q=np.asarray(g2_q).reshape(ms, 3),
        g1_q=np.asarray(g1_q).reshape(ms, 3), p_bm=np.asarray(p_bm), last_valid_idx=last,
        spearman6=[(float(sp6[2 * k]), float(sp6[2 * k + 1])) for k in range(6)] if last >= 0 else None,
        n_delta_projects=len(pre_cov[0]) if len(pre_cov) else 0, pre_cov=pre_cov, post_cov=post_cov,
        pre_median=[float(x) for x in pre_median], post_median=[float(x) for x in post_median],
        n_g2=int(cnt[E.RQ4B_G2]), n_g1=int(cnt[E.RQ4B_G1]), init_g2=np.asarray(init_g2), init_g1=np.asarray(init_g1),
        mwu_p=float(tests[E.RQ4B_MWU_P]) if both else None, cliff=float(tests[E.RQ4B_CLIFF]) if both else None,
        bm=(float(tests[E.RQ4B_BM_STAT]), float(tests[E.RQ4B_BM_P])) if both else None,
        levene=(float(tests[E.RQ4B_LEVENE_W]), float(tests[E.RQ4B_LEVENE_P])) if both else None)


def rq4b(eng: E.Engine) -> RQ4bResult:
    """rq4b_coverage.main's analysis (rq4b_coverage.py:1209-1261) on the GPU."""
    b = rq4b_buffers(eng)
    rq4b_launch(eng, b)
    return rq4b_collect(eng, b)
