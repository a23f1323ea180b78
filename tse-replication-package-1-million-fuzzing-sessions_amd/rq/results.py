"""Result objects shared by the GPU compute path and the CPU oracle.

Every field is a plain int / float / numpy array so two results can be compared field by
field (integers bit-exact, floats within the north-star tolerance of 1e-9 relative).
Row indices (``*_issue``, ``*_build``, ``*_cov``) point into the *original* rows of the
``Tables`` the computation ran on, so the renderer can fetch strings (names, modules,
revisions) and raw column values without the compute side ever touching text.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np


@dataclass
class Describe:
    """``print_summary_statistics`` of rq3 (``rq3_diff_coverage_at_detection.py:25-66``) and
    the RQ1 late-stage block (``rq1_detection_rate.py:256-268``)."""
    count: int = 0
    n_pos: int = 0
    n_zero: int = 0
    n_neg: int = 0
    mean: float = float("nan")
    median: float = float("nan")
    std: float = float("nan")          # ddof = 0
    min: float = float("nan")
    max: float = float("nan")
    q1: float = float("nan")           # np.percentile(x, 25), linear
    q3: float = float("nan")
    min_nonzero: Optional[float] = None


@dataclass
class RQ1Result:
    n_issues_lim: int
    n_issues_lim_projects: int
    n_fixed_lim: int
    n_fixed_lim_projects: int
    eligible: np.ndarray               # project ids in query order
    n_without_matching: int
    n_target: int
    n_target_projects: int
    total_fuzz_builds: int
    matched_issue: np.ndarray          # SAME_DATE_BUILD_ISSUE rows (ORDER BY project, rts)
    matched_build: np.ndarray
    n_matched_projects: int
    iter_total: np.ndarray             # [max_iter], entry i-1 = projects with >= i Fuzzing builds
    iter_detected: np.ndarray          # [max_iter], distinct projects detecting at iteration i
    min_project_threshold: int = 100
    late: Optional[Describe] = None


@dataclass
class RQ2CountResult:
    eligible: np.ndarray
    raw_n: np.ndarray                  # rows fetched per project (GET_TOTAL_COVERAGE_EACH_PROJECT)
    n_trend: np.ndarray                # values after the ``total != 0`` filter
    sw_w: np.ndarray                   # Shapiro-Wilk per project (NaN when n < 3)
    sw_p: np.ndarray
    corr: np.ndarray                   # Spearman vs index (NaN when undefined)
    session_offsets: np.ndarray        # CSR of coverage_by_session_index
    session_values: np.ndarray
    corr_mean: float
    corr_median: float
    ge100: np.ndarray                  # session indices with >= 100 values
    average_trend: np.ndarray          # statistics.mean per ge100 session
    median_trend: np.ndarray           # statistics.median per ge100 session
    spearman_median: Optional[Tuple[float, float]]
    shapiro_median_p: Optional[float]
    dist_percentiles: np.ndarray       # [5, n_ge100]: 5/25/50/75/95 (figure data)
    dist_mean: np.ndarray


@dataclass
class RQ2AddResult:
    projects: np.ndarray               # projects processed (ORDER BY project)
    row_project: np.ndarray            # one row per consecutive run pair
    row_first_build: np.ndarray        # first build of run i (modules_i / revisions_i)
    row_end_build: np.ndarray          # last build of run i
    row_start_build: np.ndarray        # first build of run i+1
    row_cov_i: np.ndarray              # coverage row matched on date_i (-1: none)
    row_cov_i1: np.ndarray             # coverage row matched on date_{i+1}
    diff_total: np.ndarray             # float64, NaN where invalid
    diff_coverage: np.ndarray
    covered_is_float: np.ndarray       # [P] pandas upcast of the project's covered_line column
    total_is_float: np.ndarray         # [P]


@dataclass
class RQ3Result:
    n_all_issues: int
    det_pct: np.ndarray
    det_cov: np.ndarray
    det_tot: np.ndarray
    det_project: np.ndarray
    det_issue: np.ndarray
    non_pct: np.ndarray
    non_cov: np.ndarray
    non_tot: np.ndarray
    desc_detected: Optional[Describe]
    desc_non: Optional[Describe]
    desc_det_total: Optional[Describe]
    anderson_det: Optional[Tuple[float, np.ndarray]]
    anderson_non: Optional[Tuple[float, np.ndarray]]
    levene: Optional[Tuple[float, float]]
    brunnermunzel: Optional[Tuple[float, float]]
    n_non_last: int = 0                # sharded runs: non-detected rows of the last project (tail)
    n_null_total: int = 0              # shards: pairs meeting a NULL total_line (rq3:253,297 raise)
    n_null_last: int = 0               # shards: those in the last project's flush (dropped with the tail)


@dataclass
class RQ4aResult:
    groups: Dict[str, List[int]]       # group1..group4 project ids (group1 includes CSV-missing)
    g1_total: np.ndarray               # [max_iter]
    g1_det: np.ndarray
    g2_total: np.ndarray
    g2_det: np.ndarray
    after: Dict[str, Optional[Tuple[float, float]]]   # 'g1'/'g2': (median, IQR) of rates after first < 5
    intro: List[Tuple[int, int]]       # (project, introduction iteration), CSV order
    intro_stats: Optional[Tuple[float, float, int, int]]   # mean, median, min, max of > 0
    g4_steps: Dict[int, Tuple[int, int]]   # step -> (n_total, detected)
    g4_transition: Tuple[int, int, int, int]   # pre&post, pre only, post only, neither
    g4_overall: Tuple[float, float]    # pooled pre / post rates
    n_g4_analyzed: int
    has_g4_transition: bool = True


@dataclass
class RQ4bResult:
    group_counts: Tuple[int, int, int, int]
    n_sessions: int
    c2: np.ndarray                     # per session counts
    c1: np.ndarray
    g2_q: np.ndarray                   # [n_sessions, 3] percentiles 25/50/75 (NaN when empty)
    g1_q: np.ndarray
    p_bm: np.ndarray                   # Brunner-Munzel p per session (NaN when not computed)
    last_valid_idx: int
    spearman6: Optional[List[Tuple[float, float]]]   # A Q1, A Med, A Q3, B Q1, B Med, B Q3
    n_delta_projects: int
    pre_cov: List[np.ndarray]          # [7] values per Pre-(i+1)
    post_cov: List[np.ndarray]         # [7] values per Post-(i+1)
    pre_median: List[float]
    post_median: List[float]
    n_g2: int
    n_g1: int
    init_g2: np.ndarray
    init_g1: np.ndarray
    mwu_p: Optional[float]
    cliff: Optional[float]
    bm: Optional[Tuple[float, float]]
    levene: Optional[Tuple[float, float]]
    extra: dict = field(default_factory=dict)
