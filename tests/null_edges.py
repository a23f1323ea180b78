"""NULL line-count edge tables: the 'tiny' golden table with one total_coverage row changed so that
a NULL covered_line / total_line reaches the reference's arithmetic.

    rq3_diff_coverage_at_detection.py:263   fetches rows with covered_line IS NOT NULL only, then
                                             tests `prev_cov[2] > 0 and curr_cov[2] > 0` (:253 in
                                             the non-detected flush, :297 for a detection pair):
                                             None > 0 raises TypeError
    rq2_coverage_count.py:300-303           `float(x[0]) / float(x[1])` for rows with x[1] != 0:
                                             a NULL total (None != 0) or a NULL covered_line raises
                                             TypeError, a zero total skips the row

Edges (the reference's behaviour on each is recorded by tests/golden/make_goldens.py; both its
return code and stdout/stderr are fixtures under tests/golden/tiny+<edge>/):

    null_total_mid       total NULL on a row of the FIRST issue-bearing project (flushed):
                         rq3 raises, rq2_coverage_count raises
    null_total_last      total NULL on a row of the LAST issue-bearing project (never flushed,
                         rq3:245-257), away from its issue days: rq3 runs; rq2_coverage_count raises
    covered_null         covered NULL, total kept: rq2_coverage_count raises; rq3 skips the row
    covered_null_zero    covered NULL and total 0: both run (the row is skipped by x[1] != 0)
"""
from __future__ import annotations

import dataclasses

import numpy as np

from tse_amd.schema import US_PER_DAY

EDGES = ["null_total_mid", "null_total_last", "covered_null", "covered_null_zero"]
SCRIPTS = ["rq2_coverage_count", "rq3_diff_coverage_at_detection"]
RQ3_LIMIT_US = 1736380800000000   # '2025-01-09' (rq3:262-263)
LIMIT_US = 1736294400000000       # '2025-01-08'


def _issue_projects(t):
    """Projects of rq3's issue loop in ORDER BY project order (fixed, eligible, rts < LIMIT)."""
    from oracle import rq_oracle as orc
    elig = np.zeros(len(t.projects), bool)
    elig[orc.eligible_projects(t)] = True
    m = np.isin(t.i_status, (0, 1)) & elig[t.i_project] & (t.i_rts < LIMIT_US)
    return sorted(set(t.i_project[m].tolist())), m


def _pick_row(t, p, issue_mask):
    """A coverage row k of project p (rq3's fetch order) with k and k + 1 away from every issue
    day and the day after it, so no detection pair or excluded day involves k or its successor."""
    rows = np.nonzero((t.c_project == p) & t.c_covered_valid & (t.c_date < RQ3_LIMIT_US)
                      & t.c_coverage_valid & (t.c_coverage > 0) & (t.c_date < LIMIT_US))[0]
    rows = rows[np.argsort(t.c_date[rows], kind="stable")]
    days = set()
    for r in t.i_rts[issue_mask & (t.i_project == p)].tolist():
        d = r // US_PER_DAY
        days.update((d - 1, d, d + 1, d + 2))
    for k in range(len(rows) // 2, len(rows) - 1):
        if t.c_date[rows[k]] // US_PER_DAY not in days and t.c_date[rows[k + 1]] // US_PER_DAY not in days:
            return int(rows[k])
    raise AssertionError(f"no quiet coverage row in project {p}")


def apply(t, edge: str):
    """A copy of table t with the edge's one-row change."""
    projs, im = _issue_projects(t)
    covered_valid = t.c_covered_valid.copy()
    total_valid = t.c_total_valid.copy()
    covered = t.c_covered.copy()
    total = t.c_total.copy()
    if edge == "null_total_mid":
        r = _pick_row(t, projs[0], im)
        total_valid[r], total[r] = False, 0
    elif edge == "null_total_last":
        r = _pick_row(t, projs[-1], im)
        total_valid[r], total[r] = False, 0
    elif edge == "covered_null":
        r = _pick_row(t, projs[0], im)
        covered_valid[r], covered[r] = False, 0
    elif edge == "covered_null_zero":
        r = _pick_row(t, projs[0], im)
        covered_valid[r], covered[r], total[r] = False, 0, 0
    else:
        raise KeyError(edge)
    return dataclasses.replace(t, c_covered=covered, c_covered_valid=covered_valid, c_total=total,
                               c_total_valid=total_valid)


def fingerprint(t) -> str:
    """synth.table_fingerprint plus the per-column validity bits it does not cover."""
    import hashlib

    import tse_amd.synth as synth
    h = hashlib.sha256(synth.table_fingerprint(t).encode())
    for a in (t.c_covered_valid, t.c_total_valid):
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def split(case: str):
    """'tiny+null_total_mid' -> ('tiny', 'null_total_mid'); plain cases -> (case, None)."""
    base, _, edge = case.partition("+")
    return base, (edge or None)
