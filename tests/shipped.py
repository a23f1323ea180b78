"""Reference-held known-answer vectors (tests/golden/shipped/, built by make_shipped.py from the
reference's shipped real-data outputs under data/result_data/).

* ``rq1_tables()``      rq1_detection_rate_stats.csv -> (iter_total, iter_detected): the kept
                        iterations 1..2341 of the real dataset (rq1_detection_rate.py:330-336).
* ``rq4a_tables()``     rq4_g1_g2_detection_trend.csv -> G1 / G2 totals and detected counts of
                        iterations 1..1600 (rq4a_bug.py:193-204) + the CSV bytes.
* ``intro_rows()``      rq4_gc_introduction_iteration.csv -> [(project, iteration)] (rq4a:272-290).
* ``detected_changes()`` detected_coverage_changes.csv -> (pct, covered delta, total delta)
                        (rq3_diff_coverage_at_detection.py:307-312).
* ``change_analysis_tables()`` session tables whose rq2_coverage_and_added.py:73-238 output is
                        data/result_data/rq3/change_analysis/<project>.csv (revisions text mapped
                        to ids, see make_shipped.py), and ``change_analysis_expected()`` the
                        per-file sha256 of those bytes.

The known answers the reference itself prints for the real data are quoted where a test uses them
(rq1_detection_rate.py:401-407; SURVEY.md 4 for the RQ4 / RQ3 figures).
"""
from __future__ import annotations

import csv
import json
import os
from functools import lru_cache

import numpy as np

from tse_amd.schema import BT_COVERAGE, CODE_NULL, R_FINISH, US_PER_DAY, Tables, ts_from_str

DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "shipped")


def _rows(name):
    with open(os.path.join(DIR, name), newline="") as f:
        r = list(csv.reader(f))
    return r[0], r[1:]


def raw_bytes(name):
    with open(os.path.join(DIR, name), "rb") as f:
        return f.read()


@lru_cache(maxsize=1)
def rq1_tables():
    _, rows = _rows("rq1_detection_rate_stats.csv")
    it = np.array([int(r[0]) for r in rows])
    assert np.array_equal(it, np.arange(1, len(rows) + 1))  # a prefix of the iteration axis
    return (np.array([int(r[1]) for r in rows], np.int64), np.array([int(r[2]) for r in rows], np.int64))


@lru_cache(maxsize=1)
def rq4a_tables():
    _, rows = _rows("rq4_g1_g2_detection_trend.csv")
    it = np.array([int(r[0]) for r in rows])
    assert np.array_equal(it, np.arange(1, len(rows) + 1))
    cols = [np.array([int(r[k]) for r in rows], np.int64) for k in (1, 2, 4, 5)]
    return tuple(cols)


def intro_rows():
    _, rows = _rows("rq4_gc_introduction_iteration.csv")
    return [(r[0], int(r[1])) for r in rows]


def detected_changes():
    _, rows = _rows("detected_coverage_changes.csv")
    return (np.array([float(r[0]) for r in rows]), np.array([int(r[1]) for r in rows], np.int64),
            np.array([int(r[2]) for r in rows], np.int64))


@lru_cache(maxsize=1)
def _ca_meta():
    with open(os.path.join(DIR, "change_analysis.json")) as f:
        return json.load(f)


def change_analysis_expected():
    return _ca_meta()["files"]


FILLER_DAY0 = ts_from_str("2000-01-01")  # before every build of the fixture (make_shipped asserts it)


@lru_cache(maxsize=1)
def change_analysis_tables() -> Tables:
    """The inverted session tables (see make_shipped.py).  Per project the loader adds 365 filler
    coverage rows (coverage 50.0) on the days from 2000-01-01, so every project passes the
    >= 365-row eligibility query (rq2_coverage_and_added.py:20-27) without touching a joined date,
    and one all-NULL coverage row on 1999-12-31, the NULL that makes pandas print every shipped
    file's covered/total columns as floats (e.g. 2471.0).  Rows are shuffled (heap order)."""
    meta = _ca_meta()
    z = np.load(os.path.join(DIR, "change_analysis.npz"), allow_pickle=False)
    P = len(meta["projects"])
    nb = len(z["b_time"])
    # coverage rows: the joined dates + fillers + one NULL row per project
    fill_day = FILLER_DAY0 + np.arange(365, dtype=np.int64) * US_PER_DAY
    pr = np.arange(P, dtype=np.uint32)
    c_project = np.concatenate([z["c_project"], np.repeat(pr, 365), pr])
    c_date = np.concatenate([z["c_date"], np.tile(fill_day, P), np.full(P, FILLER_DAY0 - US_PER_DAY, np.int64)])
    c_covered = np.concatenate([z["c_covered"], np.ones(365 * P, np.int64), np.zeros(P, np.int64)])
    c_total = np.concatenate([z["c_total"], np.full(365 * P, 2, np.int64), np.zeros(P, np.int64)])
    cvd_ok = np.concatenate([z["c_covered_valid"], np.ones(365 * P, bool), np.zeros(P, bool)])
    tot_ok = np.concatenate([z["c_total_valid"], np.ones(365 * P, bool), np.zeros(P, bool)])
    n0 = len(z["c_date"])
    cov = np.zeros(len(c_date))
    cov_ok = np.zeros(len(c_date), bool)
    m = cvd_ok & tot_ok & (c_total > 0)
    cov[m] = c_covered[m] / c_total[m] * 100.0
    cov_ok[m] = True
    cov[n0:n0 + 365 * P] = 50.0
    rng = np.random.default_rng(2025)
    cp = rng.permutation(len(c_date))
    bp = rng.permutation(nb)
    names = np.empty(nb, dtype=object)
    names[:] = [None] * nb
    return Tables(
        projects=list(meta["projects"]),
        b_project=z["b_project"][bp], b_type=np.full(nb, BT_COVERAGE, np.uint8),
        b_result=np.full(nb, R_FINISH, np.uint8), b_time=z["b_time"][bp], b_modules=z["b_modules"][bp],
        b_revisions=z["b_revisions"][bp], b_name=names, modules_pool=list(meta["modules_pool"]),
        revisions_pool=["{r%d}" % k for k in range(meta["n_revisions"])],
        c_project=c_project[cp], c_date=c_date[cp], c_coverage=cov[cp], c_coverage_valid=cov_ok[cp],
        c_covered=c_covered[cp], c_covered_valid=cvd_ok[cp], c_total=c_total[cp], c_total_valid=tot_ok[cp],
        i_number=np.zeros(0, np.int64), i_project=np.zeros(0, np.uint32), i_rts=np.zeros(0, np.int64),
        i_status=np.zeros(0, np.uint8), i_new_id=np.zeros(0, np.int64),
        pi_project=np.zeros(0, np.uint32), pi_first_commit=np.zeros(0, np.int64))


def check_change_files(files: dict):
    """Rendered rq2_add files -> list of mismatches against the shipped change_analysis bytes."""
    import hashlib
    exp = change_analysis_expected()
    got = {os.path.basename(k)[:-4]: v for k, v in files.items() if "/change_analysis/" in k}
    errs = []
    if set(got) != set(exp):
        errs.append(f"projects: {len(got)} files vs {len(exp)} shipped; "
                    f"missing {sorted(set(exp) - set(got))[:5]}, extra {sorted(set(got) - set(exp))[:5]}")
    for name, e in exp.items():
        if name in got and hashlib.sha256(got[name]).hexdigest() != e["sha256"]:
            n = got[name].count(b"\n") - 1
            errs.append(f"{name}: bytes differ ({n} rows vs {e['rows']} shipped)")
        if len(errs) > 10:
            break
    return errs


# rq1_detection_rate.py:401-407 - what the reference printed on the real data (the stale run log at
# the end of the script; its per-iteration lines predate the shipped CSV, this block reproduces)
RQ1_LATE_BLOCK = [
    "Analysis of detection rates from iteration 26 onwards (for paper replication):",
    "  - Min/Max: 0.00% / 5.47%",
    "value min and than 0 0.30303030303030304",
    "  - IQR (25th-75th percentile): 1.68% - 2.77%",
    "  - Median: 2.20%",
    "  - Mean: 2.24%",
    "  - Zero count: 1.04%(24/2314)",
]

# rq4a_bug.py:698-747 on the shipped trend table (G2 > G1 in 1405/1600; G1 first < 5 %
# at iteration 13 (4.11 %), G2 at 33 (2.78 %); G1 median 1.29 IQR 0.93; G2 median 3.15 IQR 2.15).
# trend_df.iloc[k]['Iteration'] is read from a mixed int/float row, which pandas upcasts to float64:
# the reference prints "13.0th" (as in the golden stdout of tests/golden/*/rq4a_bug).
RQ4A_MAIN_LINES = [
    "Count of Group B exceeding Group A within valid data range: 1405/1600 (87.81%)",
    "Group A: 13.0th iteration fell below 5% (value: 4.11%)",
    "Group B: 33.0th iteration fell below 5% (value: 2.78%)",
    "Group A: median 1.29, IQR 0.93",
    "Group A: Last valid data count 1600.0th",
    "Group B: median 3.15, IQR 2.15",
    "Group B: Last valid data count 1600.0th",
]
# rq4a_bug.py:277-285 on rq4_gc_introduction_iteration.csv (56 rows > 0)
RQ4A_INTRO_LINES = ["[RESULT] Introduction Iteration (N=56):", "  - Mean: 475.04", "  - Median: 274.0"]
