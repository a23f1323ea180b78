"""Host-side glue shared by the GPU compute path, the oracle and the renderer.

These helpers hold the reference's control logic that is neither a kernel nor text:
the iteration-dictionary bookkeeping of RQ1, the corpus-CSV grouping of RQ4, the row
filter of ``calculate_and_save_stats``.  They operate on small host arrays (thousands of
entries) and are deliberately written the way the reference writes them.
"""
from __future__ import annotations

import io
from typing import Dict, List, Tuple

import numpy as np
import pandas as pd

from ..schema import Tables

DAYS_THRESHOLD = 7                 # rq4a_bug.py:44, rq4b_coverage.py:53
CORPUS_COLUMNS = ["project_name", "is_Corpus", "corpus_commit_time", "corpus_merged_time",  # user_corpus.py:225-233
                  "project_creation_time", "time_elapsed_seconds", "merged_time_elapsed_seconds"]


def rq1_rates(iter_total, iter_det, threshold):
    """rq1_detection_rate.py:233-258: drop iterations with total < threshold, then
    ``first_down_iteration`` = first *key* whose rate is < 5, used as a *list index*."""
    keys = [i for i in range(1, len(iter_total) + 1) if iter_total[i - 1] >= threshold]
    rates = [int(iter_det[k - 1]) / int(iter_total[k - 1]) * 100 for k in keys]
    first_down = -1
    for k, r in zip(keys, rates):
        if r < 5 and first_down == -1:
            first_down = k
    late = rates[first_down:]
    return keys, rates, first_down, late


def read_corpus(t: Tables) -> pd.DataFrame:
    """rq4a_bug.py:88-89 / rq4b_coverage.py:187-188.  No corpus file (empty text): no rows - the
    RQ4 scripts would stop there, every other analysis does not read it."""
    if not t.corpus_csv.strip():
        return pd.DataFrame({c: pd.Series([], dtype=object) for c in CORPUS_COLUMNS}).assign(
            time_elapsed_seconds=pd.Series([], dtype=float),
            corpus_commit_time=pd.Series([], dtype="datetime64[ns, UTC]"))
    df = pd.read_csv(io.StringIO(t.corpus_csv))
    df["corpus_commit_time"] = pd.to_datetime(df["corpus_commit_time"], errors="coerce", utc=True)
    return df


def _filtered(t: Tables, eligible) -> pd.DataFrame:
    df = read_corpus(t)
    names = {t.projects[p] for p in np.asarray(eligible).tolist()}
    return df[df["project_name"].isin(names)].copy()


def corpus_groups(t: Tables, eligible, add_missing_to_g1: bool):
    """rq4a_bug.py:94-121 (adds eligible projects missing from the CSV to G1) and
    rq4b_coverage.py:193-219 (does not).  Returns ({group: sorted ids}, {id: corpus UTC us})."""
    f = _filtered(t, eligible)
    pid = {n: i for i, n in enumerate(t.projects)}
    te = f["time_elapsed_seconds"]
    null = te.isna()
    cats = {
        "group1": null,
        "group2": (te == 0) & (~null),
        "group3": (te > 0) & (te < DAYS_THRESHOLD * 86400) & (~null),
        "group4": (te >= DAYS_THRESHOLD * 86400) & (~null),
    }
    groups = {g: set(f[m]["project_name"]) for g, m in cats.items()}
    if add_missing_to_g1:
        elig_names = {t.projects[p] for p in np.asarray(eligible).tolist()}
        groups["group1"].update(elig_names - set(f["project_name"]))
    out = {g: sorted(pid[n] for n in s) for g, s in groups.items()}
    corpus_us = {}
    for n, ts in zip(f[~null]["project_name"], f[~null]["corpus_commit_time"]):
        if not pd.isna(ts):
            corpus_us[pid[n]] = int(ts.value // 1000)
    return out, corpus_us


def corpus_columns(t: Tables):
    """Cached per table (see ``Tables.cached``): the columns of ``_corpus_columns``."""
    return t.cached("corpus_columns", (t.projects, t.corpus_csv), lambda: _corpus_columns(t))


def _corpus_columns(t: Tables):
    """Loader of project_corpus_analysis.csv for the GPU path (fz_rq4_groups in include/fz.h).

    Eligibility-independent per-project columns, so the device can apply the eligible set itself:
    member bit g = some CSV row puts the project in G(g+1) (rq4a_bug.py:94-108), bit 4 = project
    absent from the CSV (rq4a_bug.py:110-113); corpus_us = corpus_commit_time parsed with
    ``utc=True`` (last qualifying row wins, as the reference's dict does); order = projects of the
    CSV rows with a time_elapsed_seconds value, in file order (rq4b_coverage.py:216, :744).
    """
    from ..schema import TS_NULL
    df = read_corpus(t)
    pid = {n: i for i, n in enumerate(t.projects)}
    P = len(t.projects)
    member = np.zeros(P, dtype=np.uint8)
    corpus_us = np.full(P, TS_NULL, dtype=np.int64)
    te = df["time_elapsed_seconds"]
    null = te.isna()
    masks = [null, (te == 0) & (~null), (te > 0) & (te < DAYS_THRESHOLD * 86400) & (~null),
             (te >= DAYS_THRESHOLD * 86400) & (~null)]
    names = df["project_name"]
    for g, m in enumerate(masks):
        for n in names[m]:
            if n in pid:
                member[pid[n]] |= np.uint8(1 << g)
    seen = np.zeros(P, dtype=bool)
    for n in names:
        if n in pid:
            seen[pid[n]] = True
    member[~seen] |= np.uint8(16)
    for n, ts in zip(names[~null], df["corpus_commit_time"][~null]):
        if n in pid and not pd.isna(ts):
            corpus_us[pid[n]] = int(ts.value // 1000)
    order = np.array([pid[n] for n in names[~null] if n in pid], dtype=np.int32)
    return member, corpus_us, order


def corpus_order(t: Tables, eligible) -> List[int]:
    """Row order of ``group_2_3_4_df.iterrows()`` (rq4b_coverage.py:216, :744)."""
    f = _filtered(t, eligible)
    pid = {n: i for i, n in enumerate(t.projects)}
    return [pid[n] for n in f[~f["time_elapsed_seconds"].isna()]["project_name"]]


def rq4a_rows(g1t, g1d, g2t, g2d, threshold=100):
    """rq4a_bug.py:164-193: keep iterations where BOTH groups have >= threshold projects."""
    rows = []
    for i in range(1, len(g1t) + 1):
        a, b = int(g1t[i - 1]), int(g2t[i - 1])
        if a >= threshold and b >= threshold:
            da, db = int(g1d[i - 1]), int(g2d[i - 1])
            rows.append([i, a, da, da / a * 100 if a > 0 else 0, b, db, db / b * 100 if b > 0 else 0])
    return rows


def rq4b_compare(g2_stats, g1_stats):
    """rq4b_coverage.py:828-847: sessions where both quartile triples are non-NaN."""
    wins = [0, 0, 0]
    seq2 = ([], [], [])
    seq1 = ([], [], [])
    n = 0
    for s2, s1 in zip(g2_stats, g1_stats):
        if len(s2) == 3 and len(s1) == 3:
            if np.isnan(s2).any() or np.isnan(s1).any():
                continue
            n += 1
            for j in range(3):
                if s2[j] > s1[j]:
                    wins[j] += 1
                seq2[j].append(float(s2[j]))
                seq1[j].append(float(s1[j]))
    return n, wins, seq2, seq1


def rq4b_spearman6(g2_stats, g1_stats, spearman) -> List[Tuple[float, float]]:
    """rq4b_coverage.py:879-899: Spearman(1..N, quartile sequence), A then B, Q1/Med/Q3."""
    n, _, seq2, seq1 = rq4b_compare(g2_stats, g1_stats)
    if n == 0:
        return None
    it = np.arange(1, n + 1)
    out = []
    for seq in (seq1[0], seq1[1], seq1[2], seq2[0], seq2[1], seq2[2]):
        c, p = spearman(it, seq)
        out.append((float(c), float(p)))
    return out
