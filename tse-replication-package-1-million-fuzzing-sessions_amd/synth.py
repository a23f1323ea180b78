"""Synthetic session tables with the shipped schema.

The reference ships no input tables (``.gitignore:6-8`` of the reference), so every
benchmark and parity case runs on tables generated here.  The generator is deterministic
for a given (config, seed) - numpy's PCG64 stream is stable across platforms - and is
vectorised per project so the ~1M-session "config 2" table builds in a few seconds.

Properties the generator guarantees (so PostgreSQL tie order can never matter, 8(d)):
unique timestamps per (project, build_type), unique issue numbers unless
``dup_numbers`` asks for duplicates, non-NULL build/issue timestamps, coverage NULL
exactly when covered/total are NULL.
"""
from __future__ import annotations

import datetime as _dt
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .schema import (BT_COVERAGE, BT_FUZZING, CODE_NULL, US_PER_DAY, Tables, dt_to_us)

BASE_US = dt_to_us(_dt.datetime(2016, 12, 1))
END_US = dt_to_us(_dt.datetime(2025, 3, 1))
HOUR_US = 3_600_000_000


@dataclass
class SynthConfig:
    n_projects: int = 1000
    seed: int = 7
    start_span_days: int = 2400          # project start uniform over BASE + [0, span]
    len_mean_days: float = 1400.0        # project length ~ Exp(mean) ...
    len_min_days: int = 30               # ... clipped to [min, days to END]
    len_uniform: Optional[tuple] = None  # or U[lo, hi] days (golden cases)
    p_cov_valid: float = 0.9             # coverage row valid, else a NULL row
    p_rev_change: float = 0.15           # revisions change per day
    p_mod_change: float = 0.003          # modules change per day
    issues_mean: float = 65.0            # issues/project ~ Exp(mean)
    issue_days_mean: float = 300.0       # issue day after start ~ Exp(mean)
    p_zero_total: float = 0.001          # rare covered=total=0 rows (RQ2 ``total != 0`` filter)
    hex_len: int = 40                    # revision hash width
    dup_numbers: int = 0                 # number of issues that reuse another issue's number
    p_project_info_missing: float = 0.02
    p_corpus_missing: float = 0.05       # projects absent from the corpus CSV
    group_weights: tuple = (0.42, 0.42, 0.08, 0.08)   # G1 none, G2 same time, G3 <7d, G4 >=7d
    zipf_s: Optional[float] = None       # config 5: Zipf rows/project
    coverage_only: bool = False          # config 3: only total_coverage rows
    rows_per_project: Optional[int] = None  # config 3: fixed contiguous daily length
    lengths: Optional[tuple] = None      # config 4: per-project series lengths (cycled)
    step_us: int = US_PER_DAY            # spacing of consecutive coverage rows
    tie_levels: Optional[int] = None     # config 4: covered/total on a grid of tie_levels + 1 values
    trend_mix: bool = False              # config 4: odd projects follow a monotone trend + noise


RESULT_P = np.array([0.80, 0.05, 0.05, 0.10])      # Finish, Halfway, HalfWay, Error
STATUS_NAMES = ["Fixed", "Fixed (Verified)", "New", "WontFix"]
STATUS_P = np.array([0.70, 0.08, 0.12, 0.10])


def _hex(rng, n, width):
    digits = np.frombuffer(b"0123456789abcdef", dtype=np.uint8)
    raw = digits[rng.integers(0, 16, size=(n, width))]
    return [bytes(row).decode() for row in raw]


def project_names(n):
    # fixed-width [a-z0-9] names: byte order == any sane collation's order
    return [f"proj{i:05d}" for i in range(n)]


def generate(cfg: SynthConfig) -> Tables:
    rng = np.random.default_rng(cfg.seed)
    P = cfg.n_projects
    names = project_names(P)
    start_day = rng.integers(0, cfg.start_span_days + 1, size=P)
    max_len = (END_US - BASE_US) // US_PER_DAY - start_day
    if cfg.lengths is not None:
        length = np.resize(np.asarray(cfg.lengths, dtype=np.int64), P)
        start_day = np.zeros(P, dtype=np.int64)
    elif cfg.rows_per_project is not None:
        length = np.full(P, cfg.rows_per_project, dtype=np.int64)
        start_day = np.zeros(P, dtype=np.int64)
    elif cfg.zipf_s is not None:
        w = 1.0 / np.arange(1, P + 1) ** cfg.zipf_s
        rng.shuffle(w)
        length = np.maximum(1, (w / w.sum() * cfg.len_mean_days * P)).astype(np.int64)
        start_day = np.zeros(P, dtype=np.int64)
    elif cfg.len_uniform is not None:
        length = rng.integers(cfg.len_uniform[0], cfg.len_uniform[1] + 1, size=P)
        length = np.minimum(length, max_len)
    else:
        length = np.round(rng.exponential(cfg.len_mean_days, size=P)).astype(np.int64)
        length = np.clip(length, cfg.len_min_days, np.maximum(cfg.len_min_days, max_len))

    # ---- total_coverage: one row per project-day (NULL row on "missing" days) ----
    c_proj, c_date, c_cov, c_cov_ok, c_cvd, c_tot = [], [], [], [], [], []
    for p in range(P):
        L = int(length[p])
        d0 = BASE_US + int(start_day[p]) * US_PER_DAY
        dates = d0 + np.arange(L, dtype=np.int64) * cfg.step_us
        if cfg.tie_levels:  # heavy ties: constant total, covered on a coarse grid
            total = np.full(L, cfg.tie_levels, dtype=np.int64)
        else:
            total = np.maximum(1, np.round(rng.uniform(500, 2e5) + np.cumsum(
                rng.normal(0, 60, size=L)))).astype(np.int64)
        if cfg.trend_mix and p % 2 == 1:  # monotone trend + noise
            frac = np.clip(np.linspace(0.1, 0.9, L) + rng.normal(0, 0.05, size=L), 0.0, 1.0)
        else:
            frac = np.clip(rng.uniform(0.1, 0.6) + np.cumsum(rng.normal(0, 0.002, size=L)), 0.0, 1.0)
        covered = np.clip(np.round(total * frac), 0, total).astype(np.int64)
        zero = rng.random(L) < cfg.p_zero_total
        total[zero] = 0
        covered[zero] = 0
        valid = rng.random(L) < cfg.p_cov_valid
        cov = np.zeros(L)
        nz = total > 0
        cov[nz] = covered[nz] / total[nz] * 100.0
        c_proj.append(np.full(L, p, dtype=np.uint32))
        c_date.append(dates)
        c_cov.append(np.where(valid, cov, 0.0))
        c_cov_ok.append(valid)
        c_cvd.append(np.where(valid, covered, 0))
        c_tot.append(np.where(valid, total, 0))
    c_project = np.concatenate(c_proj)
    c_cov_ok = np.concatenate(c_cov_ok)

    # ---- buildlog_data: one Fuzzing + one Coverage build per project-day ----
    b_proj, b_type, b_res, b_time, b_mod, b_rev, b_name = [], [], [], [], [], [], []
    modules_pool, revisions_pool = [], []
    if not cfg.coverage_only:
        for p in range(P):
            L = int(length[p])
            d0 = BASE_US + int(start_day[p]) * US_PER_DAY
            days = d0 + np.arange(L, dtype=np.int64) * US_PER_DAY
            # revision state per day: two hashes, first changes w.p. p_rev_change, second rarely
            ch1 = rng.random(L) < cfg.p_rev_change
            ch2 = rng.random(L) < cfg.p_rev_change / 8
            ch1[0] = ch2[0] = True
            h1 = _hex(rng, int(ch1.sum()), cfg.hex_len)
            h2 = _hex(rng, int(ch2.sum()), cfg.hex_len)
            i1 = np.cumsum(ch1) - 1
            i2 = np.cumsum(ch2) - 1
            key = i1 * (len(h2) + 1) + i2
            ukey, rev_local = np.unique(key, return_inverse=True)
            base = len(revisions_pool)
            for k in ukey.tolist():
                revisions_pool.append("{" + h1[k // (len(h2) + 1)] + "," + h2[k % (len(h2) + 1)] + "}")
            rev_day = base + rev_local.reshape(-1)
            mch = rng.random(L) < cfg.p_mod_change
            mch[0] = True
            mver = np.cumsum(mch) - 1
            mbase = len(modules_pool)
            for v in range(int(mver[-1]) + 1):
                extra = ",".join(f"dep{j}" for j in range(v % 4))
                modules_pool.append("{" + names[p] + ",afl" + ("," + extra if extra else "") + "}")
            mod_day = mbase + mver
            for bt, tag in ((BT_FUZZING, "fuzz"), (BT_COVERAGE, "cov")):
                t = days + rng.integers(HOUR_US, 22 * HOUR_US, size=L) + rng.integers(0, 1_000_000, size=L)
                b_proj.append(np.full(L, p, dtype=np.uint32))
                b_type.append(np.full(L, bt, dtype=np.uint8))
                b_res.append(rng.choice(4, size=L, p=RESULT_P).astype(np.uint8))
                b_time.append(t)
                b_mod.append(mod_day.astype(np.int32))
                b_rev.append(rev_day.astype(np.int32))
                b_name.append([f"{names[p]}/{tag}/{k:05d}.log" for k in range(L)])
    if b_proj:
        b_project = np.concatenate(b_proj)
        b_types = np.concatenate(b_type)
        b_result = np.concatenate(b_res)
        b_times = np.concatenate(b_time)
        b_modules = np.concatenate(b_mod)
        b_revisions = np.concatenate(b_rev)
        names_arr = np.empty(len(b_project), dtype=object)
        names_arr[:] = [s for chunk in b_name for s in chunk]
    else:
        b_project = np.zeros(0, np.uint32)
        b_types = b_result = np.zeros(0, np.uint8)
        b_times = np.zeros(0, np.int64)
        b_modules = b_revisions = np.zeros(0, np.int32)
        names_arr = np.empty(0, dtype=object)

    # ---- issues ----
    if cfg.coverage_only:
        n_iss = np.zeros(P, dtype=np.int64)
    else:
        n_iss = np.round(rng.exponential(cfg.issues_mean, size=P)).astype(np.int64)
    i_proj = np.repeat(np.arange(P, dtype=np.uint32), n_iss)
    start_us = BASE_US + start_day.astype(np.int64) * US_PER_DAY
    off = rng.exponential(cfg.issue_days_mean, size=len(i_proj)) * US_PER_DAY
    i_rts = start_us[i_proj] + off.astype(np.int64)
    i_status = rng.choice(len(STATUS_NAMES), size=len(i_proj), p=STATUS_P).astype(np.uint8)
    i_number = rng.choice(np.arange(1_000_000, 1_000_000 + 40 * max(1, len(i_proj))),
                          size=len(i_proj), replace=False).astype(np.int64)
    if cfg.dup_numbers and len(i_number) > 2 * cfg.dup_numbers:
        src = rng.choice(len(i_number), size=cfg.dup_numbers, replace=False)
        dst = rng.choice(np.setdiff1d(np.arange(len(i_number)), src), size=cfg.dup_numbers, replace=False)
        i_number[dst] = i_number[src]
    i_new_id = rng.integers(400_000_000, 500_000_000, size=len(i_proj)).astype(np.int64)
    # row order of a heap table is arbitrary: shuffle issues
    perm = rng.permutation(len(i_proj))
    i_proj, i_rts, i_status, i_number, i_new_id = (a[perm] for a in (i_proj, i_rts, i_status, i_number, i_new_id))

    # ---- project_info ----
    keep = rng.random(P) >= cfg.p_project_info_missing
    pi_project = np.nonzero(keep)[0].astype(np.uint32)
    pi_first = start_us[keep] - rng.integers(0, 400, size=int(keep.sum())) * US_PER_DAY

    # ---- corpus CSV (user_corpus.py:225-233 columns) ----
    creation = start_us - rng.integers(0, 30, size=P) * US_PER_DAY - rng.integers(0, 86_400, size=P) * 1_000_000
    grp = rng.choice(4, size=P, p=np.array(cfg.group_weights) / sum(cfg.group_weights))
    present = rng.random(P) >= cfg.p_corpus_missing
    lines = ["project_name,is_Corpus,corpus_commit_time,corpus_merged_time,project_creation_time,"
             "time_elapsed_seconds,merged_time_elapsed_seconds"]
    tz_choices = [0, 0, 9, -7, 2]
    for p in np.nonzero(present)[0].tolist():
        tz = tz_choices[p % len(tz_choices)]
        tzs = f"{'+' if tz >= 0 else '-'}{abs(tz):02d}:00"
        cre = _dt.datetime(1970, 1, 1) + _dt.timedelta(microseconds=int(creation[p])) + _dt.timedelta(hours=tz)
        cre_s = cre.replace(microsecond=0).isoformat() + tzs
        g = int(grp[p])
        if g == 0:
            lines.append(f"{names[p]},False,,,{cre_s},,")
            continue
        if g == 1:
            el = 0
        elif g == 2:
            el = int(rng.integers(1, 7 * 86400))
        else:
            el = int(rng.integers(7 * 86400, max(7 * 86400 + 1, int(length[p]) * 86400)))
        cc = cre.replace(microsecond=0) + _dt.timedelta(seconds=el)
        lines.append(f"{names[p]},True,{cc.isoformat()}{tzs},,{cre_s},{float(el)},")
    corpus_csv = "\n".join(lines) + "\n"

    def cat(parts, dt):
        return np.concatenate(parts).astype(dt) if parts else np.zeros(0, dt)

    # heap order: shuffle coverage and build rows too (the engine must sort)
    cperm = rng.permutation(len(c_project))
    bperm = rng.permutation(len(b_project))
    return Tables(
        projects=names,
        b_project=b_project[bperm], b_type=b_types[bperm], b_result=b_result[bperm],
        b_time=b_times[bperm], b_modules=b_modules[bperm], b_revisions=b_revisions[bperm],
        b_name=names_arr[bperm], modules_pool=modules_pool, revisions_pool=revisions_pool,
        c_project=c_project[cperm], c_date=cat(c_date, np.int64)[cperm],
        c_coverage=cat(c_cov, np.float64)[cperm], c_coverage_valid=c_cov_ok[cperm],
        c_covered=cat(c_cvd, np.int64)[cperm], c_covered_valid=c_cov_ok[cperm],
        c_total=cat(c_tot, np.int64)[cperm], c_total_valid=c_cov_ok[cperm],
        i_number=i_number, i_project=i_proj, i_rts=i_rts, i_status=i_status, i_new_id=i_new_id,
        pi_project=pi_project, pi_first_commit=pi_first.astype(np.int64),
        statuses=list(STATUS_NAMES), corpus_csv=corpus_csv,
    )


CONFIGS = {
    # golden-fixture cases (small enough for the sqlite harness)
    "tiny": SynthConfig(n_projects=40, seed=3, len_mean_days=500, dup_numbers=3, hex_len=12),
    "medium": SynthConfig(n_projects=300, seed=5, len_uniform=(380, 900), issues_mean=30,
                          dup_numbers=4, hex_len=12),
    # ~1M sessions, the bench workload
    "c2": SynthConfig(n_projects=1000, seed=7),
    # config 3: 100M coverage rows / 10k projects (rows_per_project scales it down for tests)
    "c3": SynthConfig(n_projects=10_000, seed=11, coverage_only=True, rows_per_project=10_000),
    # config 5: Zipf rows per project
    "c5": SynthConfig(n_projects=10_000, seed=13, coverage_only=True, zipf_s=1.2, len_mean_days=10_000),
    # live-row variants of configs 3 and 5: the same 100M rows, projects, seeds and Zipf giant, but
    # rows spaced below a day so EVERY row precedes the analysis limit (queries1.py:3 '2025-01-08' =
    # day 2,960 of the series) and reaches the analyses - config 3 daily puts 70 % and config 5 88 %
    # of the rows past the limit, where only the store sorts them.  c3L: 10,000 rows six hours apart
    # (2,500 days); c5L: ten seconds apart (the 20.8M-row giant spans 2,408 days)
    "c3L": SynthConfig(n_projects=10_000, seed=11, coverage_only=True, rows_per_project=10_000,
                       step_us=6 * HOUR_US),
    "c5L": SynthConfig(n_projects=10_000, seed=13, coverage_only=True, zipf_s=1.2, len_mean_days=10_000,
                       step_us=10_000_000),
    # config 4 (rank-statistics stress): series of 1e5 / 3e5 / 1e6 points (one row a minute, all
    # before the analysis limit), 256 coverage levels (heavy ties), every other one a trend + noise
    "c4": SynthConfig(n_projects=12, seed=17, coverage_only=True, lengths=(100_000, 300_000, 1_000_000),
                      step_us=60_000_000, tie_levels=255, trend_mix=True),
}


def config(name: str, **overrides) -> SynthConfig:
    base = CONFIGS[name]
    return SynthConfig(**{**base.__dict__, **overrides})


def table_fingerprint(t: Tables) -> str:
    """sha256 over every column: ties a golden fixture to the exact generated input."""
    import hashlib
    h = hashlib.sha256()
    for a in (t.b_project, t.b_type, t.b_result, t.b_time, t.b_modules, t.b_revisions,
              t.c_project, t.c_date, t.c_coverage, t.c_coverage_valid, t.c_covered, t.c_total,
              t.i_number, t.i_project, t.i_rts, t.i_status, t.i_new_id, t.pi_project, t.pi_first_commit):
        h.update(np.ascontiguousarray(a).tobytes())
    for pool in (t.modules_pool, t.revisions_pool, t.projects):
        h.update("\x00".join("" if s is None else s for s in pool).encode())
    h.update("\x00".join(t.b_name.tolist()).encode())
    h.update(t.corpus_csv.encode())
    return h.hexdigest()
