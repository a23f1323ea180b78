"""Project-sharded multi-GPU layer (tse_amd/parallel.py) on CPU: world_size 2, 3 and 8 over gloo.

Each rank runs the exchange drivers over ORACLE shards (the CPU restatement of one rank's local
analysis); rank 0 checks the recombined result against the oracle on the whole table.  The
tables are built so that the exchange steps matter: issue numbers collide across shards (the
ROW_NUMBER dedup spans projects), a "twin" project in the last shard duplicates the first
eligible project (equal build times -> tie broken by project order, i.e. by rank), and one case
leaves the last shard without issues (the never-flushed RQ3 project then sits on another rank).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from tse_amd import parallel as par
from tse_amd import synth
from tse_amd.rq import common
from tse_amd.schema import LIMIT_US, Tables


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def make_table(case: str, world: int) -> Tables:
    from oracle import rq_oracle as orc
    t = synth.generate(synth.config("tiny"))
    P = len(t.projects)
    elig = orc.eligible_projects(t)
    src, dst = int(elig[0]), P - 1
    # twin: project dst := a copy of project src (builds, coverage, issues with the same numbers)
    def twin(proj, cols):
        keep = proj != dst
        take = np.nonzero(proj == src)[0]
        out = [np.concatenate([c[keep], c[take]]) for c in cols]
        return out, int(keep.sum())
    (bp, bt, br, bti, bm, brv, bn), nb = twin(t.b_project, (t.b_project, t.b_type, t.b_result, t.b_time, t.b_modules,
                                                             t.b_revisions, t.b_name))
    bp[nb:] = dst
    (cp, cd, cc, ccv, cv, cvv, ct, ctv), nc = twin(t.c_project, (t.c_project, t.c_date, t.c_coverage,
                                                                 t.c_coverage_valid, t.c_covered, t.c_covered_valid,
                                                                 t.c_total, t.c_total_valid))
    cp[nc:] = dst
    (ip, inum, irts, ist, inew), ni = twin(t.i_project, (t.i_project, t.i_number, t.i_rts, t.i_status, t.i_new_id))
    ip[ni:] = dst
    inum = inum.copy()
    inum[:ni] = 1_000_000 + (inum[:ni] % 97)          # collisions across projects (and shards)
    inum[ni:] = inum[np.nonzero(ip[:ni] == src)[0]]   # the twin's issues reuse the source's numbers
    t = Tables(projects=t.projects, b_project=bp, b_type=bt, b_result=br, b_time=bti, b_modules=bm, b_revisions=brv,
               b_name=bn, modules_pool=t.modules_pool, revisions_pool=t.revisions_pool, c_project=cp, c_date=cd,
               c_coverage=cc, c_coverage_valid=ccv, c_covered=cv, c_covered_valid=cvv, c_total=ct, c_total_valid=ctv,
               i_number=inum, i_project=ip, i_rts=irts, i_status=ist, i_new_id=inew, pi_project=t.pi_project,
               pi_first_commit=t.pi_first_commit, build_types=t.build_types, results=t.results,
               statuses=t.statuses, corpus_csv=t.corpus_csv)
    if case == "giant":
        t = add_giant(t)
    if case == "live_giant":
        t = add_live_giant(t)
    if case == "last_shard_no_issues":
        lo, _ = par.shard_bounds(t, world)[-1]
        keep = t.i_project.astype(np.int64) < lo
        import dataclasses
        t = dataclasses.replace(t, i_number=t.i_number[keep], i_project=t.i_project[keep], i_rts=t.i_rts[keep],
                                i_status=t.i_status[keep], i_new_id=t.i_new_id[keep])
    return t


def add_giant(t: Tables, extra: int = 90000) -> Tables:
    """The tiny table with one eligible project grown into a Zipf-like giant: `extra` more daily
    coverage rows after its last one (past the analyses' date bounds; NULL and non-positive rows
    among them), and its corpus commit moved into those rows (group 4: the delta window of
    rq4b_coverage.py:745-772 then lies among the rows split_plan would move).  Issue numbers and
    builds unchanged."""
    import dataclasses
    import datetime as dt
    from oracle import rq_oracle as orc
    from tse_amd.schema import US_PER_DAY
    elig = orc.eligible_projects(t)
    g = int(elig[0])
    rng = np.random.default_rng(77)
    last = int(t.c_date[t.c_project == g].max())
    d0 = max(last + US_PER_DAY, par.SPLIT_BOUND_US + 3 * US_PER_DAY)
    dates = d0 + np.arange(extra, dtype=np.int64) * US_PER_DAY
    total = rng.integers(1000, 5000, size=extra).astype(np.int64)
    covered = (total * rng.uniform(0.0, 0.8, size=extra)).astype(np.int64)
    covered[::97] = 0                                  # zero coverage (not positive)
    valid = rng.random(extra) < 0.9
    cov = np.where(valid, covered / total * 100.0, 0.0)
    cat = lambda a, b: np.concatenate([a, b.astype(a.dtype)])  # noqa: E731
    t = dataclasses.replace(
        t, c_project=cat(t.c_project, np.full(extra, g)), c_date=cat(t.c_date, dates), c_coverage=cat(t.c_coverage, cov),
        c_coverage_valid=cat(t.c_coverage_valid, valid), c_covered=cat(t.c_covered, np.where(valid, covered, 0)),
        c_covered_valid=cat(t.c_covered_valid, valid), c_total=cat(t.c_total, np.where(valid, total, 0)),
        c_total_valid=cat(t.c_total_valid, valid))
    # corpus commit 500 days into the new rows: the project becomes group 4 (>= 7 days after creation)
    lines = t.corpus_csv.splitlines()
    name = t.projects[g]
    cc = dt.datetime(1970, 1, 1) + dt.timedelta(microseconds=int(dates[500]) + 3_600_000_000)
    for k, ln in enumerate(lines):
        if ln.startswith(name + ","):
            f = ln.split(",")
            cre = dt.datetime.fromisoformat(f[4])
            el = (cc.replace(tzinfo=cre.tzinfo) - cre).total_seconds()
            lines[k] = f"{name},True,{cc.isoformat()}+00:00,,{f[4]},{float(int(el))},"
            break
    else:
        lines.append(f"{name},True,{cc.isoformat()}+00:00,,{cc.isoformat()}+00:00,{float(30 * 86400)},")
    return dataclasses.replace(t, corpus_csv="\n".join(lines) + "\n")


def add_live_giant(t: Tables, extra: int = 80000) -> Tables:
    """A coverage-only project (its builds and issues dropped) grown to `extra` more coverage rows ten
    minutes apart BEFORE its first row - all of them before the analysis limit, so every analysis
    that reads coverage reads them (rq2_coverage_count.py:292-333 and rq4b's full series) - and put
    in rq4b's group 2: larger than a rank's share at worlds 2, 3 and 8, live_plan cuts it into
    pieces.  (NULL rows and zero coverage among the new rows.)"""
    import dataclasses
    from oracle import rq_oracle as orc
    elig = orc.eligible_projects(t)
    g = int(elig[3])
    rng = np.random.default_rng(91)
    first = int(t.c_date[t.c_project == g].min())
    dates = first - (np.arange(extra, dtype=np.int64)[::-1] + 1) * 600_000_000
    total = rng.integers(1000, 5000, size=extra).astype(np.int64)
    covered = (total * rng.uniform(0.0, 0.8, size=extra)).astype(np.int64)
    covered[::89] = 0
    total[::1999] = 0                                  # zero total: kept only by raw_n (:300-303)
    covered[::1999] = 0
    valid = rng.random(extra) < 0.93
    cov = np.where(valid & (total > 0), covered / np.maximum(total, 1) * 100.0, 0.0)
    cat = lambda a, b: np.concatenate([a, b.astype(a.dtype)])  # noqa: E731
    kb, ki = t.b_project != g, t.i_project != g
    t = dataclasses.replace(
        t, c_project=cat(t.c_project, np.full(extra, g)), c_date=cat(t.c_date, dates), c_coverage=cat(t.c_coverage, cov),
        c_coverage_valid=cat(t.c_coverage_valid, valid), c_covered=cat(t.c_covered, np.where(valid, covered, 0)),
        c_covered_valid=cat(t.c_covered_valid, valid), c_total=cat(t.c_total, np.where(valid, total, 0)),
        c_total_valid=cat(t.c_total_valid, valid),
        b_project=t.b_project[kb], b_type=t.b_type[kb], b_result=t.b_result[kb], b_time=t.b_time[kb],
        b_modules=t.b_modules[kb], b_revisions=t.b_revisions[kb], b_name=t.b_name[kb],
        i_number=t.i_number[ki], i_project=t.i_project[ki], i_rts=t.i_rts[ki], i_status=t.i_status[ki],
        i_new_id=t.i_new_id[ki])
    lines = t.corpus_csv.splitlines()
    name = t.projects[g]
    for k, ln in enumerate(lines):
        if ln.startswith(name + ","):
            f = ln.split(",")
            lines[k] = f"{name},True,{f[4]},,{f[4]},0.0,"  # group 2: corpus at creation (rq4b:183-219)
            break
    else:  # (not in the CSV: a row in group 2)
        lines.append(f"{name},True,2016-01-01T00:00:00+00:00,,2016-01-01T00:00:00+00:00,0.0,")
    return dataclasses.replace(t, corpus_csv="\n".join(lines) + "\n")


import contextlib  # noqa: E402


@contextlib.contextmanager
def elig_override(ov):
    """The oracle's eligible set with the cut projects' flags of parallel.fix_cut_eligibility (its
    functions look eligible_projects up at call time)."""
    from oracle import rq_oracle as orc
    if not ov:
        yield
        return
    orig = orc.eligible_projects

    def patched(t):
        e = set(orig(t).tolist())
        for p, f in ov.items():
            (e.add if f else e.discard)(p)
        return np.array(sorted(e), np.int64)
    orc.eligible_projects = patched
    try:
        yield
    finally:
        orc.eligible_projects = orig


class OracleEligibility:
    """fix_cut_eligibility's store access on a rank's oracle table: its qualifying-row counts and an
    override the rank's oracle shards apply (elig_override)."""

    def __init__(self, t, ov):
        self.t, self.ov = t, ov

    def elig_counts(self, ids):
        t = self.t
        m = t.c_coverage_valid & (t.c_coverage > 0) & (t.c_date < LIMIT_US)
        cnt = np.bincount(t.c_project[m].astype(np.int64), minlength=len(t.projects))
        return torch.from_numpy(cnt[np.asarray(ids, np.int64)].astype(np.int64))

    def set_eligible(self, ids, flags):
        for p, f in zip(np.asarray(ids).tolist(), np.asarray(flags).tolist()):
            self.ov[int(p)] = bool(f)


class OracleExchange:
    """The project-major exchange primitives and a cut project's tests in numpy / scipy (what
    fz_pack_runs, fz_transpose_runs, fz_sort_f64 and fz_series_dist_* do on the GPU)."""

    def pack(self, a, b, runs, sl, own, n):
        out = np.zeros(n)
        dst = np.concatenate([[0], np.cumsum(sl.sum(1))[:-1]])
        for j, (src, off, ln, base) in enumerate(runs):
            x = (a if src == 0 else b).numpy()
            for d, (lo, hi) in enumerate(own):
                s0, s1 = max(base, lo), min(base + ln, hi)
                if s1 > s0:
                    at = int(dst[d] + sl[d, :j].sum())
                    out[at:at + s1 - s0] = x[off + s0 - base:off + s1 - base]
        return torch.from_numpy(out)

    def transpose(self, vals, roffs, grp, S):
        G = 1 if grp is None else 2
        v = vals.numpy()
        lens = np.diff(roffs)
        key = np.concatenate([np.arange(ln) * G + (0 if grp is None else int(grp[k])) for k, ln in enumerate(lens)]) \
            if len(lens) else np.zeros(0, np.int64)
        o = np.argsort(key, kind="stable")
        offs = np.concatenate([[0], np.cumsum(np.bincount(key, minlength=S * G))]).astype(np.int64)
        return torch.from_numpy(v[o].copy()), torch.from_numpy(offs[:S * G + 1])

    def sort(self, x):
        o = np.argsort(x.numpy(), kind="stable")
        return torch.from_numpy(x.numpy()[o]), torch.from_numpy(o.astype(np.int32))

    def dist_state(self):
        return np.zeros(10), np.full(4, np.nan)

    def dist_partials(self, ps, v, g, m, g0, n, params, x0):
        # (the bucket itself: values and their series indices; the combine rebuilds the series)
        return torch.cat([v, g.to(torch.float64)]) if ps == 0 else torch.zeros(0, dtype=torch.float64)

    def dist_combine(self, ps, parts, k, n, params, result, sizes=None):
        if ps != 0:
            return
        p = parts.numpy()
        x = np.empty(n)
        o = 0
        for m in np.asarray(sizes).tolist():
            x[p[o + m:o + 2 * m].astype(np.int64)] = p[o:o + m]
            o += 2 * m
        result[:] = OracleRQ2CountShard.series_tests(None, torch.from_numpy(x))


def _trend_values(t, p):
    """RQ2 count's trend of project p on this table (queries1.py:120-129, rq2_coverage_count.py:
    300-303) and its fetched rows / NULL-line rows."""
    m = (t.c_project == p) & t.c_coverage_valid & (t.c_coverage != 0) & (t.c_date < LIMIT_US)
    rows = np.nonzero(m)[0]
    rows = rows[np.argsort(t.c_date[rows], kind="stable")]
    keep = (t.c_total[rows] != 0) | ~t.c_total_valid[rows]
    kr = rows[keep]
    null = int((~(t.c_total_valid[kr] & t.c_covered_valid[kr])).sum())
    vals = t.c_covered[kr].astype(np.float64) / t.c_total[kr].astype(np.float64) * 100
    return vals, len(rows), null


def _series_values(t, p):
    """rq4b's full series of project p on this table (coverage > 0, date < LIMIT, rq4b:315-326)."""
    m = (t.c_project == p) & t.c_coverage_valid & (t.c_coverage > 0) & (t.c_date < LIMIT_US)
    rows = np.nonzero(m)[0]
    return t.c_coverage[rows[np.argsort(t.c_date[rows], kind="stable")]]


class OracleRQ1Shard:
    def __init__(self, t, rows, max_iter, threshold=100, ov=None):
        self.ov = ov
        self.t, self.rows, self.M, self.threshold = t, rows, max_iter, threshold

    def run(self, ext):
        from oracle import rq_oracle as orc
        with elig_override(self.ov):
            r = orc.rq1(self.t, self.threshold, ext=None if ext is None else tuple(x.numpy() for x in ext))
        self.result = r
        c = np.zeros(par.RQ1_NCOUNTS, np.int64)
        c[par.RQ1_ISSUES_LIM], c[par.RQ1_ISSUES_LIM_PROJECTS] = r.n_issues_lim, r.n_issues_lim_projects
        c[par.RQ1_FIXED_LIM], c[par.RQ1_FIXED_LIM_PROJECTS] = r.n_fixed_lim, r.n_fixed_lim_projects
        c[par.RQ1_ELIGIBLE], c[par.RQ1_WITHOUT_MATCHING] = len(r.eligible), r.n_without_matching
        c[par.RQ1_TARGET], c[par.RQ1_TARGET_PROJECTS] = r.n_target, r.n_target_projects
        c[par.RQ1_TOTAL_FUZZ], c[par.RQ1_MATCHED] = r.total_fuzz_builds, len(r.matched_issue)
        c[par.RQ1_MATCHED_PROJECTS], c[par.RQ1_MAX_ITER] = r.n_matched_projects, len(r.iter_total)
        it = np.zeros(self.M, np.int64)
        idt = np.zeros(self.M, np.int64)
        it[:len(r.iter_total)] = r.iter_total
        idt[:len(r.iter_detected)] = r.iter_detected
        return {"counts": torch.from_numpy(c), "iter_total": torch.from_numpy(it),
                "iter_detected": torch.from_numpy(idt),
                "number": torch.from_numpy(self.t.i_number[r.matched_issue].astype(np.int64)),
                "build_time": torch.from_numpy(self.t.b_time[r.matched_build].astype(np.int64)),
                "matched_issue": torch.from_numpy(self.rows.issues[r.matched_issue].astype(np.int64)),
                "matched_build": torch.from_numpy(self.rows.builds[r.matched_build].astype(np.int64))}

    def finish(self, counts, it, idt):
        M = int(counts[par.RQ1_MAX_ITER])
        keys, rates, first_down, late = common.rq1_rates(it.numpy()[:M], idt.numpy()[:M], self.threshold)
        counts[par.RQ1_KEPT_ITERS] = len(keys)
        counts[par.RQ1_FIRST_DOWN] = first_down
        counts[par.RQ1_LATE] = len(late)
        self.late = late


class OracleRQ3Shard:
    def __init__(self, t, rows, ov=None):
        self.ov = ov
        self.t, self.rows = t, rows

    def run(self):
        from oracle import rq_oracle as orc
        with elig_override(self.ov):
            r = orc.rq3(self.t, flush_last=True, on_null="count")
        c = np.zeros(par.RQ3_NCOUNTS, np.int64)
        c[par.RQ3_ISSUES], c[par.RQ3_DETECTED], c[par.RQ3_NON_DETECTED] = r.n_all_issues, len(r.det_pct), len(r.non_pct)
        c[par.RQ3_ELIGIBLE], c[par.RQ3_NON_LAST] = len(orc.eligible_projects(self.t)), r.n_non_last
        c[par.RQ3_NULL_TOTAL], c[par.RQ3_NULL_LAST] = r.n_null_total, r.n_null_last
        T = lambda a, dt=np.int64: torch.from_numpy(np.ascontiguousarray(a, dtype=dt))  # noqa: E731
        return {"counts": T(c), "det_pct": T(r.det_pct, np.float64), "det_cov": T(r.det_cov), "det_tot": T(r.det_tot),
                "det_project": T(r.det_project), "det_issue": T(self.rows.issues[r.det_issue]),
                "non_pct": T(r.non_pct, np.float64), "non_cov": T(r.non_cov), "non_tot": T(r.non_tot)}

    def stats(self, det_pct, det_tot, non_pct):
        from oracle import rq_oracle as orc
        return orc.rq3_stats(det_pct.numpy(), det_tot.numpy(), non_pct.numpy())


def _offs_to_ids(offs, S):
    """Segment id of every value of a segment-grouped layout (offsets [S + 1])."""
    o = offs.to(torch.int64)
    return torch.repeat_interleave(torch.arange(S, dtype=torch.int64), o[1:S + 1] - o[:S])


class OracleRQ2CountShard(OracleExchange):
    """One rank's RQ2 count on the CPU restatement (per-project columns over the global project
    axis + the local trend values project-major), and the session / series statistics the exchange
    needs, computed exactly as rq_oracle.rq2_count does."""

    def __init__(self, t, cont=-1, ov=None):
        self.t, self.cont, self.ov = t, cont, ov

    def run(self):
        from oracle import rq_oracle as orc
        with elig_override(self.ov):
            r = orc.rq2_count(self.t)
        P = len(self.t.projects)
        el = np.zeros(P, np.int64)
        el[r.eligible] = 1
        cols = {"eligible": el, "raw_n": np.zeros(P, np.int64), "n_trend": np.zeros(P, np.int64),
                "sw_w": np.full(P, np.nan), "sw_p": np.full(P, np.nan), "corr": np.full(P, np.nan)}
        cols["raw_n"][r.eligible] = r.raw_n
        cols["n_trend"][r.eligible] = r.n_trend
        cols["sw_w"][r.eligible] = r.sw_w
        cols["sw_p"][r.eligible] = r.sw_p
        cols["corr"][r.eligible[r.raw_n > 0]] = r.corr
        out = {k: torch.from_numpy(v) for k, v in cols.items()}
        vals = [_trend_values(self.t, p)[0] for p in r.eligible.tolist()]
        out["values"] = torch.from_numpy(np.concatenate(vals) if vals else np.zeros(0))
        out["null_lines"] = torch.zeros(1, dtype=torch.int64)
        if self.cont >= 0:
            v, raw, null = _trend_values(self.t, self.cont)
            out["piece_values"] = torch.from_numpy(v)
            out["piece_counts"] = torch.tensor([len(v), raw, null], dtype=torch.int64)
        return out

    def merge_runs(self, vals, runs):
        return par.merge_runs_torch(vals, runs)

    def session_stats_grouped(self, vals, offs, S, max_len):
        return self.session_stats(vals, _offs_to_ids(offs, S), S, max_len)

    def session_stats(self, vals, sids, S, max_len):
        import statistics
        v, s_ = vals.numpy(), sids.numpy()
        avg, med, pct = np.full(S, np.nan), np.full(S, np.nan), np.full(5 * S, np.nan)
        for i in range(S):
            x = list(v[s_ == i])
            if x:
                avg[i] = statistics.mean(x)
                med[i] = statistics.median(x)
                pct[5 * i:5 * i + 5] = [np.percentile(x, q) for q in (5, 25, 50, 75, 95)]
        T = torch.from_numpy
        return {"average": T(avg), "median": T(med), "percentiles": T(pct),
                "ge100": torch.tensor([int(np.sum(np.bincount(s_, minlength=S) >= 100))])}

    def series_tests(self, x):
        import warnings
        from scipy import stats
        m = list(x.numpy())
        rho = p = w = sp = float("nan")
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            if len(m) > 1:
                r = stats.spearmanr(list(range(len(m))), m)
                rho, p = float(r.statistic), float(r.pvalue)
            if len(m) >= 3:
                w, sp = (float(z) for z in stats.shapiro(m))
        return rho, p, w, sp

    def mean_median(self, x):
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            return float(np.mean(x.numpy())), float(np.median(x.numpy()))


class OracleRQ2AddShard:
    """One rank's RQ2 add on the CPU restatement: flags over the global project axis, change rows
    with global build / coverage row ids (-1 kept)."""

    def __init__(self, t, rows, ov=None):
        self.t, self.rows, self.ov = t, rows, ov

    def run(self):
        from oracle import rq_oracle as orc
        with elig_override(self.ov):
            return rq2_add_part(orc.rq2_add(self.t), len(self.t.projects), self.rows)


def rq2_add_part(r, P, rows):
    """An RQ2AddResult of one shard in rq2_add_sharded's run() layout, row ids mapped to the table's."""
    def gid(ids, table):
        ids = np.asarray(ids, np.int64)
        return np.where(ids >= 0, table[np.maximum(ids, 0)] if len(table) else ids, -1).astype(np.int64)
    el = np.zeros(P, np.int64)
    el[r.projects] = 1
    T = lambda a, dt=np.int64: torch.from_numpy(np.ascontiguousarray(a, dtype=dt))  # noqa: E731
    return {"eligible": T(el), "covered_is_float": T(r.covered_is_float), "total_is_float": T(r.total_is_float),
            "row_project": T(r.row_project), "row_first_build": T(gid(r.row_first_build, rows.builds)),
            "row_end_build": T(gid(r.row_end_build, rows.builds)),
            "row_start_build": T(gid(r.row_start_build, rows.builds)),
            "row_cov_i": T(gid(r.row_cov_i, rows.coverage)), "row_cov_i1": T(gid(r.row_cov_i1, rows.coverage)),
            "diff_total": T(r.diff_total, np.float64), "diff_coverage": T(r.diff_coverage, np.float64)}


def rq2_add_result(flags, cols):
    """The recombined RQ2AddResult of rq2_add_sharded's output."""
    from tse_amd.rq.results import RQ2AddResult
    f = {k: np.asarray(v) for k, v in flags.items()}
    return RQ2AddResult(projects=np.nonzero(f["eligible"])[0],
                        **{k: np.asarray(cols[k]) for k in par.RQ2A_ROW_COLS},
                        covered_is_float=f["covered_is_float"].astype(bool),
                        total_is_float=f["total_is_float"].astype(bool))


class OracleRQ4aShard:
    """One rank's RQ4a on the CPU restatement, in fz_rq4a's output layout."""

    def __init__(self, t, max_iter, ov=None):
        self.ov = ov
        self.t, self.M = t, max_iter

    def run(self):
        from oracle import rq_oracle as orc
        with elig_override(self.ov):
            r = orc.rq4a(self.t)
        P = len(self.t.projects)
        c = np.zeros(12, np.int64)
        c[0] = len(r.g1_total)
        for g in range(4):
            c[2 + g] = len(r.groups[f"group{g + 1}"])
        c[6] = int(r.has_g4_transition)
        c[9] = sum(1 for _, k in r.intro if k > 0)
        member = np.zeros(P, np.int64)
        for g in range(4):
            member[r.groups[f"group{g + 1}"]] |= 1 << g
        intro = np.full(P, -1, np.int64)
        for p, k in r.intro:
            intro[p] = k
        steps = np.zeros((15, 2), np.int64)
        for s_, (a, b) in r.g4_steps.items():
            steps[s_ + 7] = (a, b)
        out = {"counts": torch.from_numpy(c), "member": torch.from_numpy(member), "intro": torch.from_numpy(intro),
               "g4_steps": torch.from_numpy(steps.reshape(-1)),
               "g4_transition": torch.from_numpy(np.array(r.g4_transition, np.int64))}
        for k in ("g1_total", "g1_det", "g2_total", "g2_det"):
            a = np.zeros(self.M, np.int64)
            a[:len(getattr(r, k))] = getattr(r, k)
            out[k] = torch.from_numpy(a)
        return out

    def finish(self, tables, intro, steps, counts):
        from oracle import rq_oracle as orc
        M = int(counts[0])
        t4 = [x.numpy()[:M] for x in tables]
        st = steps.numpy().reshape(15, 2)
        sd = {s_: tuple(st[s_ + 7]) for s_ in list(range(-7, 0)) + list(range(1, 8))}
        iv = [int(k) for k in intro.numpy() if k >= 0]
        after, istats, overall = orc.rq4a_finish(*t4, iv, sd)
        rows = common.rq4a_rows(*t4)
        counts[1] = len(rows)
        sc = np.full(12, np.nan)
        for key, n, m in (("g1", 7, 0), ("g2", 8, 2)):
            counts[n] = 1 if after[key] is not None else 0
            if after[key] is not None:
                sc[m], sc[m + 1] = after[key]
        if istats is not None:
            sc[4:8] = istats
        sc[8], sc[9] = overall
        return sc


class OracleRQ4bShard(OracleRQ2CountShard):
    """One rank's RQ4b on the CPU restatement, in fz_rq4b_ex's shard output layout."""

    def run(self):
        with elig_override(self.ov):
            return self._run()

    def _run(self):
        from oracle import rq_oracle as orc
        t = self.t
        P = len(t.projects)
        elig = orc.eligible_projects(t)
        groups, corpus_us = common.corpus_groups(t, elig, add_missing_to_g1=False)
        member = np.zeros(P, np.int64)
        for g in range(4):
            member[groups[f"group{g + 1}"]] |= 1 << g
        full = orc.rq4b_full_series(t, P)
        # the G1/G2 series project-major (project order, date order inside one)
        vals = [t.c_coverage[full.rows(p)] if member[p] & 3 else np.zeros(0) for p in range(P)]
        offs = np.concatenate([[0], np.cumsum([len(v) for v in vals])]).astype(np.int64)
        m_loc = max([len(v) for v in vals] + [0])
        vals = np.concatenate(vals) if vals else np.zeros(0)
        order = common.corpus_columns(t)[2].tolist()
        projs, pre, post = orc.rq4b_deltas(t, elig, groups, corpus_us)
        # CSV row of each delta column: the k-th qualifying row of the corpus order
        dord, k0 = [], 0
        for p in projs:
            k0 = order.index(p, k0)
            dord.append(k0)
            k0 += 1
        init = {g: np.array([t.c_coverage[full.rows(p)[0]] for p in sorted(groups[g]) if len(full.rows(p))],
                            np.float64) for g in ("group2", "group1")}
        c = np.zeros(12, np.int64)
        c[par.RQ4B_DELTA_PROJECTS], c[par.RQ4B_INIT_G2], c[par.RQ4B_INIT_G1] = len(projs), len(init["group2"]), \
            len(init["group1"])
        c[par.RQ4B_SESSIONS] = m_loc
        c[par.RQ4B_VALUES] = len(vals)
        for g in range(4):
            c[5 + g] = len(groups[f"group{g + 1}"])
        T = lambda a, dt=np.float64: torch.from_numpy(np.ascontiguousarray(a, dtype=dt))  # noqa: E731
        out = {"counts": T(c, np.int64), "member": T(member, np.int64),
                "trend_values": T(vals), "trend_offsets": T(offs, np.int64),
                "pre_cov": T(np.concatenate(pre) if projs else np.zeros(0)),
                "post_cov": T(np.concatenate(post) if projs else np.zeros(0)), "delta_order": T(dord, np.int64),
                "init_g2": T(init["group2"]), "init_g1": T(init["group1"])}
        if self.cont >= 0:
            v = _series_values(t, self.cont)
            out["piece_values"] = T(v)
            out["piece_counts"] = torch.tensor([len(v), len(v), 0], dtype=torch.int64)
        return out

    def spearman_prefix(self, rows, n):
        n = int(n)
        return np.array([self.series_tests(r[:n])[:2] for r in rows])

    def session_stats_grouped(self, vals, offs2, S, max_len):
        from oracle import rq_oracle as orc
        v, o = vals.numpy(), offs2.numpy()
        s2 = [list(v[o[2 * i]:o[2 * i + 1]]) for i in range(S)]
        s1 = [list(v[o[2 * i + 1]:o[2 * i + 2]]) for i in range(S)]
        c2, c1, q2, q1, pb = orc.rq4b_session_stats(s2, s1)
        T = torch.from_numpy
        return {"c2": T(c2), "c1": T(c1), "g2_q": T(q2.reshape(-1)), "g1_q": T(q1.reshape(-1)), "p_bm": T(pb)}

    def row_medians(self, rows):
        r = rows.numpy()
        return np.array([float(np.median(x)) if len(x) else np.nan for x in r])

    def two_sample(self, x, y):
        from oracle import rq_oracle as orc
        mwu, cliff, bm, lv = orc.rq4b_init_tests(x.numpy(), y.numpy())
        out = np.full(8, np.nan)
        if mwu is not None:
            out[:6] = [mwu, cliff, bm[0], bm[1], lv[0], lv[1]]
        return out


def _worker(rank, world, port, case, errfile, threaded=False, deferred=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _check(rank, world, case, threaded, deferred)
    except BaseException as e:  # report to the parent (mp.spawn only sees the exit code)
        with open(f"{errfile}.{rank}", "w") as f:
            import traceback
            f.write(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


def _check(rank, world, case, threaded=False, deferred=False):
    from oracle import rq_oracle as orc
    from gpu_common import assert_same
    t = make_table(case, world)
    cont, ov = -1, {}
    if case == "giant":  # the giant's movable coverage rows spread over the ranks (split_plan)
        plan = par.split_plan(t, world)
        assert plan.moved > 0, "the giant's rows past the date bounds were meant to move"
        lo, hi = plan.bounds[rank]
        ts, rows = par.take_split(t, plan, rank)
    elif case == "live_giant":  # the live giant cut into date-range pieces (live_plan)
        plan = par.live_plan(t, world)
        assert len(plan.cut) == 1 and plan.moved > 0, "the live giant was meant to be cut"
        lo, hi = plan.bounds[rank]
        ts, rows = par.take_split(t, plan, rank)
        cont = plan.cont[rank]
        par.fix_cut_eligibility(OracleEligibility(ts, ov), plan.cut, lo, hi, world)
    else:
        lo, hi = par.shard_bounds(t, world)[rank]
        ts, rows = par.take_shard(t, lo, hi)
    nF = np.bincount(ts.b_project[ts.b_type == 0].astype(np.int64), minlength=len(t.projects))
    M = par.agree_max(int(nF.max()) if len(nF) else 0)
    nF4 = np.bincount(ts.b_project[(ts.b_type == 0) & (ts.b_time < LIMIT_US)].astype(np.int64),
                      minlength=len(t.projects))
    M4 = par.agree_max(int(nF4.max()) if len(nF4) else 1)

    def rq1():
        sh = OracleRQ1Shard(ts, rows, max(M, 1), ov=ov)
        part, counts, it, idt, reran = par.rq1_sharded(sh, rank, world)
        rows1 = par.gather_rows({"matched_issue": part["matched_issue"], "matched_build": part["matched_build"]},
                                world)
        any_rerun = torch.tensor([int(reran)])
        par.all_reduce(any_rerun)
        return counts, it, idt, rows1, any_rerun

    # deferred: the drivers' final host copies left to one par.finalize_all at the end (the bench's
    # single-thread sharded step)
    drivers = {"rq1": rq1,
               "rq3": lambda: par.rq3_sharded(OracleRQ3Shard(ts, rows, ov=ov), rank, world),
               "rq2a": lambda: par.rq2_add_sharded(OracleRQ2AddShard(ts, rows, ov=ov), rank, world),
               "rq2": lambda: par.rq2_count_sharded(OracleRQ2CountShard(ts, cont, ov), rank, world, lo, hi,
                                                    finish_later=deferred, cont=cont),
               "rq4a": lambda: par.rq4a_sharded(OracleRQ4aShard(ts, M4, ov=ov), rank, world, lo, hi,
                                                finish_later=deferred),
               "rq4b": lambda: par.rq4b_sharded(OracleRQ4bShard(ts, cont, ov), rank, world, lo=lo, hi=hi,
                                                finish_later=deferred, cont=cont)}
    if threaded:
        # the bench's sharded step: every driver in its own thread over its own process group (their
        # collectives interleave differently on every rank)
        from concurrent.futures import ThreadPoolExecutor
        groups = {k: torch.distributed.new_group(backend="gloo") for k in drivers}

        def run(k):
            with par.use_group(groups[k]):
                return drivers[k]()
        with ThreadPoolExecutor(len(drivers)) as pool:
            futs = {k: pool.submit(run, k) for k in (list(drivers)[::-1] if rank % 2 else list(drivers))}
            res = {k: f.result() for k, f in futs.items()}
    else:
        res = {k: f() for k, f in drivers.items()}
    if deferred:
        ks = list(res)
        assert any(isinstance(res[k], par.Deferred) for k in ks)
        res = dict(zip(ks, par.finalize_all([res[k] for k in ks])))
    counts, it, idt, rows1, any_rerun = res["rq1"]
    total3, cols3, st3 = res["rq3"]
    r2, r4, r4b = res["rq2"], res["rq4a"], res["rq4b"]
    if not threaded and not deferred and case in ("collide", "live_giant"):
        _check_owner_sessions(rank, world, case, r2, r4b, lambda: (
            par.rq2_count_sharded(OracleRQ2CountShard(ts, cont, ov), rank, world, lo, hi, cont=cont,
                                  host_sessions=False),
            par.rq4b_sharded(OracleRQ4bShard(ts, cont, ov), rank, world, lo=lo, hi=hi, cont=cont,
                             host_sessions=False)))
    if rank != 0:
        return
    assert_same(rq2_add_result(*res["rq2a"]), orc.rq2_add(t), "rq2_add")
    g = orc.rq1(t)
    assert case in ("giant", "live_giant") or world == 1 or int(any_rerun) > 0, \
        "the table was built to need the cross-shard dedup"
    c = counts.numpy()
    assert c[par.RQ1_ISSUES_LIM] == g.n_issues_lim and c[par.RQ1_ISSUES_LIM_PROJECTS] == g.n_issues_lim_projects
    assert c[par.RQ1_FIXED_LIM] == g.n_fixed_lim and c[par.RQ1_FIXED_LIM_PROJECTS] == g.n_fixed_lim_projects
    assert c[par.RQ1_ELIGIBLE] == len(g.eligible) and c[par.RQ1_WITHOUT_MATCHING] == g.n_without_matching
    assert c[par.RQ1_TARGET] == g.n_target and c[par.RQ1_TARGET_PROJECTS] == g.n_target_projects
    assert c[par.RQ1_TOTAL_FUZZ] == g.total_fuzz_builds
    assert c[par.RQ1_MATCHED] == len(g.matched_issue) and c[par.RQ1_MATCHED_PROJECTS] == g.n_matched_projects
    Mg = int(c[par.RQ1_MAX_ITER])
    assert Mg == len(g.iter_total)
    np.testing.assert_array_equal(it.numpy()[:Mg], g.iter_total)
    np.testing.assert_array_equal(idt.numpy()[:Mg], g.iter_detected)
    np.testing.assert_array_equal(rows1["matched_issue"].numpy(), g.matched_issue)
    np.testing.assert_array_equal(rows1["matched_build"].numpy(), g.matched_build)
    _, _, first_down, late = common.rq1_rates(g.iter_total, g.iter_detected, 100)
    assert c[par.RQ1_FIRST_DOWN] == first_down and c[par.RQ1_LATE] == len(late)
    g3 = orc.rq3(t)
    assert total3[par.RQ3_ISSUES] == g3.n_all_issues
    for k in ("det_pct", "det_cov", "det_tot", "det_project", "det_issue", "non_pct", "non_cov", "non_tot"):
        np.testing.assert_array_equal(cols3[k].numpy(), getattr(g3, k), err_msg=k)
    for k, v in st3.items():
        assert_same(v, getattr(g3, k), k)
    from tse_amd.rq import compute
    ours2 = compute.rq2_count_result(r2["proj"], r2["session_offsets"], r2["session_values"], r2["K"],
                                     r2["average"], r2["median"], r2["percentiles"], r2["average"],
                                     (r2["tests"][0], r2["tests"][1], r2["tests"][3]), r2["corr_mm"], r2["null_lines"])
    assert_same(ours2, orc.rq2_count(t), "rq2_count")
    ours4 = compute.rq4a_result(r4["counts"], r4["scalars"], r4["member"], r4["tables"], r4["intro"], r4["g4_steps"],
                                r4["g4_transition"])
    assert_same(ours4, orc.rq4a(t), "rq4a")
    ours4b = compute.rq4b_result(r4b["counts"], r4b["c2"], r4b["c1"], r4b["g2_q"], r4b["g1_q"], r4b["p_bm"],
                                 r4b["sp6"], r4b["pre_cov"], r4b["post_cov"], r4b["pre_median"], r4b["post_median"],
                                 r4b["init_g2"], r4b["init_g1"], r4b["tests"])
    assert_same(ours4b, orc.rq4b(t), "rq4b")


def _check_owner_sessions(rank, world, case, r2, r4b, again):
    """host_sessions=False (the bench's step): the per-session rows stay on their owners and only the
    prefixes the tails read are gathered - the same tests, and the owners' rows in session order are
    the gathered ones."""
    r2o, r4o = again()
    assert r2o["K"] == r2["K"]
    np.testing.assert_array_equal(np.array(r2o["tests"] + r2o["corr_mm"]), np.array(r2["tests"] + r2["corr_mm"]))
    np.testing.assert_array_equal(r4o["sp6"], r4b["sp6"])
    np.testing.assert_array_equal(r4o["counts"], r4b["counts"])
    nt = 6  # (MWU p, Cliff, BM stat / p, Levene W / p; the last two of FZ_RQ4B_NTESTS slots are padding)
    np.testing.assert_array_equal(r4o["tests"][:nt], r4b["tests"][:nt])
    s2, s4 = r2o["sessions"], r4o["sessions"]
    h = lambda x: x.cpu().numpy()  # noqa: E731
    a, b = s2["range"]
    np.testing.assert_array_equal(h(s2["median"]), r2["median"][a:b])
    np.testing.assert_array_equal(h(s2["average"]), r2["average"][a:b])
    np.testing.assert_array_equal(h(s2["percentiles"]), r2["percentiles"][5 * a:5 * b])
    a, b = s4["range"]
    np.testing.assert_array_equal(h(s4["cols"][0]), r4b["c2"][a:b])
    np.testing.assert_array_equal(h(s4["cols"][1]), r4b["c1"][a:b])
    np.testing.assert_array_equal(h(s4["cols"][8]), r4b["p_bm"][a:b])


def _rehearse(rank, world, port, case, errfile, threaded=False, deferred=False):
    """bench.py --strong --shard-of W at world 1: every shard of a W-rank live_plan run alone (its
    leading piece, without the earlier pieces, starts at session 0).  The runs the owner transposes
    must be exactly what the pack sends - the shard holding only the giant's later piece once read
    past its packed values on the GPU; the piece's values are a contiguous date range of the
    project's trend values."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        t = make_table("live_giant", 1)
        plan = par.live_plan(t, world)
        p_cut = int(plan.cut[0])
        full = _trend_values(t, p_cut)[0]
        seen = 0
        for r in range(world):
            lo, hi = plan.bounds[r]
            ts, rows = par.take_split(t, plan, r)
            cont = plan.cont[r]
            ov = {}
            par.fix_cut_eligibility(OracleEligibility(ts, ov), plan.cut, lo, hi, 1)
            r2 = par.rq2_count_sharded(OracleRQ2CountShard(ts, cont, ov), 0, 1, lo, hi, cont=cont)
            par.rq4b_sharded(OracleRQ4bShard(ts, cont, ov), 0, 1, lo=lo, hi=hi, cont=cont)
            if cont == p_cut:
                seen += 1
                piece = _trend_values(ts, p_cut)[0]
                assert len(piece) and int(r2["proj"]["n_trend"][p_cut]) == len(piece)
                b0 = sum(len(_trend_values(par.take_split(t, plan, q)[0], p_cut)[0]) for q in plan.ranks[p_cut] if q < r)
                assert b0 > 0 and np.array_equal(full[b0:b0 + len(piece)], piece, equal_nan=True)
        assert seen >= 1, "no rank held a continuation piece"
    except BaseException:
        with open(f"{errfile}.{rank}", "w") as f:
            import traceback
            f.write(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


def test_one_gpu_rehearsal_shards_of_live_giant(tmp_path):
    errfile = str(tmp_path / "err")
    try:
        mp.spawn(_rehearse, args=(3, _free_port(), "live_giant", errfile), nprocs=1, join=True)
    except Exception:
        msgs = [open(f"{errfile}.0").read()] if os.path.exists(f"{errfile}.0") else []
        raise AssertionError("\n".join(msgs) or "worker failed")


def _spawn(world, case, tmp_path, threaded=False, deferred=False):
    errfile = str(tmp_path / "err")
    try:
        mp.spawn(_worker, args=(world, _free_port(), case, errfile, threaded, deferred), nprocs=world, join=True)
    except Exception:
        msgs = [open(f"{errfile}.{r}").read() for r in range(world) if os.path.exists(f"{errfile}.{r}")]
        raise AssertionError("\n".join(msgs) or "worker failed")


def test_shard_bounds_cover_and_balance():
    t = synth.generate(synth.config("tiny"))
    for world in (1, 2, 3, 8):
        b = par.shard_bounds(t, world)
        assert b[0][0] == 0 and b[-1][1] == len(t.projects)
        assert all(b[r][1] == b[r + 1][0] for r in range(world - 1))
        parts = [par.take_shard(t, lo, hi)[0] for lo, hi in b]
        assert sum(p.n_rows for p in parts) == t.n_rows
        if world > 1:
            sizes = np.array([p.n_rows for p in parts], float)
            assert sizes.max() <= 2.5 * t.n_rows / world


@pytest.mark.parametrize("world,case", [(1, "collide"), (2, "collide"), (3, "collide"), (3, "last_shard_no_issues"), (8, "collide"),
                                        (8, "last_shard_no_issues"), (2, "giant"), (3, "giant"), (8, "giant"),
                                        (2, "live_giant"), (3, "live_giant"), (8, "live_giant")])
def test_sharded_rq1_rq3_match_whole_table(world, case, tmp_path):
    _spawn(world, case, tmp_path)


@pytest.mark.parametrize("world,case", [(2, "collide"), (3, "last_shard_no_issues")])
def test_sharded_drivers_concurrent_groups(world, case, tmp_path):
    """The five drivers at once, one thread and one process group each (bench.py's sharded step),
    started in a different order on odd ranks: the same exact results as one after another."""
    _spawn(world, case, tmp_path, threaded=True)


@pytest.mark.parametrize("world,case", [(2, "collide"), (3, "last_shard_no_issues")])
def test_sharded_drivers_deferred_results(world, case, tmp_path):
    """The drivers one after another in one thread with their final host copies deferred to one
    finalize_all (the bench's sharded step: one collective order on every rank): the same exact
    results."""
    _spawn(world, case, tmp_path, deferred=True)


def test_host_many_round_trips_dtypes():
    import torch
    ts = [torch.arange(5, dtype=torch.int64), torch.tensor([1.5, -2.0]), torch.tensor([[1, 2], [3, 4]], dtype=torch.uint8),
          np.array([7, 8], dtype=np.int32)]
    out = par.host_many(*ts)
    for t, o in zip(ts, out):
        ref = t.numpy() if isinstance(t, torch.Tensor) else t
        assert o.dtype == ref.dtype and o.shape == ref.shape and np.array_equal(o, ref)
