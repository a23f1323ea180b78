"""The libfz primitives behind a project cut across ranks (fz.h "a project cut across ranks";
parallel.live_plan / _exchange_runs / _series_tests_cut), each against a plain numpy / scipy
restatement on one GPU:

* fz_series_dist_partials / _combine over value buckets (ties never crossing a bucket) equal
  fz_series_tests of the whole series - spearmanr(range(n), x) and shapiro(x),
  rq2_coverage_count.py:305-322 - and scipy, on tie-heavy and continuous series;
* fz_transpose_runs (coverage_by_session_index, :329-333, per group as rq4b:917-931) and
  fz_pack_runs (the runs' slices per session owner) value for value;
* fz_piece_values: one project's RQ2 trend values and rq4b series from the store, as the oracle
  filters them (queries1.py:120-129, rq4b_coverage.py:315-326);
* fz_store_elig_counts / fz_store_set_eligible: the counts of rq1:144-152 and an override every
  analysis then reads."""

import numpy as np
import pytest
import torch

from gpu_common import assert_same

pytestmark = pytest.mark.gpu


def _series(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "ties":
        return np.round(rng.normal(50, 10, n)).astype(np.float64)      # ~60 distinct values
    if kind == "trend":
        return np.linspace(10, 90, n) + rng.normal(0, 3, n)
    return rng.uniform(0, 100, n)


@pytest.mark.parametrize("kind,n,k", [("ties", 200_000, 3), ("trend", 50_000, 2), ("uniform", 123_457, 5),
                                      ("ties", 9, 2), ("uniform", 3_000_000, 8)])
def test_series_dist_equals_one_series(engine, kind, n, k):
    from scipy import stats
    from tse_amd import parallel as par
    eng = engine
    x = _series(kind, n, 7 + n)
    xd = torch.from_numpy(x).to(eng.dev)
    whole = torch.empty(4, dtype=torch.float64, device=eng.dev)
    import ctypes as C
    from tse_amd import engine as E
    E._check(eng.lib, eng.lib.fz_series_tests(eng.ctx, C.c_void_p(xd.data_ptr()), n, C.c_void_p(whole.data_ptr())))
    whole = whole.cpu().numpy()
    # buckets of the sorted series at value boundaries (ties inside one bucket)
    o = np.argsort(x, kind="stable")
    xs = x[o]
    cuts = [0]
    for q in range(1, k):
        c = int(np.searchsorted(xs, xs[n * q // k], "right"))
        cuts.append(max(c, cuts[-1]))
    cuts.append(n)
    sh = par.GpuRQ2CountShard.__new__(par.GpuRQ2CountShard)
    sh.E, sh.C, sh.eng = E, C, eng
    params, result = sh.dist_state()
    x0 = xd[n // 2:n // 2 + 1]
    for ps in range(3):
        parts = []
        for b in range(k):
            a, e = cuts[b], cuts[b + 1]
            # (the bucket's values in a shuffled order, sorted again as the driver does)
            sel = o[a:e][np.random.default_rng(b).permutation(e - a)]
            v, pos = sh.sort(torch.from_numpy(x[sel]).to(eng.dev))
            g = torch.from_numpy(sel.astype(np.int64)).to(eng.dev)[pos.to(torch.int64)]
            parts.append(sh.dist_partials(ps, v, g, e - a, a, n, params, x0 if (ps == 0 and b == 0) else None))
        sh.dist_combine(ps, torch.cat(parts), k, n, params, result)
    got = result.cpu().numpy()
    assert_same(got, whole, f"{kind} n={n} k={k}")
    if n >= 3:
        r = stats.spearmanr(np.arange(n), x)
        w = stats.shapiro(x)
        # (scipy warns that its Shapiro-Wilk p-value is not accurate past 5,000 values: W only there)
        k_cmp = 4 if n <= 5000 else 3
        assert_same(got[:k_cmp], np.array([r.statistic, r.pvalue, w.statistic, w.pvalue])[:k_cmp], "scipy")


@pytest.mark.parametrize("G", [1, 2])
def test_transpose_and_pack_runs(engine, G):
    from tse_amd import parallel as par
    import ctypes as C
    from tse_amd import engine as E
    eng = engine
    sh = par.GpuRQ4bShard.__new__(par.GpuRQ4bShard)
    sh.E, sh.C, sh.eng = E, C, eng
    rng = np.random.default_rng(3)
    lens = np.r_[rng.integers(0, 300, size=200), [50_000, 7, 0, 20_000]].astype(np.int64)
    grp = rng.integers(0, 2, size=len(lens)).astype(np.uint8) if G == 2 else None
    offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    vals = rng.normal(size=int(offs[-1]))
    S = int(lens.max())
    out, oo = sh.transpose(torch.from_numpy(vals).to(eng.dev), offs, grp, S)
    key = np.concatenate([np.arange(L) * G + (0 if grp is None else int(grp[k])) for k, L in enumerate(lens)])
    o = np.argsort(key, kind="stable")
    exp_offs = np.concatenate([[0], np.cumsum(np.bincount(key, minlength=S * G))])
    assert np.array_equal(oo.cpu().numpy(), exp_offs)
    assert np.array_equal(out.cpu().numpy(), vals[o])
    # pack: runs (src, src_off, len, base) cut by four owners' session ranges
    b_vals = rng.normal(size=5000)
    runs = [(1, 100, 4000, 60_000)] + [(0, int(offs[k]), int(lens[k]), 0) for k in range(len(lens)) if lens[k]]
    own = [(0, 100), (100, 1000), (1000, 61_000), (61_000, 70_000)]
    sl = par._Runs.slices(runs, own)
    packed = sh.pack(torch.from_numpy(vals).to(eng.dev), torch.from_numpy(b_vals).to(eng.dev), runs, sl, own,
                     int(sl.sum())).cpu().numpy()
    exp = []
    for lo, hi in own:
        for src, off, ln, base in runs:
            s0, s1 = max(base, lo), min(base + ln, hi)
            if s1 > s0:
                exp.append((vals if src == 0 else b_vals)[off + s0 - base:off + s1 - base])
    assert np.array_equal(packed, np.concatenate(exp))


def test_piece_values_and_eligibility_override(engine):
    import ctypes as C
    from tse_amd import engine as E
    from tse_amd import parallel as par
    from tse_amd import synth
    from tse_amd.rq import compute
    from tse_amd.schema import LIMIT_US
    from oracle import rq_oracle as orc
    t = synth.generate(synth.config("tiny"))
    eng = engine
    eng.upload(t)
    eng.build_store()
    sh = par.GpuRQ2CountShard(eng)
    for p in range(len(t.projects)):
        m = (t.c_project == p) & t.c_coverage_valid & (t.c_coverage != 0) & (t.c_date < LIMIT_US)
        rows = np.nonzero(m)[0]
        rows = rows[np.argsort(t.c_date[rows], kind="stable")]
        keep = (t.c_total[rows] != 0) | ~t.c_total_valid[rows]
        kr = rows[keep]
        sh.cont = p
        sh._piece(E.FZ_PIECE_RQ2)
        cnt = sh._pc.cpu().numpy()
        n = int(cnt[0])
        assert n == len(kr) and cnt[1] == len(rows)
        assert cnt[2] == int((~(t.c_total_valid[kr] & t.c_covered_valid[kr])).sum())
        got = sh._pv[:n].cpu().numpy()
        ok = t.c_total_valid[kr] & t.c_covered_valid[kr]
        exp = t.c_covered[kr].astype(np.float64) / t.c_total[kr].astype(np.float64) * 100
        assert np.array_equal(got[ok], exp[ok]) and np.isnan(got[~ok]).all()
        sh._piece(E.FZ_PIECE_RQ4B)
        m4 = (t.c_project == p) & t.c_coverage_valid & (t.c_coverage > 0) & (t.c_date < LIMIT_US)
        r4 = np.nonzero(m4)[0]
        r4 = r4[np.argsort(t.c_date[r4], kind="stable")]
        assert int(sh._pc[0]) == len(r4) and np.array_equal(sh._pv[:len(r4)].cpu().numpy(), t.c_coverage[r4])
    # eligibility counts and an override: every analysis reads the overridden set
    q = t.c_coverage_valid & (t.c_coverage > 0) & (t.c_date < LIMIT_US)
    cnt = np.bincount(t.c_project[q].astype(np.int64), minlength=len(t.projects))
    ctl = par.GpuEligibility(eng)
    ids = np.arange(len(t.projects))
    assert np.array_equal(ctl.elig_counts(ids).cpu().numpy(), cnt)
    elig = orc.eligible_projects(t)
    flip = np.array([int(elig[0]), int(np.nonzero(cnt < 365)[0][0])], np.int64)
    ctl.set_eligible(flip, torch.tensor([0, 1], dtype=torch.uint8, device=eng.dev))
    r1 = compute.rq1(eng)
    want = np.array(sorted((set(elig.tolist()) - {int(flip[0])}) | {int(flip[1])}))
    assert np.array_equal(r1.eligible, want)
    r2 = compute.rq2_count(eng)
    assert np.array_equal(r2.eligible, want)
    eng.build_store()  # a rebuild recomputes the set
    assert np.array_equal(compute.rq1(eng).eligible, elig)
