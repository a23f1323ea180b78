"""Config 4: rank-statistics stress.  Long series (1e5 - 1e6 points) with heavy
ties (256 levels) and a monotone + noise variant through the trend tests (A8 Shapiro-Wilk above
scipy's n = 5000 warning, A9 Spearman vs index), two samples of >= 1e5 values through the rank-sum
tests (A23 Mann-Whitney / Cliff / Brunner-Munzel / Levene) and per-session Brunner-Munzel with
sessions of >= 1e5 values per group (A21).  Checker: the CPU oracle (scipy, as the reference calls
it); tolerance 1e-9 relative (north star)."""
import numpy as np
import pytest

import tse_amd.synth as synth
from gpu_common import assert_same
from oracle import rq_oracle as orc

pytestmark = pytest.mark.gpu

LEVELS = 255


def _ties(rng, n):
    return np.round(rng.uniform(0, 1, n) * LEVELS) / LEVELS * 100.0


def _trend(rng, n):
    return np.round(np.clip(np.linspace(0.1, 0.9, n) + rng.normal(0, 0.05, n), 0, 1) * LEVELS) / LEVELS * 100.0


def _dev(engine, a):
    return engine.torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(engine.dev)


@pytest.mark.parametrize("n", [100_000, 300_000, 1_000_000])
@pytest.mark.parametrize("kind", ["ties", "trend"])
def test_series_tests_long(engine, n, kind):
    from tse_amd.parallel import gpu_series_tests
    rng = np.random.default_rng(n + (kind == "trend"))
    x = (_ties if kind == "ties" else _trend)(rng, n)
    assert len(np.unique(x)) <= LEVELS + 1
    got = tuple(float(v) for v in gpu_series_tests(engine, _dev(engine, x)).cpu())
    assert_same(got, orc.series_tests(x), path=f"series[{kind},{n}]")


@pytest.mark.parametrize("nx,ny,shift", [(100_000, 130_000, 0.0), (250_000, 100_000, 0.4)])
def test_two_sample_large(engine, nx, ny, shift):
    import ctypes as C
    from tse_amd import engine as E
    rng = np.random.default_rng(nx + ny)
    x, y = _ties(rng, nx), np.minimum(_ties(rng, ny) + shift, 100.0)
    out = engine.torch.full((E.FZ_RQ4B_NTESTS,), float("nan"), dtype=engine.torch.float64, device=engine.dev)
    dx, dy = _dev(engine, x), _dev(engine, y)
    E._check(engine.lib, engine.lib.fz_two_sample_tests(engine.ctx, C.c_void_p(dx.data_ptr()), nx,
                                                        C.c_void_p(dy.data_ptr()), ny, C.c_void_p(out.data_ptr())))
    got = out.cpu().numpy()
    mwu_p, cliff, bm, lv = orc.rq4b_init_tests(x, y)
    assert_same([got[E.RQ4B_MWU_P], got[E.RQ4B_CLIFF], got[E.RQ4B_BM_STAT], got[E.RQ4B_BM_P],
                 got[E.RQ4B_LEVENE_W], got[E.RQ4B_LEVENE_P]],
                [mwu_p, cliff, bm[0], bm[1], lv[0], lv[1]], path="two_sample")


@pytest.mark.parametrize("n", [1, 2, 3, 7, 100, 1000, 4096])
@pytest.mark.parametrize("kind", ["ties", "trend", "const"])
def test_series_tests_small(engine, n, kind):
    """Series of at most 4096 values: the one-workgroup kernel (LDS sort, Spearman, Shapiro-Wilk)."""
    from tse_amd.parallel import gpu_series_tests
    rng = np.random.default_rng(n * 3 + len(kind))
    x = np.full(n, 42.5) if kind == "const" else (_ties if kind == "ties" else _trend)(rng, n)
    got = tuple(float(v) for v in gpu_series_tests(engine, _dev(engine, x)).cpu())
    with np.errstate(all="ignore"):
        ref = orc.series_tests(x)
    assert_same(got, ref, path=f"series[{kind},{n}]")


@pytest.mark.parametrize("nx,ny,kind", [(5, 7, "cont"), (8, 300, "cont"), (3, 4, "ties"), (1000, 990, "ties"),
                                         (4096, 4096, "ties"), (4096, 17, "cont"), (2, 2, "cont"), (1, 5, "ties"),
                                         (4097, 100, "ties")])
def test_two_sample_small(engine, nx, ny, kind):
    """The one-workgroup two-sample kernel (both samples <= 4096 values: config 2's per-project
    initial coverages) and, past 4096, the multi-launch path: the exact Mann-Whitney null
    distribution (min(nx, ny) <= 8, no ties), heavy ties, one-value samples."""
    import ctypes as C
    from tse_amd import engine as E
    rng = np.random.default_rng(nx * 7 + ny)
    gen = (lambda n: rng.normal(50, 10, n)) if kind == "cont" else (lambda n: _ties(rng, n))
    x, y = gen(nx), gen(ny) + 0.3
    out = engine.torch.full((E.FZ_RQ4B_NTESTS,), float("nan"), dtype=engine.torch.float64, device=engine.dev)
    dx, dy = _dev(engine, x), _dev(engine, y)
    E._check(engine.lib, engine.lib.fz_two_sample_tests(engine.ctx, C.c_void_p(dx.data_ptr()), nx,
                                                        C.c_void_p(dy.data_ptr()), ny, C.c_void_p(out.data_ptr())))
    got = out.cpu().numpy()
    with np.errstate(all="ignore"):
        mwu_p, cliff, bm, lv = orc.rq4b_init_tests(x, y)
    assert_same([got[E.RQ4B_MWU_P], got[E.RQ4B_CLIFF], got[E.RQ4B_BM_STAT], got[E.RQ4B_BM_P],
                 got[E.RQ4B_LEVENE_W], got[E.RQ4B_LEVENE_P]],
                [mwu_p, cliff, bm[0], bm[1], lv[0], lv[1]], path=f"two_sample[{nx},{ny},{kind}]")


def test_session_bm_large(engine):
    """fz_rq4b_session_stats with sessions of >= 1e5 values per group (plus small / one-sided ones)."""
    from tse_amd.parallel import gpu_rq4b_session_stats
    rng = np.random.default_rng(4)
    sizes = [(100_000, 120_000), (150_000, 7), (4, 100_000), (0, 3), (60_000, 60_000)]
    s2, s1, vals, sids, grp = [], [], [], [], []
    for i, (a, b) in enumerate(sizes):
        va, vb = _ties(rng, a), _trend(rng, b)
        s2.append(va.tolist())
        s1.append(vb.tolist())
        both = np.concatenate([va, vb])
        g = np.concatenate([np.zeros(a, np.uint8), np.ones(b, np.uint8)])
        p = rng.permutation(len(both))  # sessions arrive interleaved, in any order
        vals.append(both[p])
        grp.append(g[p])
        sids.append(np.full(len(both), i, np.int64))
    torch = engine.torch
    dv = _dev(engine, np.concatenate(vals))
    dsid = torch.from_numpy(np.concatenate(sids)).to(engine.dev)
    dg = torch.from_numpy(np.concatenate(grp)).to(engine.dev)
    got = gpu_rq4b_session_stats(engine, dv, dsid, dg, len(sizes), max(max(a, b) for a, b in sizes))
    c2, c1, q2, q1, pb = orc.rq4b_session_stats(s2, s1)
    S = len(sizes)
    assert_same(got["c2"][:S].cpu().numpy(), c2, path="c2")
    assert_same(got["c1"][:S].cpu().numpy(), c1, path="c1")
    assert_same(got["g2_q"][:3 * S].cpu().numpy().reshape(S, 3), q2, path="g2_q")
    assert_same(got["g1_q"][:3 * S].cpu().numpy().reshape(S, 3), q1, path="g1_q")
    assert_same(got["p_bm"][:S].cpu().numpy(), pb, path="p_bm")


def test_config4_shape_all_scripts(engine):
    """The c4 table shape (scaled: 3 series, 30k-200k points) through all six analyses."""
    from test_gpu_scale import _check_all
    t = synth.generate(synth.config("c4", n_projects=3, lengths=(100_000, 30_000, 200_000)))
    _check_all(engine, t)
