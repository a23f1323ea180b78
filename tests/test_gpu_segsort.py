"""Segmented value sort (csrc/fz_series.hip seg_sort_f64: value bucket sort per length class, its
in-workgroup bitonic fallback for skewed segments, the merge sort for flagged / > 16384-value
segments, and the one-wave / one-thread sorts of the many-segments list path) through the two C-ABI
entry points that consume it: fz_rq2_session_stats (per-segment median + np.percentile 5/25/50/75/95
of the sorted values, rq2_coverage_count.py:285-361) and fz_spearman_index_seg (tie-aware ranks vs
position: scipy.stats.spearmanr(range(n), x), rq2_coverage_count.py:305-322).  Segment lengths sit
on every class boundary; value kinds: spread (bucket path), heavy ties and one dominant value
(skew fallback), constant, signed values with +-0.0.  Checker: numpy / scipy; bit-exact for the
order statistics, 1e-9 relative for rho / p."""
import math

import numpy as np
import pytest
from scipy import stats

pytestmark = pytest.mark.gpu

LENGTHS = [1, 2, 3, 7, 8, 9, 63, 64, 65, 500, 1023, 1024, 1025, 2047, 2048, 2049, 4095, 4096, 4097, 10_000,
           16_384, 16_385, 40_000]
KINDS = ["spread", "ties", "dominant", "constant", "signed"]


def _values(rng, kind, n):
    if kind == "spread":
        return rng.uniform(10.0, 60.0, n)
    if kind == "ties":
        return np.round(rng.uniform(0, 1, n) * 7) / 7 * 100.0
    if kind == "dominant":  # one value holds most of the segment: its bucket overflows
        x = np.full(n, 42.5)
        k = rng.random(n) < 0.2
        x[k] = rng.uniform(0, 100, int(k.sum()))
        return x
    if kind == "constant":
        return np.full(n, 3.25)
    if kind == "cluster":  # most values inside one tiny key interval: the selection refines its bucket
        x = 50.0 + rng.uniform(0, 1e-9, n)
        k = rng.random(n) < 0.1
        x[k] = rng.uniform(0, 100, int(k.sum()))
        return x
    if kind == "powers":  # values spread over many binades (keys far from linear in the value)
        return np.ldexp(1.0, rng.integers(-60, 60, n)) * rng.choice([1.0, 1.5], n)
    x = rng.normal(0, 10, n)  # signed, with both zeros
    x[rng.random(n) < 0.05] = 0.0
    x[rng.random(n) < 0.05] = -0.0
    return x


def _segments(seed, lengths, kinds):
    rng = np.random.default_rng(seed)
    return [_values(rng, kinds[i % len(kinds)], n) for i, n in enumerate(lengths)]


def _session_stats(engine, segs):
    from tse_amd.parallel import gpu_session_stats
    torch = engine.torch
    vals = np.concatenate(segs)
    sids = np.concatenate([np.full(len(s), i, np.int64) for i, s in enumerate(segs)])
    rng = np.random.default_rng(len(vals))
    p = rng.permutation(len(vals))  # (session, value) pairs arrive in any order
    got = gpu_session_stats(engine, torch.from_numpy(vals[p]).to(engine.dev), torch.from_numpy(sids[p]).to(engine.dev),
                            len(segs), max(len(s) for s in segs))
    S = len(segs)
    med = got["median"][:S].cpu().numpy()
    avg = got["average"][:S].cpu().numpy()
    pct = got["percentiles"][:5 * S].cpu().numpy().reshape(S, 5)
    assert int(got["ge100"][0]) == sum(len(s) >= 100 for s in segs)
    for i, s in enumerate(segs):
        if len(s) == 0:  # an empty session: every statistic NaN
            assert np.isnan(med[i]) and np.isnan(avg[i]) and np.isnan(pct[i]).all(), i
            continue
        # statistics.mean: the exactly rounded mean (double-double sum), within 1e-12 relative
        want_mean = math.fsum(s) / len(s)
        assert abs(avg[i] - want_mean) <= 1e-12 * abs(want_mean) + 1e-300, (i, len(s), avg[i], want_mean)
        # the per-session order of equal values follows the arrival order: compare as multisets
        assert med[i] == np.median(s) or (np.isnan(med[i]) and np.isnan(np.median(s))), (i, len(s))
        want = np.percentile(s, [5, 25, 50, 75, 95])
        assert np.array_equal(pct[i], want), (i, len(s), pct[i], want)


def _spearman(engine, segs):
    from tse_amd.parallel import gpu_spearman_prefix  # noqa: F401  (module import: engine bindings)
    import ctypes as C
    from tse_amd import engine as E
    torch = engine.torch
    x = torch.from_numpy(np.concatenate(segs)).to(engine.dev)
    offs = torch.from_numpy(np.concatenate([[0], np.cumsum([len(s) for s in segs])]).astype(np.int64)).to(engine.dev)
    S = len(segs)
    out = torch.empty(2 * S, dtype=torch.float64, device=engine.dev)
    E._check(engine.lib, engine.lib.fz_spearman_index_seg(engine.ctx, C.c_void_p(x.data_ptr()), x.numel(),
                                                         C.c_void_p(offs.data_ptr()), S, max(len(s) for s in segs),
                                                         C.c_void_p(out.data_ptr()), C.c_void_p(out[S:].data_ptr())))
    got = out.cpu().numpy()
    import warnings
    for i, s in enumerate(segs):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            r = stats.spearmanr(range(len(s)), s) if len(s) >= 2 else (float("nan"), float("nan"))
        for a, b, what in ((got[i], float(r[0]), "rho"), (got[S + i], float(r[1]), "p")):
            if np.isnan(b):
                assert np.isnan(a), (i, len(s), what, a)
            else:
                assert abs(a - b) <= 1e-9 * max(abs(b), 1e-300) + 1e-15, (i, len(s), what, a, b)


@pytest.mark.parametrize("kind", KINDS)
def test_session_order_stats_every_class(engine, kind):
    _session_stats(engine, _segments(11 + KINDS.index(kind), LENGTHS, [kind]))


def test_session_order_stats_mixed(engine):
    _session_stats(engine, _segments(5, LENGTHS * 2, KINDS))


def test_spearman_every_class(engine):
    _spearman(engine, _segments(7, LENGTHS, ["spread", "ties", "dominant", "signed"]))


def test_many_segments_lists(engine):
    """> 16384 segments: the size-class list path (one thread <= 8, one wave <= 64, buckets above)."""
    rng = np.random.default_rng(3)
    lengths = rng.choice([1, 3, 8, 9, 40, 64, 65, 300, 1500, 3000], size=20_000,
                         p=[.2, .2, .1, .1, .2, .05, .05, .06, .03, .01]).tolist() + [5000, 17_000]
    segs = _segments(9, lengths, KINDS)
    _session_stats(engine, segs)
    _spearman(engine, segs[:2000] + segs[-2:])


@pytest.mark.parametrize("kinds", [["spread"], ["ties", "dominant", "spread"], ["signed", "powers"]])
def test_long_segments_radix_path(engine, kinds):
    """Segments above 2^20 values among short and flagged ones (longer than 16384, or skewed): the
    long-segment sort (the merge rounds; radix_big_segments in an FZ_BIG_RADIX=1 build) - order
    statistics and Spearman vs numpy / scipy."""
    lengths = [1_500_000, 5, 20_000, 16_385, 3000, 0, 1_100_000, 40_000, 64]
    segs = _segments(31 + len(kinds), lengths, kinds)
    _session_stats(engine, segs)
    _spearman(engine, segs)


# The per-session statistics by SELECTION (fz_series.hip seg_qstats: no sorted copy) run when no
# segment exceeds 16384 values (a session holds one value per project); the lists above reach 40000
# and take the sort path.  Same checks against numpy on lengths up to the selection's bound.
QS_LENGTHS = [n for n in LENGTHS if n <= 16_384]
QS_KINDS = KINDS + ["cluster", "powers"]


@pytest.mark.parametrize("kind", QS_KINDS)
def test_session_order_stats_selection(engine, kind):
    _session_stats(engine, _segments(21 + QS_KINDS.index(kind), QS_LENGTHS, [kind]))


def test_session_order_stats_selection_mixed(engine):
    _session_stats(engine, _segments(6, QS_LENGTHS * 2 + [0, 0, 5], QS_KINDS))


def test_session_order_stats_selection_many_segments(engine):
    """> 16384 segments, sizes in any order (the size-class lists of the workgroup classes), empty
    segments between them."""
    rng = np.random.default_rng(4)
    lengths = rng.choice([0, 1, 3, 8, 9, 40, 64, 65, 300, 1025, 3000, 9000], size=20_000,
                         p=[.05, .15, .2, .1, .1, .2, .05, .05, .06, .02, .01, .01]).tolist() + [16_384]
    _session_stats(engine, _segments(10, lengths, QS_KINDS))
