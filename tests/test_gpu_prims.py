"""Kernel-level GPU tests of the libfz primitives against numpy (bit-exact for sort/order,
1e-9 relative for the describe statistics)."""
import numpy as np
import pytest

from gpu_common import assert_same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,bits,seed", [(0, 64, 0), (1, 64, 1), (4095, 12, 2), (4097, 64, 3),
                                         (100_003, 40, 4), (1_000_000, 59, 5), (300_000, 3, 6)])
def test_radix_sort_stable(engine, n, bits, seed):
    torch = engine.torch
    rng = np.random.default_rng(seed)
    hi = (1 << bits) if bits < 64 else None
    k = rng.integers(0, hi, size=n, dtype=np.uint64) if hi else rng.integers(0, 2**63, size=n, dtype=np.uint64) * 2 + 1
    if n > 10:
        k[: n // 10] = k[n // 2]                                  # heavy ties: stability matters
    v = np.arange(n, dtype=np.uint32)
    dk = torch.from_numpy(k.view(np.int64)).to(engine.dev)
    dv = torch.from_numpy(v.view(np.int32)).to(engine.dev)
    engine.radix_sort(dk, dv, bits)
    engine.synchronize()
    order = np.argsort(k, kind="stable")
    assert np.array_equal(dk.cpu().numpy().view(np.uint64), k[order])
    assert np.array_equal(dv.cpu().numpy().view(np.uint32), v[order])


def _f64_keys(x):
    u = x.view(np.uint64)
    return np.where(u >> np.uint64(63) != 0, ~u, u | np.uint64(1 << 63))


def _sort_input(kind, n, rng):
    if kind == "rq3like":  # percentage-point changes: zeros, ties, rounding noise around them
        a = np.where(rng.random(n) < 0.4, 0.0, (rng.integers(0, 400, n) + 1) / rng.integers(300, 2000, n) * 100.0)
        return np.where(rng.random(n) < 0.5, -a, a) + np.where(rng.random(n) < 0.1, 1e-15, 0.0)
    if kind == "normal":
        return np.round(rng.normal(0, 3, size=n), 2)
    if kind == "allsame":
        return np.full(n, 2.5)
    if kind == "sorted":
        return np.sort(rng.normal(size=n))
    if kind == "reverse":
        return np.sort(rng.normal(size=n))[::-1].copy()
    if kind == "special":  # NaN last, -0.0 before +0.0, infinities at the ends
        a = rng.normal(size=n)
        k = rng.integers(0, 6, size=n)
        a[k == 0] = np.nan
        a[k == 1] = -0.0
        a[k == 2] = 0.0
        a[k == 3] = np.inf
        a[k == 4] = -np.inf
        return a
    if kind in ("cluster", "cluster_tied"):  # the strided samples spread, everything else in one range
        # bucket far past the LDS capacity: the run / merge path
        a = 0.5 + np.arange(n) * 1e-12 if kind == "cluster" else np.full(n, 0.5)
        sp = (np.arange(4096, dtype=np.int64) * n) // 4096
        a[sp] = rng.uniform(-1e6, 1e6, size=len(sp))
        return a
    if kind.startswith("tie_"):  # runs of one value that no strided sample hits, inside one range
        # bucket of <= 12,288 values, past the bucket's comparison-ranking thresholds (FZ_SS_SKEW /
        # FZ_SS_WORK): the LDS radix sort of the bucket, stable for the ties
        a = rng.normal(size=n)
        sp = (np.arange(4096, dtype=np.int64) * n) // 4096
        free = np.setdiff1d(np.arange(n), sp)
        runs = {"tie_rank": [(0.1234, 1000), (0.12345, 1000)], "tie_fallback": [(0.1234, 3000)],
                "tie_work": [(0.1234, 1500), (0.12345, 1500), (0.123456, 1500)]}[kind]
        at = rng.permutation(free)
        o = 0
        for v, m in runs:
            a[at[o:o + m]] = v
            o += m
        return a
    raise ValueError(kind)


@pytest.mark.parametrize("kind,n,seed", [
    ("tie_rank", 100_000, 12), ("tie_fallback", 100_000, 13), ("tie_work", 100_000, 14),
    ("rq3like", 16_385, 0), ("rq3like", 790_000, 1), ("rq3like", 1_310_720, 2), ("rq3like", 2_000_000, 3),
    ("normal", 100_003, 4), ("allsame", 50_000, 5), ("sorted", 300_000, 6), ("reverse", 300_000, 7),
    ("special", 200_000, 8), ("cluster", 100_003, 9), ("cluster_tied", 60_000, 10), ("rq3like", 5, 11)])
def test_sort_f64_stable(engine, kind, n, seed):
    """fz_sort_f64 (the single-segment sort of RQ3's union: splitter buckets + one scatter pass +
    LDS bucket sorts up to 1.3 M values, the LSD radix sort beyond) = numpy's stable argsort of the
    order-preserving keys, bit for bit."""
    torch = engine.torch
    x = _sort_input(kind, n, np.random.default_rng(seed))
    dx = torch.from_numpy(x).to(engine.dev)
    val, pos = engine.sort_f64(dx)
    engine.synchronize()
    order = np.argsort(_f64_keys(x), kind="stable")
    assert np.array_equal(pos.cpu().numpy(), order.astype(np.int32))
    assert np.array_equal(val.cpu().numpy().view(np.uint64), x[order].view(np.uint64))


def _np_describe(a):
    return dict(count=len(a), n_pos=int((a > 0).sum()), n_zero=int((a == 0).sum()), n_neg=int((a < 0).sum()),
                mean=float(np.mean(a)), median=float(np.median(a)), std=float(np.std(a)), min=float(a.min()),
                max=float(a.max()), q1=float(np.percentile(a, 25)), q3=float(np.percentile(a, 75)))


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (5, 2), (1000, 3), (777_777, 4),
                                    # k_describe_sel's network classes: 512 / 1,024 / 2,048 / 4,096 / 8,192 keys
                                    (64, 5), (511, 6), (512, 7), (513, 8), (1024, 9), (1025, 10), (2048, 11),
                                    (2049, 12), (4096, 13), (4097, 14), (8192, 15), (8193, 16)])
def test_describe_matches_numpy(engine, n, seed):
    torch = engine.torch
    rng = np.random.default_rng(seed)
    a = np.round(rng.normal(0, 3, size=n), 2)                     # ties, zeros, both signs
    a[: n // 7] = 0.0
    d = engine.describe(torch.from_numpy(a).to(engine.dev))
    ours = {k: getattr(d, k) for k in _np_describe(a)}
    assert_same(ours, _np_describe(a))


def _gen(kind, n, rng):
    if kind == "ints":       # RQ3's total-line differences: few hundred distinct integers, heavy ties
        return np.round(rng.normal(0, 60, size=n)).astype(np.float64)
    if kind == "const":
        return np.full(n, 3.25)
    if kind == "twovals":
        return np.where(rng.random(n) < 0.5, -1.0, 7.0)
    if kind == "wide":       # magnitudes from 1e-150 to 1e150 (key buckets span whole binades)
        return rng.choice([-1.0, 1.0], n) * 10.0 ** rng.uniform(-150, 150, n)
    if kind == "cluster":    # one dense cluster plus far outliers (re-histogrammed intervals)
        a = 1.0 + rng.normal(0, 1e-12, n)
        a[: max(1, n // 50)] = rng.uniform(-1e6, 1e6, max(1, n // 50))
        return a
    if kind == "pos":        # no negatives, zeros: the smallest non-zero value is not the minimum
        a = np.round(rng.exponential(5, n), 1)
        return a
    raise ValueError(kind)


@pytest.mark.parametrize("kind", ["ints", "const", "twovals", "wide", "cluster", "pos"])
@pytest.mark.parametrize("n", [63, 9022, 12288, 12289, 65536])
def test_describe_selection_shapes(engine, kind, n):
    """k_describe_sel's selection paths: samples staged in LDS (<= 12288) or re-read, key buckets
    holding one value (ties), narrowed intervals of several targets at once, the smallest non-zero."""
    torch = engine.torch
    rng = np.random.default_rng(n + len(kind))
    a = _gen(kind, n, rng)
    d = engine.describe(torch.from_numpy(a).to(engine.dev))
    ours = {k: getattr(d, k) for k in _np_describe(a)}
    assert_same(ours, _np_describe(a))
    nz = a[a != 0]
    assert bool(d.has_nonzero) == (len(nz) > 0)
    if len(nz):
        assert d.min_nonzero == nz.min()
