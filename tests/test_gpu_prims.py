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


def _np_describe(a):
    return dict(count=len(a), n_pos=int((a > 0).sum()), n_zero=int((a == 0).sum()), n_neg=int((a < 0).sum()),
                mean=float(np.mean(a)), median=float(np.median(a)), std=float(np.std(a)), min=float(a.min()),
                max=float(a.max()), q1=float(np.percentile(a, 25)), q3=float(np.percentile(a, 75)))


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (5, 2), (1000, 3), (777_777, 4)])
def test_describe_matches_numpy(engine, n, seed):
    torch = engine.torch
    rng = np.random.default_rng(seed)
    a = np.round(rng.normal(0, 3, size=n), 2)                     # ties, zeros, both signs
    a[: n // 7] = 0.0
    d = engine.describe(torch.from_numpy(a).to(engine.dev))
    ours = {k: getattr(d, k) for k in _np_describe(a)}
    assert_same(ours, _np_describe(a))
