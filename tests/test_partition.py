"""parallel.partition_rows (shard_bounds): contiguous project ranges, one per rank, with the
smallest possible largest shard - checked against exhaustive search on small random row counts
and on config 5's Zipf sizes (the 20.8 M-row giant)."""
import itertools

import numpy as np
import pytest

from tse_amd import parallel as par
from tse_amd import synth


def _check(rows, world, bounds):
    P = len(rows)
    assert len(bounds) == world
    assert bounds[0][0] == 0 and bounds[-1][1] == P
    for (a, b), (c, d) in zip(bounds, bounds[1:]):
        assert b == c and a <= b
    return max(int(np.sum(rows[a:b])) for a, b in bounds)


def _best(rows, world):
    P = len(rows)
    best = None
    for cuts in itertools.combinations(range(P + 1), world - 1):
        edges = (0,) + cuts + (P,)
        if any(edges[i] > edges[i + 1] for i in range(world)):
            continue
        m = max(int(np.sum(rows[edges[i]:edges[i + 1]])) for i in range(world))
        best = m if best is None else min(best, m)
    return best


@pytest.mark.parametrize("seed", range(12))
def test_partition_is_min_max(seed):
    rng = np.random.default_rng(seed)
    P = int(rng.integers(1, 9))
    rows = rng.integers(0, 50, P) * (rng.random(P) < 0.8) + (rng.random(P) < 0.2) * 400
    for world in (1, 2, 3, 4):
        got = _check(rows, world, par.partition_rows(rows, world))
        assert got == _best(rows, world), (rows, world)


def test_partition_zipf_giant():
    cfg = synth.config("c5")
    rng = np.random.default_rng(cfg.seed)
    P = cfg.n_projects
    rng.integers(0, cfg.start_span_days + 1, size=P)
    w = 1.0 / np.arange(1, P + 1) ** cfg.zipf_s
    rng.shuffle(w)
    rows = np.maximum(1, (w / w.sum() * cfg.len_mean_days * P)).astype(np.int64)
    giant = int(rows.max())
    for world, cap in ((2, 50_030_117), (4, 29_148_845), (8, giant)):
        assert _check(rows, world, par.partition_rows(rows, world)) <= cap


def test_partition_more_ranks_than_projects():
    b = par.partition_rows(np.array([5, 1, 1]), 6)
    _check(np.array([5, 1, 1]), 6, b)
    assert par.partition_rows(np.zeros(0, np.int64), 3) == [(0, 0)] * 3
