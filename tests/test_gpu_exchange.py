"""The sharded path's session exchange (tse_amd/parallel.py exchange_grouped): fz_runs_merge (the
receive side - R runs of segment-grouped values interleaved segment by segment, sources in rank
order) and the grouped per-session statistics fz_rq2_session_stats_grouped /
fz_rq4b_session_stats_grouped (values already grouped by session / (session, group) segment: no
per-value ids, no sort).  Checkers: parallel.merge_runs_torch (itself checked against a loop here,
on the CPU), the id-based entry points on the same pools in the same order (bit-identical), numpy
percentiles and oracle/rq_oracle.rq4b_session_stats."""
import numpy as np
import pytest
import torch

from gpu_common import assert_same
from test_gpu_segsort import LENGTHS, KINDS, _segments


def _runs(seed, R, S, zero_frac=0.3, hi=40):
    rng = np.random.default_rng(seed)
    sizes = rng.integers(0, hi, (R, S))
    sizes[rng.random((R, S)) < zero_frac] = 0
    return sizes.astype(np.int64), rng.normal(50.0, 20.0, int(sizes.sum()))


def _merge_loop(vals, sizes):
    R, S = sizes.shape
    st = np.concatenate([[0], np.cumsum(sizes.reshape(-1))])
    out = []
    for s in range(S):
        for r in range(R):
            q = r * S + s
            out.append(vals[st[q]:st[q + 1]])
    offs = np.concatenate([[0], np.cumsum(sizes.sum(0))]).astype(np.int64)
    return (np.concatenate(out) if out else np.zeros(0)), offs


@pytest.mark.parametrize("R,S", [(1, 5), (2, 7), (3, 1), (8, 64)])
def test_merge_runs_torch_matches_loop(R, S):
    from tse_amd.parallel import merge_runs_torch
    sizes, vals = _runs(R * 100 + S, R, S)
    got, offs = merge_runs_torch(torch.from_numpy(vals), torch.from_numpy(sizes))
    want, woffs = _merge_loop(vals, sizes)
    assert np.array_equal(got.numpy(), want) and np.array_equal(offs.numpy(), woffs)


@pytest.mark.gpu
@pytest.mark.parametrize("R,S,hi", [(1, 1, 10), (1, 300, 40), (2, 3000, 20), (3, 17, 5000), (8, 2500, 30),
                                    (16, 40, 200), (4, 0, 1)])
def test_runs_merge_matches(engine, R, S, hi):
    from tse_amd.parallel import gpu_merge_runs
    sizes, vals = _runs(R * 7 + S, R, S, hi=hi)
    got, offs = gpu_merge_runs(engine, torch.from_numpy(vals).to(engine.dev), torch.from_numpy(sizes).to(engine.dev))
    want, woffs = _merge_loop(vals, sizes)
    assert np.array_equal(offs.cpu().numpy(), woffs)
    assert np.array_equal(got.cpu().numpy().view(np.int64), want.view(np.int64))  # bit patterns


@pytest.mark.gpu
@pytest.mark.parametrize("lengths", [LENGTHS, [0, 5, 0, 1, 100, 0], [3] * 5000])
def test_grouped_session_stats_match_id_path(engine, lengths):
    """Grouped statistics == the id-based entry point on the same pools in the same order (every
    output bit-identical: the mean sums in the same order), and np.percentile."""
    from tse_amd.parallel import gpu_session_stats, gpu_session_stats_grouped
    segs = _segments(len(lengths), lengths, KINDS)
    vals = np.concatenate(segs)
    S = len(segs)
    offs = np.concatenate([[0], np.cumsum([len(s) for s in segs])]).astype(np.int64)
    sids = np.repeat(np.arange(S, dtype=np.int64), [len(s) for s in segs])
    dv = torch.from_numpy(vals).to(engine.dev)
    mx = max(max(len(s) for s in segs), 1)
    g = gpu_session_stats_grouped(engine, dv, torch.from_numpy(offs).to(engine.dev), S, mx)
    r = gpu_session_stats(engine, dv, torch.from_numpy(sids).to(engine.dev), S, mx)
    for k in ("average", "median", "percentiles", "ge100"):
        a, b = g[k].cpu().numpy(), r[k].cpu().numpy()
        n = {"average": S, "median": S, "percentiles": 5 * S, "ge100": 1}[k]
        assert np.array_equal(a[:n].view(np.int64), b[:n].view(np.int64)), k
    pct = g["percentiles"][:5 * S].cpu().numpy().reshape(S, 5)
    for i, s in enumerate(segs):
        if len(s):
            assert np.array_equal(pct[i], np.percentile(s, [5, 25, 50, 75, 95])), (i, len(s))
    assert int(g["ge100"][0]) == sum(len(s) >= 100 for s in segs)


@pytest.mark.gpu
@pytest.mark.parametrize("sizes", [[(3, 4), (0, 0), (7, 7), (120, 90), (1, 0), (0, 9)],
                                   [(200, 150)] * 40 + [(6, 5)] * 300,
                                   [(20_000, 16_000), (5, 30_000), (0, 2)],
                                   [(6000, 5000), (3000, 3000), (7, 9)]])
def test_rq4b_grouped_matches_oracle(engine, sizes):
    from oracle import rq_oracle as orc
    from tse_amd.parallel import gpu_rq4b_session_stats_grouped
    rng = np.random.default_rng(len(sizes))
    s2, s1, vals, seg = [], [], [], []
    for a, b in sizes:
        va = np.round(rng.uniform(0, 100, a) * 4) / 4  # ties
        vb = rng.uniform(0, 100, b)
        s2.append(va.tolist())
        s1.append(vb.tolist())
        vals += [va, vb]
        seg += [a, b]
    offs2 = np.concatenate([[0], np.cumsum(seg)]).astype(np.int64)
    S = len(sizes)
    got = gpu_rq4b_session_stats_grouped(engine, torch.from_numpy(np.concatenate(vals)).to(engine.dev),
                                         torch.from_numpy(offs2).to(engine.dev), S,
                                         max(a + b for a, b in sizes))  # (bound of a whole session)
    c2, c1, q2, q1, pb = orc.rq4b_session_stats(s2, s1)
    assert_same(got["c2"][:S].cpu().numpy(), c2, path="c2")
    assert_same(got["c1"][:S].cpu().numpy(), c1, path="c1")
    assert_same(got["g2_q"][:3 * S].cpu().numpy().reshape(S, 3), q2, path="g2_q")
    assert_same(got["g1_q"][:3 * S].cpu().numpy().reshape(S, 3), q1, path="g1_q")
    assert_same(got["p_bm"][:S].cpu().numpy(), pb, path="p_bm")
