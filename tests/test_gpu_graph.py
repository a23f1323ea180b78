"""HIP graphs (fz_capture_begin / fz_capture_end / fz_graph_launch, Engine.record): the six
analyses recorded once - some on a child context, the rest on the engine's own context after its
store build - and replayed over several store rebuilds give exactly the direct calls' results
(every output buffer is cleared before each replay, so the replay really wrote them); direct calls
on both contexts after the replays are still right (the look-back ticket / epoch state and the
radix digit-total buffers are restored by every replay).  Checker: the direct (already oracle-
tested) calls of the same case."""
import pytest

import goldens
from gpu_common import assert_same
from tse_amd.rq import compute

pytestmark = pytest.mark.gpu

DIRECT = {"rq1": compute.rq1, "rq2_count": compute.rq2_count, "rq2_add": compute.rq2_add,
          "rq3": compute.rq3, "rq4a": compute.rq4a, "rq4b": compute.rq4b}
PARTS = {"rq1": (compute.RQ1Buffers, compute.rq1_launch, compute.rq1_collect),
         "rq2_count": (compute.rq2_count_buffers, compute.rq2_count_launch, compute.rq2_count_collect),
         "rq2_add": (compute.rq2_add_buffers, compute.rq2_add_launch, compute.rq2_add_collect),
         "rq3": (compute.rq3_buffers, compute.rq3_launch, compute.rq3_collect),
         "rq4a": (compute.rq4a_buffers, compute.rq4a_launch, compute.rq4a_collect),
         "rq4b": (compute.rq4b_buffers, compute.rq4b_launch, compute.rq4b_collect)}
ON_CHILD = ("rq3", "rq4b")
ON_PARENT = ("rq1", "rq2_count", "rq2_add", "rq4a")


def _clear(b, torch):
    for v in vars(b).values():
        if isinstance(v, torch.Tensor):
            v.zero_()


@pytest.mark.parametrize("case", goldens.CASES)
def test_graph_replay_matches_direct(engine_for, case):
    eng = engine_for(case)
    torch = eng.torch
    want = {k: f(eng) for k, f in DIRECT.items()}
    ch = eng.child()
    try:
        bufs = {k: mk(eng) for k, (mk, _, _) in PARTS.items()}
        ch.follow_parent()
        for k in ON_CHILD:  # warm the child context (its scratch reaches full size)
            PARTS[k][1](ch, bufs[k])
        eng.join_children()
        torch.cuda.synchronize()
        g_child = ch.record(lambda e: [PARTS[k][1](e, bufs[k]) for k in ON_CHILD])
        g_parent = eng.record(lambda e: [PARTS[k][1](e, bufs[k]) for k in ON_PARENT])
        try:
            for _ in range(3):
                for b in bufs.values():
                    _clear(b, torch)
                eng.join_children()
                eng.build_store()
                ch.follow_parent()
                g_child.launch()
                g_parent.launch()
                eng.join_children()
                torch.cuda.synchronize()
                for k, (_, _, collect) in PARTS.items():
                    assert_same(collect(eng, bufs[k]), want[k], f"{k} (replay)")
        finally:
            g_child.close()
            g_parent.close()
        # direct calls after replays, on both contexts
        with torch.cuda.stream(ch.stream):
            assert_same(DIRECT["rq3"](ch), want["rq3"], "rq3 on the child after replays")
        torch.cuda.synchronize()
        for k in ("rq2_count", "rq4b"):
            assert_same(DIRECT[k](eng), want[k], f"{k} after replays")
    finally:
        eng.join_children()
        torch.cuda.synchronize()
        ch.close()


@pytest.mark.parametrize("case", goldens.CASES)
def test_rq3_split_across_streams(engine_for, case):
    """RQ3's sample extraction (fz_rq3_ex, FZ_RQ3_SKIP_STATS) recorded on a child, its statistics
    (fz_rq3_stats_dn: device sample lengths) recorded on the engine's own context, ordered by an
    event between the two streams - the bench's split grouping - equal the direct fz_rq3."""
    eng = engine_for(case)
    torch = eng.torch
    want = compute.rq3(eng)
    ch = eng.child()
    try:
        b = compute.rq3_buffers(eng)
        ch.follow_parent()
        compute.rq3_main_launch(ch, b)  # warm both contexts
        eng.join_children()
        compute.rq3_stats_launch(eng, b)
        torch.cuda.synchronize()
        assert_same(compute.rq3_collect(eng, b), want, "rq3 split (direct)")
        g_main = ch.record(lambda e: compute.rq3_main_launch(e, b))
        g_stats = eng.record(lambda e: compute.rq3_stats_launch(e, b))
        ev = torch.cuda.Event()
        try:
            for _ in range(3):
                _clear(b, torch)
                eng.join_children()
                eng.build_store()
                ch.follow_parent()
                g_main.launch()
                ev.record(ch.stream)
                eng.stream.wait_event(ev)
                g_stats.launch()
                torch.cuda.synchronize()
                assert_same(compute.rq3_collect(eng, b), want, "rq3 split (replay)")
        finally:
            g_main.close()
            g_stats.close()
    finally:
        eng.join_children()
        torch.cuda.synchronize()
        ch.close()


def test_replay_refused_after_rebuild_over_other_tables(engine):
    """A recording holds raw device pointers into the store and the context's buffers: after the
    store is rebuilt over a larger table (its columns reallocated) a replay is refused with
    FZ_E_STATE instead of reading freed memory; recording again works."""
    from tse_amd import engine as E
    small, big = goldens.tables("tiny"), goldens.tables("medium")
    engine.upload(small)
    engine.build_store()
    b = compute.rq2_count_buffers(engine)
    compute.rq2_count_launch(engine, b)  # warm
    engine.synchronize()
    g = engine.record(lambda e: compute.rq2_count_launch(e, b))
    try:
        g.launch()  # same store: accepted
        engine.synchronize()
        engine.upload(big)
        engine.build_store()
        with pytest.raises(E.FzError, match="record the graph again"):
            g.launch()
    finally:
        g.close()
    want = compute.rq2_count(engine)
    b = compute.rq2_count_buffers(engine)
    compute.rq2_count_launch(engine, b)
    engine.synchronize()
    g = engine.record(lambda e: compute.rq2_count_launch(e, b))
    try:
        _clear(b, engine.torch)
        g.launch()
        engine.synchronize()
        assert_same(compute.rq2_count_collect(engine, b), want, "rq2_count (re-recorded)")
    finally:
        g.close()
