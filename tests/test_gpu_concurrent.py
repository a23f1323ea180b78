"""Concurrent analyses (Engine.child / fz_ctx_create_child): the six analyses of one store run on
four child contexts, each with its own HIP stream, arena and host thread, give exactly the serial
results; across store rebuilds (parent waits for the children, children wait for the build) and
with the children's launches racing each other on the device."""
from concurrent.futures import ThreadPoolExecutor

import pytest

import goldens
from gpu_common import assert_same
from tse_amd.rq import compute

pytestmark = pytest.mark.gpu

ANALYSES = {"rq1": compute.rq1, "rq2_count": compute.rq2_count, "rq2_add": compute.rq2_add,
            "rq3": compute.rq3, "rq4a": compute.rq4a, "rq4b": compute.rq4b}
GROUPS = [["rq2_count"], ["rq4b", "rq1"], ["rq3", "rq4a"], ["rq2_add"]]


@pytest.mark.parametrize("helpers", [False, True])
@pytest.mark.parametrize("case", goldens.CASES)
def test_children_match_serial(engine_for, case, helpers):
    """(helpers: the store build also forks its table sorts and time-sort classes onto three of
    the children - fz_store_set_helpers - as bench.py does; destroying the children removes them
    as helpers, so the rebuild after close runs on the engine alone.)"""
    eng = engine_for(case)
    torch = eng.torch
    serial = {k: f(eng) for k, f in ANALYSES.items()}
    children = [eng.child() for _ in GROUPS]
    if helpers:
        eng.set_store_helpers(children[:3])

    def run(ch, names):
        with torch.cuda.stream(ch.stream):
            return {n: ANALYSES[n](ch) for n in names}

    try:
        with ThreadPoolExecutor(len(GROUPS)) as pool:
            for _ in range(3):
                eng.join_children()
                eng.build_store()
                for ch in children:
                    ch.follow_parent()
                got = {}
                for f in [pool.submit(run, ch, g) for ch, g in zip(children, GROUPS)]:
                    got.update(f.result())
                for k in ANALYSES:
                    assert_same(got[k], serial[k], k)
        eng.join_children()
        torch.cuda.synchronize()
    finally:
        for ch in children:
            ch.close()
    assert not eng.__dict__.get("_children")
    assert_same(compute.rq3(eng), serial["rq3"], "rq3 after children closed")
    if helpers:
        eng.build_store()
        for k in ("rq1", "rq4b"):
            assert_same(ANALYSES[k](eng), serial[k], f"{k} after a rebuild without the closed helpers")
