"""Graph-recording diagnostics, one stage per process (scripts/graph_diag.sh runs them in order and
stops at the first failure): record a call sequence on a context (Engine.record), replay it, and
compare with the direct calls.

    python scripts/graph_diag.py radix parent|child
    python scripts/graph_diag.py rq <rq1|rq2_count|rq2_add|rq3|rq4a|rq4b> parent|child [case] [rebuild|norebuild|sync]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]

import numpy as np  # noqa: E402


def radix(where):
    from tse_amd import engine as E
    eng = E.Engine(0)
    torch = eng.torch
    ctx = eng.child() if where == "child" else eng
    n = 300_000
    rng = np.random.default_rng(1)
    keys = torch.empty(n, dtype=torch.int64, device=eng.dev)
    vals = torch.empty(n, dtype=torch.int32, device=eng.dev)

    def fill(seed):
        k = np.random.default_rng(seed).integers(0, 1 << 40, n).astype(np.int64)
        keys.copy_(torch.from_numpy(k))
        vals.copy_(torch.arange(n, dtype=torch.int32))
        torch.cuda.synchronize()
        return k

    def run(e):
        E._check(e.lib, e.lib.fz_radix_sort_u64(e.ctx, E._P(keys.data_ptr()), E._P(vals.data_ptr()), n, 40))

    fill(0)
    run(ctx)  # warm
    torch.cuda.synchronize()
    g = ctx.record(run)
    print("recorded", flush=True)
    for seed in (1, 2, 3):
        k = fill(seed)
        g.launch()
        torch.cuda.synchronize()
        got_k, got_v = keys.cpu().numpy(), vals.cpu().numpy()
        order = np.argsort(k, kind="stable")
        assert np.array_equal(got_k, k[order]) and np.array_equal(got_v, order.astype(np.int32)), seed
        print("replay ok", seed, flush=True)
    run(ctx)  # a direct call after replays
    torch.cuda.synchronize()
    g.close()
    print("PASS radix", where, flush=True)


def rq(name, where, case, mode="rebuild"):
    import goldens
    from gpu_common import assert_same
    from tse_amd import engine as E
    from tse_amd.rq import compute
    parts = {"rq1": (compute.RQ1Buffers, compute.rq1_launch, compute.rq1_collect),
             "rq2_count": (compute.rq2_count_buffers, compute.rq2_count_launch, compute.rq2_count_collect),
             "rq2_add": (compute.rq2_add_buffers, compute.rq2_add_launch, compute.rq2_add_collect),
             "rq3": (compute.rq3_buffers, compute.rq3_launch, compute.rq3_collect),
             "rq4a": (compute.rq4a_buffers, compute.rq4a_launch, compute.rq4a_collect),
             "rq4b": (compute.rq4b_buffers, compute.rq4b_launch, compute.rq4b_collect)}
    mk, launch, collect = parts[name]
    eng = E.Engine(0)
    torch = eng.torch
    eng.upload(goldens.tables(case))
    eng.build_store()
    want = getattr(compute, name)(eng)
    ctx = eng.child() if where == "child" else eng
    b = mk(eng)
    if ctx is not eng:
        ctx.follow_parent()
    print("warm-up (direct)", flush=True)
    launch(ctx, b)  # warm
    eng.join_children()
    torch.cuda.synchronize()
    assert_same(collect(eng, b), want, name + " direct")
    print("recording", flush=True)
    g = ctx.record(lambda e: launch(e, b))
    print("recorded", flush=True)
    for it in range(int(os.environ.get("DIAG_REPLAYS", "3"))):
        for v in vars(b).values():
            if isinstance(v, torch.Tensor):
                v.zero_()
        eng.join_children()
        if mode != "norebuild":
            eng.build_store()
        if mode == "sync":
            torch.cuda.synchronize()
        if ctx is not eng:
            ctx.follow_parent()
        g.launch()
        eng.join_children()
        torch.cuda.synchronize()
        assert_same(collect(eng, b), want, f"{name} replay {it}")
        print("replay ok", it, flush=True)
    g.close()
    print("PASS", name, where, flush=True)


if __name__ == "__main__":
    if sys.argv[1] == "radix":
        radix(sys.argv[2])
    else:
        rq(sys.argv[2], sys.argv[3], sys.argv[4] if len(sys.argv) > 4 else "tiny",
           sys.argv[5] if len(sys.argv) > 5 else "rebuild")
