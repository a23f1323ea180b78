"""RCCL on the GPU box: the device-tensor branches of the collectives (parallel.py all_reduce /
all_gather / all_gather_v / all_to_all_v with `_staged` false) and bench.py's sharded step as the
multi-GPU runs use it - one fresh process over the "nccl" backend (RCCL; one rank per GPU, so one
rank on the one-GPU box), the six drivers' local phases recorded per analysis group and replayed on
four child contexts' streams (bench.py --shard-local streams), the drivers in one host thread in
the fixed order rq3, rq4b, rq2_count, rq1, rq4a, rq2_add on their analysis' stream, their final
copies deferred to one finalize_all - against the single-table analyses of the same store
(compute.*, pinned to the oracle by test_gpu_scale / test_gpu_rq*).  Reference: queries1.py:29-32
(the cross-shard ROW_NUMBER the RQ1 exchange serves), rq2_coverage_count.py:329-333 (the session
transposition the all-to-all serves)."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from test_parallel import _free_port

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

ORDER = ("rq3", "rq4b", "rq2_count", "rq1", "rq4a", "rq2_add")
GROUPS = (("rq3",), ("rq4b",), ("rq2_count",), ("rq1", "rq4a", "rq2_add"))


def _worker(rank, port, errfile, session_major=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        _collectives()
        _six_drivers(session_major)
    except BaseException:
        import traceback
        with open(f"{errfile}.{rank}", "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


def _collectives():
    """Each wrapper on device tensors through RCCL (no host staging), on a side stream too."""
    import torch.distributed as dist
    from tse_amd import parallel as par
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(3)
    x = torch.randint(-1000, 1000, (4099,), generator=g, dtype=torch.int64).to(dev)
    f = torch.randn(777, generator=g, dtype=torch.float64).to(dev)
    assert not par._staged(x)
    side = torch.cuda.Stream(dev)
    for stream in (torch.cuda.current_stream(dev), side):
        with torch.cuda.stream(stream):
            y = x.clone()
            par.all_reduce(y)
            m = f.clone()
            par.all_reduce(m, dist.ReduceOp.MAX)
            got = par.all_gather(f)
            gv = par.all_gather_v(x[:1234])
            a2a = par.all_to_all_v(x[:100], [100])
            cols = par.all_gather_cols([x[:50], f[:50]])
            a2c = par.all_to_all_cols([x[:60], f[:60]], [60])
        torch.cuda.synchronize(dev)
        assert y.is_cuda and torch.equal(y, x) and torch.equal(m, f)
        assert len(got) == 1 and got[0].is_cuda and torch.equal(got[0], f)
        assert len(gv) == 1 and torch.equal(gv[0], x[:1234])
        assert torch.equal(a2a, x[:100])
        assert torch.equal(cols[0][0], x[:50]) and torch.equal(cols[0][1], f[:50])
        assert torch.equal(a2c[0], x[:60]) and torch.equal(a2c[1], f[:60])
    assert par.agree_max(17, dev) == 17


def _six_drivers(session_major=False):
    import torch.distributed as dist
    from gpu_common import assert_same
    from test_parallel import rq2_add_result
    from tse_amd import engine as E
    from tse_amd import parallel as par
    from tse_amd import synth
    from tse_amd.rq import compute
    dev = torch.device("cuda", 0)
    t = synth.generate(synth.config("c2", dup_numbers=4000))
    P = len(t.projects)
    ts, rows = par.take_shard(t, 0, P)
    # (one rank holds the whole table: its row ids are the table's, no mapping anywhere below)
    assert all(np.array_equal(r, np.arange(len(r))) for r in (rows.builds, rows.coverage, rows.issues))
    eng = E.Engine(0)
    eng.upload(ts)
    st = eng.build_store()
    M = par.agree_max(int(st.max_fuzz_per_project), dev)
    # one child context per analysis group (bench.py --shard-local streams), the store build's helpers
    kids, lch = {}, []
    for g in GROUPS:
        ch = eng.child()
        lch.append(ch)
        for n in g:
            kids[n] = ch
    eng.set_store_helpers(lch)
    pg = dist.new_group(backend="nccl")
    shards = {"rq1": par.GpuRQ1Shard(kids["rq1"], M), "rq3": par.GpuRQ3Shard(kids["rq3"]),
              "rq2_count": par.GpuRQ2CountShard(kids["rq2_count"], session_major=session_major),
              "rq4a": par.GpuRQ4aShard(kids["rq4a"], M),
              "rq4b": par.GpuRQ4bShard(kids["rq4b"], session_major=session_major),
              "rq2_add": par.GpuRQ2AddShard(kids["rq2_add"])}
    graphs = []

    def step():
        eng.join_children()
        eng.build_store()
        for ch in lch:
            ch.follow_parent()
        for g, gr in graphs:  # every local phase at once, one recording per group on its stream
            gr.launch()
            for n in g:
                shards[n].pre = True
        pend, rq1 = {}, None
        for n in ORDER:
            with torch.cuda.stream(kids[n].stream), par.use_group(pg):
                if n == "rq3":
                    pend[n] = par.rq3_sharded(shards[n], 0, 1)
                elif n == "rq4b":
                    pend[n] = par.rq4b_sharded(shards[n], 0, 1, finish_later=True)
                elif n == "rq2_count":
                    pend[n] = par.rq2_count_sharded(shards[n], 0, 1, 0, P, finish_later=True)
                elif n == "rq1":
                    part, counts, it, idt, _ = par.rq1_sharded(shards[n], 0, 1)
                    rows1 = par.gather_rows({"matched_issue": part["matched_issue"],
                                             "matched_build": part["matched_build"]}, 1)
                    rq1 = (counts, it, idt, rows1)
                elif n == "rq4a":
                    pend[n] = par.rq4a_sharded(shards[n], 0, 1, 0, P, finish_later=True)
                else:
                    pend[n] = par.rq2_add_sharded(shards[n], 0, 1)
        cur = torch.cuda.current_stream(dev)
        for ch in lch:
            cur.wait_stream(ch.stream)
        ks = list(pend)
        res = dict(zip(ks, par.finalize_all([pend[k] for k in ks])))
        torch.cuda.synchronize(dev)
        return _to_results(res, rq1, shards["rq1"], rows)

    def _to_results(res, rq1, s1, rows):
        host = lambda v: v.cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)  # noqa: E731
        counts, it, idt, rows1 = rq1
        c = host(counts)
        n_it = int(c[E.RQ1_MAX_ITER])
        mi, mb = host(rows1["matched_issue"]), host(rows1["matched_build"])
        out = {"rq1": compute.rq1_result(c, host(it)[:n_it], host(idt)[:n_it], host(s1.bufs.late),
                                         rows.issues[mi], rows.builds[mb], np.nonzero(host(s1.bufs.eligible))[0])}
        total3, cols3, st3 = res["rq3"]
        cols = {k: host(v) for k, v in cols3.items()}
        cols["det_issue"] = rows.issues[cols["det_issue"]]
        out["rq3"] = compute.rq3_result(total3, cols, host(st3["describe"]), host(st3["tests"]))
        r2 = res["rq2_count"]
        out["rq2_count"] = compute.rq2_count_result(
            r2["proj"], r2["session_offsets"], r2["session_values"], r2["K"], r2["average"], r2["median"],
            r2["percentiles"], r2["average"], (r2["tests"][0], r2["tests"][1], r2["tests"][3]), r2["corr_mm"],
            r2["null_lines"])
        r4 = res["rq4a"]
        out["rq4a"] = compute.rq4a_result(r4["counts"], r4["scalars"], r4["member"], r4["tables"], r4["intro"],
                                          r4["g4_steps"], r4["g4_transition"])
        r4b = res["rq4b"]
        out["rq4b"] = compute.rq4b_result(r4b["counts"], r4b["c2"], r4b["c1"], r4b["g2_q"], r4b["g1_q"], r4b["p_bm"],
                                          r4b["sp6"], r4b["pre_cov"], r4b["post_cov"], r4b["pre_median"],
                                          r4b["post_median"], r4b["init_g2"], r4b["init_g1"], r4b["tests"])
        flags, cols2 = res["rq2_add"]
        out["rq2_add"] = rq2_add_result({k: host(v) for k, v in flags.items()}, {k: host(v) for k, v in cols2.items()})
        return out

    first = step()  # warm-up: the eager local phases
    for g in GROUPS:  # then record each group's local phases once and replay them
        graphs.append((g, kids[g[0]].record(lambda e, g=g: [shards[n].launch() for n in g])))
    replays = [step(), step()]
    ref = {"rq1": compute.rq1(eng), "rq2_count": compute.rq2_count(eng), "rq2_add": compute.rq2_add(eng),
           "rq3": compute.rq3(eng), "rq4a": compute.rq4a(eng), "rq4b": compute.rq4b(eng)}
    assert len(ref["rq1"].matched_issue) > 0 and len(ref["rq3"].det_pct) > 0 and ref["rq4b"].n_sessions > 0
    for got in [first] + replays:
        for k in ORDER:
            assert_same(got[k], ref[k], k)
    for _, gr in graphs:
        gr.close()
    eng.close()


@pytest.mark.parametrize("session_major", [False, True])
def test_rccl_world1_six_drivers_on_streams(tmp_path, session_major):
    """session_major: RQ2 count / RQ4b as bench.py runs them on one rank (values grouped by session
    in the recorded local phase, no run exchange); else the project-major exchange path."""
    errfile = str(tmp_path / "err")
    try:
        mp.spawn(_worker, args=(_free_port(), errfile, session_major), nprocs=1, join=True)
    except Exception:
        msg = open(f"{errfile}.0").read() if os.path.exists(f"{errfile}.0") else ""
        raise AssertionError(msg or "worker failed")
