"""The project-sharded path on the FULL 100M-row tables ("100M coverage rows over
10k projects, project-sharded over 2/4/8 MI355X"): configs 3 and 5 and their live-row variants c3L /
c5L (every row before the analysis limit, synth.py).  Two, four or eight ranks on cuda:0, each
holding its ``parallel.live_plan`` share - a project larger than one share (config 5's 20.8M-row
Zipf giant) cut into date-range pieces over consecutive ranks, its eligibility summed over the
pieces - run RQ2-count and RQ4b through libfz (fz_rq2_count_ex / fz_rq4b_ex project-major, the
project-major session exchange to the session owners, fz_rq2_session_stats_grouped /
fz_rq4b_session_stats_grouped there, a cut project's Spearman / Shapiro-Wilk from value buckets,
the gathers) over gloo - the same driver code bench.py runs over RCCL.  Rank 0 then builds the whole
table on one engine and requires the recombined results to equal the single-GPU ones, which
test_gpu_fullsize.py pins to numpy / scipy at this size:

* the session transposition of rq2_coverage_count.py:329-333 - offsets and every value, exact;
* every per-project column, every per-session statistic (rq2_coverage_count.py:139-152,439-440),
  the median-trend tests (:443-458), the correlation mean / median;
* RQ4b's per-session counts, quartiles, Brunner-Munzel p (rq4b_coverage.py:910-985), last session,
  the six Spearman tests (:879-899), deltas (:725-797) and initial-coverage tests (:221-313).

Integers exact, floats within 1e-9 relative (gpu_common.assert_same)."""
import os

import numpy as np
import pytest
import torch.multiprocessing as mp

from test_parallel import _free_port

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _worker(rank, world, port, name, errfile):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _check(rank, world, name)
    except BaseException:
        import traceback
        with open(f"{errfile}.{rank}", "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


def _check(rank, world, name):
    import time

    import torch.distributed as dist

    import tse_amd.synth as synth
    from gpu_common import assert_same
    from tse_amd import engine as E
    from tse_amd import parallel as par
    from tse_amd.rq import compute
    t0 = time.perf_counter()
    t = synth.generate(synth.config(name))
    assert t.n_rows >= 99_000_000
    # project shards; a project larger than a rank's share (config 5's Zipf giant) cut into date-range
    # pieces over consecutive ranks (parallel.live_plan)
    plan = par.live_plan(t, world)
    bounds = plan.bounds
    lo, hi = bounds[rank]
    if rank == 0:
        rows = (np.bincount(t.b_project.astype(np.int64), minlength=len(t.projects))
                + np.bincount(t.c_project.astype(np.int64), minlength=len(t.projects))
                + np.bincount(t.i_project.astype(np.int64), minlength=len(t.projects)))
        share = [(len(b) + len(c) + len(i)) / (t.n_rows / world)
                 for b, c, i in zip(plan.builds, plan.coverage, plan.issues)]
        print(f"{name} world {world}: largest project {int(rows.max()):,} rows, cut projects {plan.cut} over "
              f"{[plan.ranks[p] for p in plan.cut]}, {plan.moved:,} rows off their owner; shard shares of the mean "
              + " ".join(f"{x:.2f}" for x in share), flush=True)
        if name.startswith("c5") and world == 8:
            assert plan.moved > 0 and max(share) < 1.15, "the Zipf giant was meant to be cut"
    ts, _ = par.take_split(t, plan, rank)
    cont = plan.cont[rank]
    eng = E.Engine(0)
    eng.upload(ts)
    eng.build_store()
    par.fix_cut_eligibility(par.GpuEligibility(eng), plan.cut, lo, hi, world)
    r2 = par.rq2_count_sharded(par.GpuRQ2CountShard(eng, cont), rank, world, lo, hi, cont=cont)
    r4b = par.rq4b_sharded(par.GpuRQ4bShard(eng, cont), rank, world, lo=lo, hi=hi, cont=cont)
    eng.close()
    del ts, eng
    print(f"rank {rank}: shard [{lo}, {hi}) of {len(t.projects)} projects, sharded RQ2-count + RQ4b "
          f"{time.perf_counter() - t0:.1f} s", flush=True)
    dist.barrier()  # both shard engines are gone before the whole-table engine is built
    if rank != 0:
        return
    assert len(bounds) == world and bounds[0][0] == 0 and bounds[-1][1] == len(t.projects)
    ours2 = compute.rq2_count_result(r2["proj"], r2["session_offsets"], r2["session_values"], r2["K"],
                                     r2["average"], r2["median"], r2["percentiles"], r2["average"],
                                     (r2["tests"][0], r2["tests"][1], r2["tests"][3]), r2["corr_mm"], r2["null_lines"])
    ours4b = compute.rq4b_result(r4b["counts"], r4b["c2"], r4b["c1"], r4b["g2_q"], r4b["g1_q"], r4b["p_bm"],
                                 r4b["sp6"], r4b["pre_cov"], r4b["post_cov"], r4b["pre_median"], r4b["post_median"],
                                 r4b["init_g2"], r4b["init_g1"], r4b["tests"])
    one = E.Engine(0)
    one.upload(t)
    one.build_store()
    ref2 = compute.rq2_count(one)
    ref4b = compute.rq4b(one)
    one.close()
    # the transposition (rq2_coverage_count.py:329-333) value for value, then every field
    assert np.array_equal(ours2.session_offsets, ref2.session_offsets), "session offsets"
    assert np.array_equal(ours2.session_values, ref2.session_values), "session values"
    assert len(ref2.ge100) > 0 and len(ref2.eligible) > 0
    # the sharded driver reports statistics.mean as the per-session average; the single-GPU
    # result carries np.mean separately (dist_mean): equal within the tolerance (1 ulp apart)
    assert_same(ours2, ref2, "rq2_count")
    assert ref4b.n_sessions > 0 and np.all(ref4b.c2 + ref4b.c1 > 0)
    assert_same(ours4b, ref4b, "rq4b")


@pytest.mark.parametrize("name,world", [("c3", 2), ("c3", 8), ("c5", 4), ("c5", 8), ("c3L", 4), ("c5L", 2),
                                        ("c5L", 8)])
def test_sharded_fullsize_matches_single_gpu(name, world, tmp_path):
    errfile = str(tmp_path / "err")
    try:
        mp.spawn(_worker, args=(world, _free_port(), name, errfile), nprocs=world, join=True)
    except Exception:
        msgs = [open(f"{errfile}.{r}").read() for r in range(world) if os.path.exists(f"{errfile}.{r}")]
        raise AssertionError("\n".join(msgs) or "worker failed")
