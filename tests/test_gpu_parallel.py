"""Project-sharded RQ1 / RQ3 on the GPU: 2 ranks (both on cuda:0 - the box has one GPU), each
with its own libfz context holding only its projects' rows, exchanging over gloo (RCCL needs
one GPU per rank).  The exchange is the same code bench.py runs over RCCL; rank 0 checks the
recombined results against the oracle on the whole table."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from test_parallel import _free_port, make_table

pytestmark = pytest.mark.gpu


class _HostView:
    """Wraps a GPU shard so the gloo collectives see CPU tensors."""

    def __init__(self, shard, dev):
        self.s, self.dev = shard, dev

    def run(self, *a):
        a = tuple(None if x is None else tuple(v.to(self.dev) for v in x) for x in a)
        return {k: v.cpu() if isinstance(v, torch.Tensor) else v for k, v in self.s.run(*a).items()}

    def numbers(self, part):
        got = self.s.numbers({k: part[k].to(self.dev) for k in ("matched_issue", "matched_build")})
        return {k: v.cpu() for k, v in got.items()}

    def finish(self, counts, it, idt):
        c, i, d = (x.to(self.dev) for x in (counts, it, idt))
        self.s.finish(c, i, d)
        counts.copy_(c.cpu())

    def stats(self, *a):
        return {k: v.cpu() for k, v in self.s.stats(*(x.to(self.dev) for x in a)).items()}


class _RQ3View(_HostView):
    """... and maps the shard's detected issue rows to global row ids before they are gathered."""

    def __init__(self, shard, dev, issue_rows):
        super().__init__(shard, dev)
        self.issue_rows = issue_rows

    def run(self):
        out = super().run()
        out["det_issue"] = torch.from_numpy(self.issue_rows[out["det_issue"].numpy()].astype(np.int64))
        return out


class _RQ2View(_HostView):
    def run(self):
        return super().run()

    def session_stats_grouped(self, vals, offs, S, max_len):
        out = self.s.session_stats_grouped(vals.to(self.dev), offs.to(self.dev), S, max_len)
        return {k: v.cpu() for k, v in out.items()}

    def merge_runs(self, vals, runs):
        return tuple(v.cpu() for v in self.s.merge_runs(vals.to(self.dev), runs.to(self.dev)))

    def series_tests(self, x):
        return self.s.series_tests(x.to(self.dev))

    def mean_median(self, x):
        return self.s.mean_median(x.to(self.dev))


class _RQ4aView(_HostView):
    def finish(self, tables, intro, steps, counts):
        c = counts.to(self.dev)
        sc = self.s.finish([x.to(self.dev) for x in tables], intro.to(self.dev), steps.to(self.dev), c)
        counts.copy_(c.cpu())
        return sc


class _RQ4bView(_RQ2View):
    def spearman_prefix(self, rows, n):
        return self.s.spearman_prefix(rows.to(self.dev), n.to(self.dev)).cpu()

    def trends(self, cols):
        last, sp = self.s.trends([c.to(self.dev) for c in cols])
        return last.cpu(), sp.cpu()

    def two_sample(self, x, y):
        return self.s.two_sample(x.to(self.dev), y.to(self.dev))

    def row_medians(self, rows):
        return self.s.row_medians(rows.to(self.dev))


def _worker(rank, world, port, case, errfile):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _check(rank, world, case)
    except BaseException:
        import traceback
        with open(f"{errfile}.{rank}", "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


def _check(rank, world, case):
    from gpu_common import assert_same
    from oracle import rq_oracle as orc
    from tse_amd import engine as E
    from tse_amd import parallel as par
    from tse_amd.rq import compute
    t = make_table(case, world)
    lo, hi = par.shard_bounds(t, world)[rank]
    ts, rows = par.take_shard(t, lo, hi)
    eng = E.Engine(0)
    eng.upload(ts)
    st = eng.build_store()
    M = par.agree_max(int(st.max_fuzz_per_project))
    g1 = _HostView(par.GpuRQ1Shard(eng, M), eng.dev)
    part, counts, it, idt, reran = par.rq1_sharded(g1, rank, world)
    mi = torch.from_numpy(rows.issues[part["matched_issue"].numpy()].astype(np.int64))
    mb = torch.from_numpy(rows.builds[part["matched_build"].numpy()].astype(np.int64))
    rows1 = par.gather_rows({"matched_issue": mi, "matched_build": mb}, world)
    elig = g1.s.bufs.eligible.cpu().to(torch.int64)
    torch.distributed.all_reduce(elig)
    late = g1.s.bufs.late.cpu().numpy()
    total3, cols3, st3 = par.rq3_sharded(_RQ3View(par.GpuRQ3Shard(eng), eng.dev, rows.issues), rank, world)
    r2 = par.rq2_count_sharded(_RQ2View(par.GpuRQ2CountShard(eng), eng.dev), rank, world, lo, hi)
    r4 = par.rq4a_sharded(_RQ4aView(par.GpuRQ4aShard(eng, M), eng.dev), rank, world, lo, hi)
    r4b = par.rq4b_sharded(_RQ4bView(par.GpuRQ4bShard(eng), eng.dev), rank, world)
    if rank == 0:
        ours2 = compute.rq2_count_result(r2["proj"], r2["session_offsets"], r2["session_values"], r2["K"],
                                         r2["average"], r2["median"], r2["percentiles"], r2["average"],
                                         (r2["tests"][0], r2["tests"][1], r2["tests"][3]), r2["corr_mm"], r2["null_lines"])
        assert_same(ours2, orc.rq2_count(t), "rq2_count")
        ours4 = compute.rq4a_result(r4["counts"], r4["scalars"], r4["member"], r4["tables"], r4["intro"],
                                    r4["g4_steps"], r4["g4_transition"])
        assert_same(ours4, orc.rq4a(t), "rq4a")
        ours4b = compute.rq4b_result(r4b["counts"], r4b["c2"], r4b["c1"], r4b["g2_q"], r4b["g1_q"], r4b["p_bm"],
                                     r4b["sp6"], r4b["pre_cov"], r4b["post_cov"], r4b["pre_median"],
                                     r4b["post_median"], r4b["init_g2"], r4b["init_g1"], r4b["tests"])
        assert_same(ours4b, orc.rq4b(t), "rq4b")
        ours3 = compute.rq3_result(total3, {k: v.numpy() for k, v in cols3.items()}, st3["describe"].numpy(),
                                   st3["tests"].numpy())
        assert_same(ours3, orc.rq3(t), "rq3")
        ours1 = compute.rq1_result(counts.numpy(), it.numpy()[:int(counts[E.RQ1_MAX_ITER])],
                                   idt.numpy()[:int(counts[E.RQ1_MAX_ITER])], late, rows1["matched_issue"].numpy(),
                                   rows1["matched_build"].numpy(), np.nonzero(elig.numpy())[0])
        assert_same(ours1, orc.rq1(t), "rq1")
    eng.close()


@pytest.mark.parametrize("case", ["collide", "last_shard_no_issues"])
def test_gpu_sharded_rq1_rq3(case, tmp_path):
    errfile = str(tmp_path / "err")
    try:
        mp.spawn(_worker, args=(2, _free_port(), case, errfile), nprocs=2, join=True)
    except Exception:
        msgs = [open(f"{errfile}.{r}").read() for r in range(2) if os.path.exists(f"{errfile}.{r}")]
        raise AssertionError("\n".join(msgs) or "worker failed")


def test_host_many_gather():
    """parallel.host_many (fz_gather_to_host): contiguous, strided 1-D column slices, a strided 2-D
    block, 0-d, empty and one-element tensors of every element size, mixed with CPU tensors and
    numpy arrays - the same values as .cpu(), several reads in a row (the staging area is reused)."""
    from tse_amd import parallel as par
    dev = torch.device("cuda:0")
    g = torch.Generator().manual_seed(5)
    blk = torch.randn(97, 5, generator=g, dtype=torch.float64).to(dev)
    ts = [blk[:, 2], blk[:, 0], blk, blk[::3], torch.arange(1000, dtype=torch.int64, device=dev)[7::13],
          torch.randint(0, 255, (77,), generator=g, dtype=torch.uint8).to(dev),
          torch.randint(-9, 9, (33,), generator=g, dtype=torch.int32).to(dev)[::2],
          torch.tensor(3.5, dtype=torch.float64, device=dev), torch.empty(0, dtype=torch.int64, device=dev),
          torch.tensor([True, False, True], device=dev), torch.ones(1, 3, dtype=torch.float32, device=dev)[:, 1],
          torch.arange(5).to(torch.int16).to(dev), torch.arange(4), np.arange(3.0)]
    for _ in range(3):
        got = par.host_many(*ts)
        for t, h in zip(ts, got):
            want = t.cpu().numpy() if isinstance(t, torch.Tensor) else t
            assert h.dtype == want.dtype and h.shape == want.shape
            np.testing.assert_array_equal(h, want)
    big = torch.randn(3_000_000, dtype=torch.float64, device=dev)  # (the bulk path: DMA copy)
    got = par.host_many(big[::2], big[:5], torch.tensor(7, device=dev), np.arange(2))
    np.testing.assert_array_equal(got[0], big[::2].cpu().numpy())
    np.testing.assert_array_equal(got[1], big[:5].cpu().numpy())
    assert got[2] == 7 and list(got[3]) == [0, 1]
    mid = torch.randn(300_000, dtype=torch.float64, device=dev)  # (grows the pinned staging area)
    np.testing.assert_array_equal(par.host_many(mid[::3], mid[1::2])[1], mid[1::2].cpu().numpy())
