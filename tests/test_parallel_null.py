"""The sharded drivers on the NULL line-count edge tables (tests/null_edges.py), world 2 over gloo:
every rank raises the reference's TypeError inside rq2_count_sharded / rq3_sharded - after the
collective that gave it the global counts, so no rank is left waiting in an exchange - exactly when
the reference crashed (rq2_coverage_count.py:300-303, rq3_diff_coverage_at_detection.py:253,297;
pinned by the reference-run goldens tests/golden/tiny+<edge>/), and completes where it ran."""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import goldens
import null_edges
from test_parallel import OracleRQ2CountShard, OracleRQ3Shard, _free_port
from tse_amd import parallel as par


class OracleRQ2CountShardNull(OracleRQ2CountShard):
    """OracleRQ2CountShard that reports its NULL line count (the rows fz_rq2_count_ex counts into
    counts[FZ_RQ2C_NULL_LINES]) instead of raising locally."""

    def run(self):
        from oracle import rq_oracle as orc
        t = self.t
        elig = np.zeros(len(t.projects), bool)
        elig[orc.eligible_projects(t)] = True
        sel = (elig[t.c_project.astype(np.int64)] & t.c_coverage_valid & (t.c_coverage != 0)
               & (t.c_date < null_edges.LIMIT_US) & ((t.c_total != 0) | ~t.c_total_valid))
        nulls = int(np.sum(sel & ~(t.c_covered_valid & t.c_total_valid)))
        if nulls:  # the oracle itself raises; the shard reports the count the kernel would
            cols = {"eligible": torch.from_numpy(elig.astype(np.int64))}
            for k in ("raw_n", "n_trend"):
                cols[k] = torch.zeros(len(t.projects), dtype=torch.int64)
            for k in ("sw_w", "sw_p", "corr"):
                cols[k] = torch.full((len(t.projects),), float("nan"), dtype=torch.float64)
            cols["values"] = torch.zeros(0, dtype=torch.float64)
            out = cols
        else:
            out = super().run()
        out["null_lines"] = torch.tensor([nulls], dtype=torch.int64)
        return out


def _worker(rank, world, port, edge, errfile):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = goldens.tables("tiny+" + edge)
        lo, hi = par.shard_bounds(t, world)[rank]
        ts, rows = par.take_shard(t, lo, hi)
        got = {}
        for name, f in (("rq2_coverage_count",
                         lambda: par.rq2_count_sharded(OracleRQ2CountShardNull(ts), rank, world, lo, hi)),
                        ("rq3_diff_coverage_at_detection", lambda: par.rq3_sharded(OracleRQ3Shard(ts, rows), rank, world))):
            try:
                f()
                got[name] = 0
            except TypeError:
                got[name] = 1
        for name, raised in got.items():
            want = goldens.returncode("tiny+" + edge, name) != 0
            assert bool(raised) == want, (rank, edge, name, raised, want)
    except BaseException:
        with open(f"{errfile}.{rank}", "w") as f:
            import traceback
            f.write(traceback.format_exc())
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("edge", null_edges.EDGES)
def test_sharded_drivers_raise_like_the_reference(edge, tmp_path):
    errfile = str(tmp_path / "err")
    world = 2
    try:
        mp.spawn(_worker, args=(world, _free_port(), edge, errfile), nprocs=world, join=True)
    except Exception:
        msgs = [open(f"{errfile}.{r}").read() for r in range(world) if os.path.exists(f"{errfile}.{r}")]
        raise AssertionError("\n".join(msgs) or "worker failed")
