"""Headline benchmark: session-rows/s through the RQ1-RQ4 analytics on MI355X.

Workload (BASELINE.json configs[1]): a ~1M-session synthetic table with
the shipped schema - 1,000 projects, ~1.9M buildlog_data rows, ~0.95M total_coverage rows, ~65k
issues - resident in HBM.  One step = one pass of the hot path over it: the columnar store build
(radix sorts = the PostgreSQL tables + indexes) and every implemented RQ analysis (STAGES),
results left in HBM.  `value` = session rows (builds + coverage + issues) per second, whole job.

Multi-GPU (torchrun): weak scaling, one process per GPU.  Each rank owns its own project shard (a
config-2-sized table of disjoint projects); the per-iteration RQ1 histograms are summed across
ranks with one RCCL all-reduce per step (the only exchange the path has: projects are disjoint,
so distinct-project counts add).

Also reported: `roofline` for the dominant kernel (probe = HIP events around every launch of that
kernel inside the timed region; algorithmic bytes per launch as in DESIGN.md) and `cpu_baseline`
(the oracle port timed on this host, rank 0 only, on the same table, same stages).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PROBE_KERNEL = "radix_scatter"   # dominant kernel of the step (profiles/r01_*_stats.csv)
STAGES = ["store", "rq1", "rq2_count", "rq2_add", "rq3", "rq4a", "rq4b"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--probe", default=PROBE_KERNEL)
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import tse_amd.synth as synth
    from tse_amd import engine as E
    from tse_amd.rq import compute

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    cfg = synth.config(args.config, seed=synth.config(args.config).seed + 1000 * rank)
    t = synth.generate(cfg)
    eng = E.Engine(local)
    eng.upload(t)
    eng.build_store()
    rq1_bufs = compute.RQ1Buffers(eng)
    bufs = {"rq2_count": compute.rq2_count_buffers(eng), "rq2_add": compute.rq2_add_buffers(eng),
            "rq3": compute.rq3_buffers(eng), "rq4a": compute.rq4a_buffers(eng), "rq4b": compute.rq4b_buffers(eng)}
    launch = {"rq2_count": compute.rq2_count_launch, "rq2_add": compute.rq2_add_launch, "rq3": compute.rq3_launch,
              "rq4a": compute.rq4a_launch, "rq4b": compute.rq4b_launch}

    def step():
        eng.build_store()
        compute.rq1_launch(eng, rq1_bufs)
        for name in ("rq2_count", "rq2_add", "rq3", "rq4a", "rq4b"):
            launch[name](eng, bufs[name])
        if world > 1:
            # projects are disjoint across ranks: per-iteration project counts add
            dist.all_reduce(rq1_bufs.iter_total)
            dist.all_reduce(rq1_bufs.iter_detected)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    eng.probe_begin(args.probe)
    t0 = time.perf_counter()
    ev0.record(eng.stream)
    for _ in range(args.steps):
        step()
    ev1.record(eng.stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    launches, probe_ms, probe_bytes = eng.probe_end()
    dev_ms = ev0.elapsed_time(ev1)
    elapsed = wall
    rows = float(t.n_rows)
    if world > 1:
        v = torch.tensor([elapsed, rows], dtype=torch.float64, device=dev)
        tmax = v[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        rsum = v[1:].clone()
        dist.all_reduce(rsum, op=dist.ReduceOp.SUM)
        elapsed, rows = float(tmax.item()), float(rsum.item())

    out = None
    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = rows * args.steps / elapsed
        roof = None
        if launches > 0 and probe_ms > 0:
            avg_ms = probe_ms / launches
            ach = probe_bytes / launches / (avg_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": None, "kernel": args.probe,
                    "avg_launch_us": round(avg_ms * 1e3, 3), "bytes_per_launch": probe_bytes / launches,
                    "launches_per_step": launches / args.steps}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(t)
        out = {
            "metric": "session-rows/sec through RQ1-RQ4 aggregates+stats",
            "value": round(value, 1), "unit": "session-rows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int64/fp64", "data": "synthetic",
            "config": {"workload": f"config2: ~1M-session synthetic table ({args.config}), "
                                   f"{len(t.projects)} projects/rank",
                       "rows_per_rank": t.n_rows, "builds": int(len(t.b_project)), "coverage": int(len(t.c_project)),
                       "issues": int(len(t.i_project)), "stages": STAGES, "parallelism": f"project-shard x{world}",
                       "device_ms_per_step": round(dev_ms / args.steps, 4)},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()
    return out


def cpu_baseline(t):
    """The oracle port (numpy/scipy, single thread) over the same stages on the same table."""
    from oracle import rq_oracle as orc
    fns = {"rq1": orc.rq1, "rq2_count": orc.rq2_count, "rq2_add": orc.rq2_add, "rq3": orc.rq3,
           "rq4a": orc.rq4a, "rq4b": orc.rq4b}
    stages = [s for s in STAGES if s in fns]
    t0 = time.perf_counter()
    reps = 0
    while True:
        for s in stages:
            fns[s](t)
        reps += 1
        if time.perf_counter() - t0 > 10.0 or reps >= 20:
            break
    el = time.perf_counter() - t0
    return {"value": round(t.n_rows * reps / el, 1), "unit": "session-rows/s", "cores": 1, "kind": "port",
            "sample": f"oracle/rq_oracle.py {'+'.join(stages)} on the full bench table x{reps} "
                      f"({el:.1f} s, single-threaded numpy/scipy)"}


if __name__ == "__main__":
    main()
