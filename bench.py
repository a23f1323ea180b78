"""Headline benchmark: session-rows/s through the RQ1-RQ4 analytics on MI355X.

Workload (BASELINE.json configs[1]): a ~1M-session synthetic table with
the shipped schema - 1,000 projects, ~1.9M buildlog_data rows, ~0.95M total_coverage rows, ~65k
issues - resident in HBM.  One step = one pass of the hot path over it: the columnar store build
(radix sorts = the PostgreSQL tables + indexes) and every implemented RQ analysis (STAGES),
results left in HBM.  `value` = session rows (builds + coverage + issues) per second, whole job.

Multi-GPU (torchrun): weak scaling, one process per GPU.  Each rank owns its own project shard (a
config-2-sized table of disjoint projects; global project ids rank * P + p).  A step runs the
local stages and the exchange steps of tse_amd/parallel.py over RCCL: RQ1 (all-gather of match
numbers for the cross-shard ROW_NUMBER dedup, all-reduce of counters and per-iteration tables,
finishing on the summed tables), RQ3 (all-gather of the detected / non-detected samples, last
project rule, statistics over the union) and the RQ1 / RQ2 row gathers.

Also reported: `roofline` for the dominant kernel (probe = HIP events around every launch of that
kernel inside the timed region; algorithmic bytes per launch as in DESIGN.md) and `cpu_baseline`
(the oracle port timed on this host, rank 0 only, on the same table, same stages).
"""
from __future__ import annotations

import argparse
import json
import re
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
PROBE_KERNEL = "radix_scatter"   # headline kernel of the roofline object
# the per-kernel roofline table (a separate probe window after the timed region; algorithmic bytes
# per launch as DESIGN.md 4 defines them)
TABLE_KERNELS = ["radix_scatter", "radix_hist", "elig_hist", "seg_time_sort", "store_gather", "big_compact",
                 "big_sub_sort", "seg_merge_sort", "filter_compact", "filter_select", "seg_reduce", "seg_spearman", "seg_rank_union", "seg_value_sort", "seg_qstats",
                 "ragged_transpose", "scan_i64", "describe_select", "spearman_shapiro"]
STAGES = ["store", "rq1", "rq2_count", "rq2_add", "rq3", "rq4a", "rq4b"]
# analyses run concurrently after the store build: the first groups on child streams, the last on
# the engine's own stream after the store build (about equal GPU time at config 2: rq3 0.94 ms,
# rq4b 0.74, rq2_count 0.66, rq1 + rq4a + rq2_add 0.63 of kernel time; four streams in all -
# GPU_MAX_HW_QUEUES is 4 per process on the box, a fifth stream would share a hardware queue)
GROUPS = [["rq3"], ["rq4b"], ["rq2_count"], ["rq1", "rq4a", "rq2_add"]]
# RQ3 may also be split: "rq3_main" (samples) and "rq3_stats" (statistics, fz_rq3_stats_dn) in
# different groups; the stats group's stream then waits for an event recorded after rq3_main
AFTER = {"rq3_stats": "rq3_main"}
WORKLOADS = {"c2": "config2: ~1M-session synthetic table",
             "c3": "config3: 100M-row coverage-only table, 10k projects x 10k days",
             "c4": "config4: rank-statistics stress, 12 coverage series of 1e5/3e5/1e6 points, 256 levels",
             "c5": "config5: Zipf(1.2) rows per project, coverage-only, 10k projects",
             "c3L": "config3 live rows: 100M-row coverage-only table, 10k projects x 10k rows 6 h apart "
                    "(every row before the analysis limit)",
             "c5L": "config5 live rows: Zipf(1.2) rows per project, coverage-only, 10k projects, rows 10 s "
                    "apart (every row, the 20.8M-row giant's too, before the analysis limit)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    # e.g. --config c3 --stages store,rq2_count,rq4b: the coverage-only 100M-row table (SURVEY 8(d)
    # config 3) through the stages that read total_coverage
    ap.add_argument("--stages", default=",".join(STAGES))
    ap.add_argument("--probe", default=PROBE_KERNEL)
    # rehearsal on a one-GPU box: several ranks on cuda:0 exchanging over gloo (the driver's
    # multi-GPU runs use the default, RCCL)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"])
    # one rank through the sharded step (exchanges, host syncs, recombination) over a world-1 group:
    # the floor of the multi-GPU step time on a one-GPU box
    ap.add_argument("--force-sharded", action="store_true")
    # strong scaling (BASELINE north_star: 1->8 GPUs on one 100M-row table): every rank builds the
    # same table and keeps its parallel.shard_bounds project range; value = the whole table's rows
    ap.add_argument("--strong", action="store_true")
    # steps of the per-kernel probe window after the timed region (0: no table)
    ap.add_argument("--probe-steps", type=int, default=5)
    # the analyses one after another on the engine stream (default: concurrently, one child
    # context + HIP stream per group of analyses, after the store build)
    ap.add_argument("--serial", action="store_true")
    # concurrent groups launched call by call from host threads instead of replaying each group's
    # recorded HIP graph (fz_capture_begin/end, fz_graph_launch)
    ap.add_argument("--no-graphs", action="store_true")
    # stream groups, e.g. "rq3|rq4b|rq2_count|rq1,rq4a,rq2_add" (the last on the engine's stream)
    ap.add_argument("--groups", default="|".join(",".join(g) for g in GROUPS))
    # the sharded step's host threads (one child engine + process group each), same syntax; two
    # threads measured best (same-box A/B, scripts/gpu_shard_ab.sh: the drivers are host-bound)
    # the sharded step's drivers per host thread ("|" between threads); default: ONE thread, the
    # drivers in this fixed order - every rank issues its collectives in the same order (no
    # cross-communicator ordering hazard under RCCL), and with the final host copies deferred it
    # measured faster than two threads (c2 world 1: 2.56 vs 2.91 ms, profiles/r04_sharded_ab.txt)
    ap.add_argument("--shard-groups", default="rq3,rq4b,rq2_count,rq1,rq4a,rq2_add")
    ap.add_argument("--shard-graphs", action="store_true")
    # the sharded step's local phases (every driver's local kernels) as recordings on the
    # single-table step's four analysis streams (--groups), launched together before the drivers,
    # which then read / exchange / finish on their analysis' stream (same-box A/B,
    # scripts/gpu_shard_local_ab.sh: c2 3.42 -> 2.72 ms, c3 21.1 -> 19.7 ms, an eighth of c3 5.08 ->
    # 3.95 ms); "driver": each driver launches its own local kernels
    ap.add_argument("--shard-local", choices=["driver", "streams"], default="streams")
    # software pipelining of consecutive steps (single-table graph step): LANES engines, each with
    # its own copy of the table, store, analysis streams and recordings, take the steps in turn, so
    # one step's store build overlaps the previous step's analyses (1 = off)
    ap.add_argument("--lanes", type=int, default=1)
    # strong-scaling rehearsal on one GPU (with --strong --force-sharded at world 1): the step of
    # rank SHARD_RANK of SHARD_OF over its shard_bounds shard of the table - per-rank compute with
    # no exchange (the collectives need the other ranks); value = that shard's rows / s
    ap.add_argument("--shard-of", type=int, default=1)
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--cprofile", default="", help="write a cProfile summary of the timed steps (host time) here")
    ap.add_argument("--project-major", action="store_true",
                    help="one rank: RQ2 count / RQ4b through the project-major run exchange (as at N > 1)")
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
    if args.dist_backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    sharded = world > 1 or args.force_sharded
    if sharded:
        torch.cuda.set_device(local)
        init = {} if world > 1 else {"init_method": "tcp://127.0.0.1:29533", "world_size": 1, "rank": 0}
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), **init)
        else:
            dist.init_process_group("gloo", **init)
    dev = torch.device("cuda", local)

    rehearsal = args.strong and world == 1 and args.shard_of > 1
    cont, cut = -1, []
    if args.strong:
        from tse_amd import parallel as par
        full = synth.generate(synth.config(args.config))
        # project shards of about equal rows; a project larger than one share (config 5's Zipf
        # giant) cut into date-range pieces over consecutive ranks (parallel.live_plan)
        plan = par.live_plan(full, args.shard_of if rehearsal else world)
        r = args.shard_rank if rehearsal else rank
        lo, hi = plan.bounds[r]
        t = par.take_split(full, plan, r)[0]
        cont, cut = plan.cont[r], list(plan.cut)
        job_rows = full.n_rows if not rehearsal else None
        del full, plan
    else:
        cfg = synth.config(args.config, seed=synth.config(args.config).seed + 1000 * rank)
        t = synth.generate(cfg)
        if world > 1:
            t = weak_shard(t, rank, world)
        job_rows = None
    eng = E.Engine(local)
    eng.upload(t)  # first upload: pinned-buffer / allocator warm-up
    torch.cuda.synchronize(dev)
    t_up = time.perf_counter()
    eng.upload(t)  # host columns -> HBM (PCIe), timed for the end-to-end rate (never `value`)
    torch.cuda.synchronize(dev)
    upload_ms = (time.perf_counter() - t_up) * 1e3
    up = eng.upload_timing()  # host staging memcpy vs the H2D copy itself
    st = eng.build_store()
    stages = [s for s in STAGES if s in args.stages.split(",")]
    if sharded:
        from tse_amd import parallel as par
        M = par.agree_max(int(st.max_fuzz_per_project), dev)
        # the sharded step: every analysis' driver (local kernels + its exchanges) in its own host
        # thread, on its own child engine (stream + context over the store) and its own process
        # group of all ranks - their host round trips and collectives overlap instead of queueing
        # behind each other (--serial: one after another on the engine, the default group)
        sthreads = [[n for n in g.split(",") if n in stages] for g in args.shard_groups.split("|")]
        sthreads = [g for g in sthreads if g]
        snames = [n for g in sthreads for n in g]
        if len(sthreads) > 1 and world > 1 and args.dist_backend == "nccl" and not args.serial:
            # one communicator per host thread: RCCL collectives of different communicators issued
            # in different orders on different ranks can deadlock once their kernels share one of
            # the process' four hardware queues - one driver thread, one order
            raise SystemExit("bench: --shard-groups with several threads is refused over RCCL at world > 1")
        if args.serial:
            skids = {n: eng for n in snames}
            sgroups = {n: None for n in snames}
        else:
            skids, sgroups = {}, {}
            for g in sthreads:
                ch, pg = eng.child(), dist.new_group(backend=args.dist_backend)
                for n in g:
                    skids[n], sgroups[n] = ch, pg
            if args.shard_local == "streams":
                # one child per analysis group of the single-table step (its stream runs the
                # group's local phases, then each driver's finishing); the thread's process group
                # stays the driver's.  libfz calls on one context must come from one thread at a
                # time (fz.h), so a group whose drivers run in different --shard-groups threads
                # gets one child per (group, thread) pair
                thread_of = {n: ti for ti, g in enumerate(sthreads) for n in g}
                lgroups = [[n for n in g.split(",") if n in snames] for g in args.groups.split("|")]
                lgroups = [g for g in lgroups if g]
                lch, by_pair = [], {}
                for gi, g in enumerate(lgroups):
                    for n in g:
                        key = (gi, thread_of[n])
                        if key not in by_pair:
                            by_pair[key] = eng.child()
                            lch.append(by_pair[key])
                        skids[n] = by_pair[key]
                # the local phases are recorded per child: the drivers of one (group, thread) pair
                lgroups = [[n for g in lgroups for n in g if skids[n] is ch] for ch in lch]
                eng.set_store_helpers(lch[:4])  # (idle while the store builds: the step joins them first)
        rq1_shard = par.GpuRQ1Shard(skids.get("rq1", eng), M)
        rq3_shard = par.GpuRQ3Shard(skids.get("rq3", eng))
        # (one rank without a cut project: the local kernels group the values by session themselves)
        smaj = world == 1 and cont < 0 and not args.project_major
        rq2c_shard = par.GpuRQ2CountShard(skids.get("rq2_count", eng), cont, session_major=smaj)
        rq4a_shard = par.GpuRQ4aShard(skids.get("rq4a", eng), M)
        rq4b_shard = par.GpuRQ4bShard(skids.get("rq4b", eng), cont, session_major=smaj)
        elig_ctl = par.GpuEligibility(eng)
        rq2a_shard = par.GpuRQ2AddShard(skids.get("rq2_add", eng))
        if args.strong:
            own = (lo, hi)
        else:
            own = (rank * len(t.projects) // world, (rank + 1) * len(t.projects) // world)  # weak_shard ids
    def make_bufs(e):
        b = {"rq2_count": compute.rq2_count_buffers(e), "rq2_add": compute.rq2_add_buffers(e),
             "rq3": compute.rq3_buffers(e), "rq4a": compute.rq4a_buffers(e), "rq4b": compute.rq4b_buffers(e),
             "rq1": compute.RQ1Buffers(e)}
        b["rq3_main"] = b["rq3_stats"] = b["rq3"]
        return b
    bufs = make_bufs(eng)
    launch = {"rq2_count": compute.rq2_count_launch, "rq2_add": compute.rq2_add_launch, "rq3": compute.rq3_launch,
              "rq4a": compute.rq4a_launch, "rq4b": compute.rq4b_launch}

    launch["rq1"] = lambda e, b: compute.rq1_launch(e, b)
    launch["rq3_main"], launch["rq3_stats"] = compute.rq3_main_launch, compute.rq3_stats_launch
    # concurrent analyses: groups of about equal GPU time, one child engine (stream + context over
    # the same store) and one host thread each (ctypes releases the GIL during every libfz call)
    known = set(stages) | ({"rq3_main", "rq3_stats"} if "rq3" in stages else set())
    groups = [[n for n in g.split(",") if n in known] for g in args.groups.split("|")]
    groups = [g for g in groups if g]
    concurrent = not sharded and not args.serial and len(groups) > 1
    split = any(n in AFTER for g in groups for n in g)
    # host launch order: groups holding a stage another group waits for come first
    order = sorted(range(len(groups)), key=lambda i: 0 if any(n in AFTER.values() for n in groups[i]) else 1)
    if split and (args.no_graphs or not concurrent):
        raise SystemExit("bench: rq3_main / rq3_stats groupings need the graph path")
    pool = None
    graphs = None
    sgraphs = None  # sharded step: one recording of each driver's local kernels
    if sharded:
        def sh_rq1(e):
            part = par.rq1_sharded(rq1_shard, rank, world)[0]
            par.gather_rows({"issue": part["matched_issue"], "build": part["matched_build"]}, world)

        def sh_rq2_add(e):
            if world > 1:  # flags OR-reduced, change rows gathered in rank order
                par.rq2_add_sharded(rq2a_shard, rank, world)
                return
            if not rq2a_shard.pre:  # (one rank: its rows are the result - nothing to read or gather)
                rq2a_shard.launch()
            rq2a_shard.pre = False
        # the drivers' final host copies are deferred (parallel.Deferred) and made in one copy at the
        # end of the step (par.finalize_all): the GPU is drained once, not once per driver
        pending = []

        def finalize_pending():
            # the deferred results were produced on the drivers' streams: this stream waits for
            # them, then one device->host copy of them all
            cur = torch.cuda.current_stream(dev)
            for e in {id(x): x for x in skids.values()}.values():
                cur.wait_stream(e.stream)
            par.finalize_all(pending)
            pending.clear()
        shard_step = {
            "rq1": sh_rq1,
            "rq2_count": lambda e: pending.append(par.rq2_count_sharded(rq2c_shard, rank, world, *own,
                                                                        gather_values=False, finish_later=True,
                                                                        cont=cont, host_sessions=False)),
            "rq4a": lambda e: pending.append(par.rq4a_sharded(rq4a_shard, rank, world, *own, finish_later=True)),
            "rq4b": lambda e: pending.append(par.rq4b_sharded(rq4b_shard, rank, world, *own, finish_later=True,
                                                              cont=cont, host_sessions=False)),
            "rq2_add": sh_rq2_add,
            "rq3": lambda e: par.rq3_sharded(rq3_shard, rank, world),
        }

        # the local kernels of every driver (graph-capturable: no host reads), for the recordings
        shards = {"rq1": rq1_shard, "rq3": rq3_shard, "rq2_count": rq2c_shard, "rq4a": rq4a_shard,
                  "rq4b": rq4b_shard, "rq2_add": rq2a_shard}
        local_launch = {n: shards[n].launch for n in shards}

        def mark_launched(names):
            for n in names:
                shards[n].pre = True

        drv_ms = {}  # host wall time per driver (its launches, syncs and collectives), summed over steps

        def run_sharded(names):
            for name in names:
                e = skids[name]
                if sgraphs is not None and args.shard_local == "driver":
                    # this driver's local kernels replayed from its recording right before it reads
                    # them (the next driver's local phase is enqueued only after this one's exchange
                    # and finishing kernels, as in the eager order)
                    sgraphs[name].launch()
                    mark_launched([name])
                t_d = time.perf_counter()
                with torch.cuda.stream(e.stream), par.use_group(sgroups[name]):
                    shard_step[name](e)
                drv_ms[name] = drv_ms.get(name, 0.0) + (time.perf_counter() - t_d) * 1e3
        if not args.serial:
            from concurrent.futures import ThreadPoolExecutor
            pool = ThreadPoolExecutor(len(sthreads))
    if concurrent:
        from concurrent.futures import ThreadPoolExecutor
        # the last group runs on the engine itself (its stream, after the store build)
        children = [eng.child() for _ in groups[:-1]] + [eng]
        pool = ThreadPoolExecutor(len(groups) - 1)
        # the store build forks its independent sorts onto the (then idle) children
        eng.set_store_helpers(children[:-1][:4])  # (the library takes up to four)

        def run_group(ch, names, b=None):
            with torch.cuda.stream(ch.stream):
                for n in names:
                    launch[n](ch, (b or bufs)[n])

    lanes = []  # (pipelined steps) the extra engines: eng, bufs, children, graphs, events each
    lane_turn = [0]

    def serial_step():
        eng.build_store()
        for name in ("rq1", "rq2_count", "rq2_add", "rq3", "rq4a", "rq4b"):
            if name in stages:
                launch[name](eng, bufs[name])

    def step():
        if not sharded:
            if not concurrent:
                serial_step()
                return
            if graphs is not None and lanes:
                # pipelined: the lanes take the steps in turn (lane 0 = eng); a lane's store build
                # waits only for its own previous analyses, so it overlaps the other lane's
                L = ([None] + lanes)[lane_turn[0] % (len(lanes) + 1)]
                lane_turn[0] += 1
                if L is not None:
                    le, lch, lgr, lev = L["eng"], L["children"], L["graphs"], L["events"]
                    le.join_children()
                    le.build_store()
                    for ch in lch[:-1]:
                        ch.follow_parent()
                    for gi in order:
                        for need, gr, mark in lgr[gi]:
                            if need:
                                lch[gi].stream.wait_event(lev[need])
                            gr.launch()
                            if mark:
                                lev[mark].record(lch[gi].stream)
                    return
            eng.join_children()  # the previous step's analyses have read the store
            eng.build_store()
            if graphs is not None:
                # host order: producers' events are recorded before any stream waits on them; each
                # child follows the store (one event recorded after the build, waited on by each
                # child) right before its first replay - the critical group's replay is enqueued
                # first, ahead of the other children's stream waits
                store_done.record(eng.stream)
                for gi in order:
                    if children[gi] is not eng:
                        children[gi].stream.wait_event(store_done)
                        children[gi]._share()
                    for need, gr, mark in graphs[gi]:
                        if need:
                            children[gi].stream.wait_event(events[need])
                        gr.launch()
                        if mark:
                            events[mark].record(children[gi].stream)
                return
            for ch in children[:-1]:
                ch.follow_parent()
            if split:  # warm-up before the recordings: the groups one after another (dependencies)
                for gi in order:
                    run_group(children[gi], groups[gi])
                    torch.cuda.synchronize(dev)
                return
            futs = [pool.submit(run_group, ch, g) for ch, g in zip(children[:-1], groups[:-1])]
            run_group(eng, groups[-1])
            for f in futs:
                f.result()
            return
        # sharded: exact recombination of every script over the ranks (tse_amd/parallel.py)
        eng.join_children()  # the previous step's drivers have read the store
        eng.build_store()
        # a cut project's eligibility over all of its pieces (one all-reduce, before the analyses)
        with torch.cuda.stream(eng.stream):
            par.fix_cut_eligibility(elig_ctl, cut, *own, world)
        if pool is None:
            run_sharded(snames)
            finalize_pending()
            return
        for ch in set(skids.values()):
            if ch is not eng:
                ch.follow_parent()
        if sgraphs is not None and args.shard_local == "streams":
            # every local phase at once, one recording per analysis group on its own stream
            for g, gr in sgraphs_local:
                gr.launch()
                mark_launched(g)
        if len(sthreads) == 1:  # one host thread: the drivers in order on this one
            run_sharded(sthreads[0])
        else:
            futs = [pool.submit(run_sharded, g) for g in sthreads]
            for f in futs:
                f.result()
        finalize_pending()

    # (opt-in: replaying each driver's local kernels from a recording measured no faster than the
    # eager launches - c2 3.79 vs 3.46 ms, c3 22.2 vs 21.8 ms, same box: the drivers' host work
    # between their reads hides the launches already)
    shard_graphs = sharded and pool is not None and (args.shard_graphs or args.shard_local == "streams") \
        and not args.no_graphs
    sgraphs_local = []
    for _ in range(max(args.warmup, 1 if (concurrent or shard_graphs) and not args.no_graphs else 0)):
        step()
    torch.cuda.synchronize(dev)
    if shard_graphs:
        if args.shard_local == "streams":
            sgraphs_local = [(g, skids[g[0]].record(lambda e, g=g: [local_launch[n]() for n in g])) for g in lgroups]
            sgraphs = {}
        else:
            sgraphs = {n: skids[n].record(lambda e, n=n: local_launch[n]()) for n in snames}
        step()  # one untimed replay step
        torch.cuda.synchronize(dev)
    if concurrent and not args.no_graphs:
        # record each group once (warm contexts), then every step replays the recordings; a group
        # is cut into pieces at a stage that must follow another group's stage (AFTER) and after a
        # stage another group waits for - one graph per piece, events between them
        marks = set(AFTER.values())

        def record_groups(chs, b):
            out = []
            for ch, g in zip(chs, groups):
                pieces, cur = [], []
                for n in g:
                    if n in AFTER and cur:
                        pieces.append((None if not pieces else pieces[-1][3], cur, None, None))
                        cur = []
                    cur.append(n)
                    if n in marks:
                        pieces.append((None, cur, n, None))
                        cur = []
                if cur:
                    pieces.append((None, cur, None, None))
                rec = []
                for _, names, mark, _ in pieces:
                    need = AFTER.get(names[0])
                    rec.append((need, ch.record(lambda e, names=names: [launch[n](e, b[n]) for n in names]), mark))
                out.append(rec)
            return out
        events = {m: torch.cuda.Event() for m in marks}
        store_done = torch.cuda.Event()  # (recorded after each step's store build)
        graphs = record_groups(children, bufs)
        for _ in range(args.lanes - 1):
            # another lane: its own engine (table copy, store, streams), warmed once, then recorded
            e2 = E.Engine(local)
            e2.upload(t)
            e2.build_store()
            b2 = make_bufs(e2)
            ch2 = [e2.child() for _ in groups[:-1]] + [e2]
            e2.set_store_helpers(ch2[:-1][:4])
            e2.join_children()
            e2.build_store()
            for ch in ch2[:-1]:
                ch.follow_parent()
            for gi in order:
                run_group(ch2[gi], groups[gi], b2)
                torch.cuda.synchronize(dev)
            lanes.append({"eng": e2, "bufs": b2, "children": ch2, "graphs": record_groups(ch2, b2),
                          "events": {m: torch.cuda.Event() for m in marks}})
        for _ in range(len(lanes) + 1):
            step()  # one untimed replay step per lane
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    # (the probe brackets launches on the engine's own context: with the analyses on child contexts
    # it is measured on serial steps after the timed region)
    on_children = concurrent or (sharded and pool is not None)
    if not on_children:
        eng.probe_begin(args.probe)
    if sharded:
        drv_ms.clear()
    prof = None
    if args.cprofile:
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    t0 = time.perf_counter()
    ev0.record(eng.stream)
    for _ in range(args.steps):
        step()
    if concurrent or sharded:
        eng.join_children()
        for L in lanes:
            L["eng"].join_children()
            eng.stream.wait_stream(L["eng"].stream)
    ev1.record(eng.stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    if prof is not None:
        prof.disable()
        import io
        import pstats
        buf = io.StringIO()
        pstats.Stats(prof, stream=buf).sort_stats("tottime").print_stats(45)
        pstats.Stats(prof, stream=buf).sort_stats("cumulative").print_stats(60)
        with open(args.cprofile, "w") as f:
            f.write(f"{args.steps} steps, wall {wall * 1e3:.2f} ms\n" + buf.getvalue())
    drv = {k: round(v / args.steps, 3) for k, v in drv_ms.items()} if sharded else None
    probe_window = args.steps
    if not on_children:
        launches, probe_ms, probe_bytes = eng.probe_end()
    else:  # the probe brackets launches on the engine's own context: measure it on serial steps
        probe_window = max(args.probe_steps, 1)
        eng.probe_begin(args.probe)
        for _ in range(probe_window):
            serial_step()
        launches, probe_ms, probe_bytes = eng.probe_end()
    dev_ms = ev0.elapsed_time(ev1)
    elapsed = wall
    rows = float(t.n_rows)
    # per-kernel table: a separate window (its HIP events would perturb the timed steps)
    table = []
    if args.probe_steps > 0:
        eng.probe_begin(",".join(TABLE_KERNELS))
        for _ in range(args.probe_steps):
            serial_step() if on_children or not sharded else step()
        eng.probe_end()
        for k in TABLE_KERNELS:
            n, ms_k, b_k = eng.probe_get(k)
            if n == 0 or ms_k <= 0 or b_k <= 0:  # (no bytes: an empty input's launch, e.g. no issues)
                continue
            ach = b_k / (ms_k * 1e-3) / 1e9
            tr = pmc_traffic(k, args.config)
            row = {"kernel": k, "launches_per_step": round(n / args.probe_steps, 2),
                   "avg_launch_us": round(ms_k / n * 1e3, 3), "bytes_per_launch": round(b_k / n),
                   "achieved": round(ach, 1), "frac": round(ach / HBM_PEAK_GBS, 4),
                   "ms_per_step": round(ms_k / args.probe_steps, 4), "traffic": tr}
            if tr:  # PMC bytes per launch over this window's launch time, and over the algorithmic bytes
                row["traffic_gbs"] = round(tr / (ms_k / n * 1e-3) / 1e9, 1)
                row["traffic_ratio"] = round(tr / (b_k / n), 3) if b_k > 0 else None
            table.append(row)
    if world > 1:
        v = torch.tensor([elapsed, rows], dtype=torch.float64, device=dev)
        tmax = v[:1].clone()
        par.all_reduce(tmax, dist.ReduceOp.MAX)
        rsum = v[1:].clone()
        par.all_reduce(rsum)
        elapsed, rows = float(tmax.item()), float(rsum.item())
    if job_rows is not None:  # strong scaling: the whole table, whatever the shard sizes
        rows = float(job_rows)

    out = None
    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        value = rows * args.steps / elapsed
        roof = None
        if launches > 0 and probe_ms > 0:
            avg_ms = probe_ms / launches
            ach = probe_bytes / launches / (avg_ms * 1e-3) / 1e9
            roof = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": pmc_traffic(args.probe, args.config),
                    "kernel": args.probe,
                    "avg_launch_us": round(avg_ms * 1e3, 3), "bytes_per_launch": probe_bytes / launches,
                    "launches_per_step": launches / probe_window, "kernels": table}
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            cpu = cpu_baseline(t, stages)
        out = {
            "metric": "session-rows/sec through RQ1-RQ4 aggregates+stats",
            "value": round(value, 1), "unit": "session-rows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 4), "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak", "vs_baseline": None, "dtype": "int64/fp64", "data": "synthetic",
            "config": {"workload": f"{WORKLOADS.get(args.config, args.config)} ({args.config}), "
                                   + (f"rank {args.shard_rank} of {args.shard_of}'s shard of one table - strong-scaling "
                                      f"rehearsal: per-rank compute, no exchange" if rehearsal
                                      else f"one table split over {world} ranks" if args.strong
                                      else f"{len(t.projects)} projects/rank"),
                       "rows_per_rank": t.n_rows, "builds": int(len(t.b_project)), "coverage": int(len(t.c_project)),
                       "issues": int(len(t.i_project)),
                       # rows an analysis can read: every build and issue row, and the coverage rows
                       # dated before the latest bound any script applies (RQ3's DATE(date) <
                       # '2025-01-09', rq3:263; the others '2025-01-08', queries1.py:3) - configs 3 / 5
                       # put most of their rows after it, where only the store sorts them
                       "rows_analysed": rows_analysed(t), "stages": stages, "parallelism": f"project-shard x{world}" + (" (sharded path)" if sharded and world == 1 else ""),
                       "device_ms_per_step": round(dev_ms / args.steps, 4),
                       **({"driver_host_ms": drv} if drv else {}),
                       # end-to-end (host columns -> HBM upload + one step), per rank: the loader's
                       # PCIe-inclusive rate; `value` is compute-only with inputs resident in HBM
                       "upload_ms": round(upload_ms, 3), "upload_host_ms": up["host_ms"],
                       "upload_h2d_ms": up["h2d_ms"], "upload_h2d_gbs": up["h2d_gbs"],
                       "rows_per_s_incl_upload": round(t.n_rows / ((upload_ms + ms_step) * 1e-3), 1)},
            "roofline": roof, "cpu_baseline": cpu,
            # (committed rehearsals, not this run: the strong-scaling figures beside this line's mode)
            "strong_rehearsal": strong_rehearsals(),
        }
        print(json.dumps(out), flush=True)
    if pool is not None:
        pool.shutdown()
    for rec in graphs or []:
        for _, gr, _ in rec:
            gr.close()
    for gr in (sgraphs or {}).values():
        gr.close()
    for _, gr in sgraphs_local:
        gr.close()
    for L in lanes:
        for rec in L["graphs"]:
            for _, gr, _ in rec:
                gr.close()
        L["eng"].close()
    eng.close()
    if sharded:
        dist.destroy_process_group()
    return out


def strong_rehearsals():
    """The newest committed one-GPU strong-scaling rehearsals (profiles/r*_<config>_strong.json,
    scripts/strong_summary.py: per N the slowest of the N shards' sharded steps = an N-GPU run's
    per-rank compute before any exchange), beside this line's own scaling mode."""
    import glob
    out = {}
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "r*_strong.json"))):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        if d.get("config"):
            out[d["config"]] = {"T_ms": d.get("T_ms"), "efficiency": d.get("efficiency"),
                                "source": os.path.relpath(path, REPO)}
    return out or None


def pmc_traffic(probe, config):
    """HBM bytes per launch (probe scope) of a probed kernel from the committed PMC passes
    (profiles/*_pmc_traffic.json, written by scripts/pmc_traffic.py from rocprofv3 FETCH_SIZE /
    WRITE_SIZE runs of this bench with the gfx950 FETCH_SIZE correction; newest first), or None."""
    import glob

    def version(path):  # r02v10_c2_pmc_traffic.json -> (2, 10): numeric, so v10 sorts after v6
        m = re.match(r"r(\d+)v(\d+)_", os.path.basename(path))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)
    for path in sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")), key=version, reverse=True):
        try:
            d = json.load(open(path))
        except (OSError, ValueError):
            continue
        k = d.get("kernels", {}).get(probe)
        if k and d.get("config") == config:
            return round(float(k["traffic_bytes_per_launch"]))
    return None


def rows_analysed(t):
    from tse_amd.schema import RQ3_LIMIT_US
    return int(len(t.b_project) + len(t.i_project) + np.count_nonzero(t.c_date < RQ3_LIMIT_US))


def cgroup_cpus():
    """CPUs of the cgroup v2 / v1 CPU quota of this process (None: unlimited or unreadable)."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(p)))
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, q // p)
    except (OSError, ValueError):
        return None


def weak_shard(t, rank, world):
    """Rank `rank`'s table as one shard of a world-times-larger job: project ids rank * P + p in a
    global id space of world * P projects.  Issue numbers keep their values: the ranks draw them
    from the same range, so numbers collide across shards and the cross-shard ROW_NUMBER dedup
    (fz_rq1_ex re-run, queries1.py:29-32) happens inside every timed step."""
    import dataclasses
    P = len(t.projects)
    off = np.uint32(rank * P)
    # this rank's projects keep their names (the corpus CSV refers to them); the other ranks'
    # ids get placeholder names
    names = [n if r == rank else f"~{r}-{n}" for r in range(world) for n in t.projects]
    return dataclasses.replace(
        t, projects=names, b_project=t.b_project + off, c_project=t.c_project + off, i_project=t.i_project + off,
        pi_project=t.pi_project + off)


def _oracle_stages(t, stages):
    from oracle import rq_oracle as orc
    fns = {"rq1": orc.rq1, "rq2_count": orc.rq2_count, "rq2_add": orc.rq2_add, "rq3": orc.rq3,
           "rq4a": orc.rq4a, "rq4b": orc.rq4b}
    for s in stages:
        if s in fns:
            fns[s](t)


def cpu_baseline(t, stages):
    """The multi-core C++ restatement (oracle/cpu/fz_cpu.cpp: per-project index build + the same
    analyses, OpenMP over projects / sessions) on the full bench table with the host's CPU share of
    threads: one untimed run, then repeated runs for >= 3 s, median wall time.  Beside it: the same
    code on one thread, and the numpy oracle (oracle/rq_oracle.py) single-threaded when the table is
    small enough to finish in ~10 s (<= 4 M rows)."""
    from oracle import cpu_baseline as cb
    stages = [s for s in stages if s in cb.STAGES]
    host_cpus = os.cpu_count() or 1
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else host_cpus
    quota = cgroup_cpus()
    # every core this process may use: the affinity set, capped by the cgroup CPU quota (on the GPU
    # box os.cpu_count() is the whole machine; the job's share is the quota / OMP_NUM_THREADS)
    share = min(aff, quota) if quota else aff
    cores = max(1, min(int(os.environ.get("OMP_NUM_THREADS") or share), aff))
    host = cb.HostTables(t)
    big = t.n_rows > 20_000_000  # configs 3 / 5: one run is seconds; keep the leg to ~30 s

    def timed(threads, min_s, reps_min):
        if not big:
            cb.run(host, stages, threads)  # warm: page faults, thread pool
        walls, parts = [], []
        t_end = time.perf_counter() + min_s
        while len(walls) < reps_min or (time.perf_counter() < t_end and len(walls) < 20):
            t0 = time.perf_counter()
            _, secs = cb.run(host, stages, threads)
            walls.append(time.perf_counter() - t0)
            parts.append(secs)
        k = int(np.argsort(walls)[len(walls) // 2])
        return walls[k], parts[k], len(walls)

    wall, parts, reps = timed(cores, 0.0 if big else 3.0, 2 if big else 3)
    one, _, reps1 = timed(1, 0.0 if big else 2.0, 1 if big else 3)
    how = "fastest of" if reps == 2 else "median of"
    out = {"value": round(t.n_rows / wall, 1), "unit": "session-rows/s", "cores": cores, "kind": "port",
           "host_cpus": host_cpus, "affinity_cpus": aff, "cgroup_quota_cpus": quota,
           "sample": f"oracle/cpu/fz_cpu.cpp (C++17, OpenMP, {cores} threads = every CPU of this job's share: "
                     f"affinity {aff}, cgroup quota {quota or 'none'}, machine {host_cpus}): index build + "
                     f"{'+'.join(stages)} on the full bench table ({t.n_rows} rows), {how} {reps} runs "
                     f"({wall * 1e3:.1f} ms; " + ", ".join(f"{k} {v * 1e3:.1f}" for k, v in parts.items() if v)
                     + " ms)",
           "single_core": {"value": round(t.n_rows / one, 1), "cores": 1,
                           "sample": f"the same code on one thread, median of {reps1} runs ({one * 1e3:.1f} ms)"}}
    if t.n_rows <= 4_000_000:
        t1 = time.perf_counter()
        _oracle_stages(t, stages)
        py = time.perf_counter() - t1
        out["numpy_oracle"] = {"value": round(t.n_rows / py, 1), "cores": 1,
                               "sample": f"oracle/rq_oracle.py (numpy/scipy, one process) on the same table "
                                         f"({py:.1f} s)"}
    return out


if __name__ == "__main__":
    main()
