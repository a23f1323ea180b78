"""Project-sharded multi-GPU layer (BASELINE.json north_star "Multi-GPU layer").

One process per GPU (torchrun), ``torch.distributed`` over RCCL on the GPU box (gloo in the CPU
tests).  Every per-project computation of the RQ scripts is independent, so the session tables are
cut into contiguous project-id ranges with about equal row counts (``shard_bounds``); each rank
uploads only its own projects' rows (``take_shard``; project ids stay global) and runs the
per-project kernels locally.  The exchange steps are the places where the reference's arithmetic
spans projects:

RQ1 (``rq1_sharded``)
    * per-iteration tables (``total_projects[i]``, distinct detecting projects) and the scalar
      counters are summed - projects are disjoint across ranks, so distinct-project counts add -
      and the iteration axis length is a MAX (all_reduce);
    * the SAME_DATE_BUILD_ISSUE dedup ``ROW_NUMBER() OVER (PARTITION BY i.number ORDER BY
      timecreated DESC)`` (queries1.py:29-32) partitions by issue number ACROSS projects: every
      rank all-gathers the (number, build time) of the other ranks' matches; a rank whose matches
      share a number with another rank's re-runs its match with those as competitors
      (``fz_rq1_ex``).  A rank's first-pass winners contain the global winner, so one re-run is
      exact;
    * finishing (kept iterations, first_down, late-stage summary, rq1:233-268) runs on the summed
      tables (``fz_rq1_finish``).
RQ3 (``rq3_sharded``)
    * detected / non-detected samples are all-gathered in rank (= project) order;
    * the reference flushes a project's non-detected changes when its issue loop reaches the next
      project, so only the globally last issue-bearing project is never flushed (rq3:245-257):
      every rank runs with ``FZ_RQ3_FLUSH_LAST`` and the tail of the last rank with issues is
      dropped;
    * the statistics run once over the gathered samples (``fz_rq3_stats``).
RQ2 coverage-and-added (``rq2_add_sharded``): per-project change rows, concatenated in rank order;
    the per-project flags OR-combined.

The drivers take a *shard* object (``run`` / ``finish`` / ``stats``) so the same exchange code runs
over the GPU engine (``GpuRQ1Shard``, ``GpuRQ3Shard``) and, in the CPU tests, over the oracle.
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

from .schema import LIMIT_US, RQ3_LIMIT_US, TS_NULL, US_PER_DAY, Tables

# fz.h RQ1 counter layout (FZ_RQ1_*)
(RQ1_ISSUES_LIM, RQ1_ISSUES_LIM_PROJECTS, RQ1_FIXED_LIM, RQ1_FIXED_LIM_PROJECTS, RQ1_ELIGIBLE,
 RQ1_WITHOUT_MATCHING, RQ1_TARGET, RQ1_TARGET_PROJECTS, RQ1_TOTAL_FUZZ, RQ1_MATCHED, RQ1_MATCHED_PROJECTS,
 RQ1_MAX_ITER, RQ1_KEPT_ITERS, RQ1_FIRST_DOWN, RQ1_LATE) = range(15)
RQ1_NCOUNTS = 16
# fz.h RQ3 counter layout (FZ_RQ3_*)
RQ3_ISSUES, RQ3_DETECTED, RQ3_NON_DETECTED, RQ3_ELIGIBLE, RQ3_NON_LAST, RQ3_NULL_TOTAL, RQ3_NULL_LAST = range(7)
RQ3_NCOUNTS = 8


# ------------------------------------------------------------------------------------- sharding
def shard_bounds(t: Tables, world: int) -> List[Tuple[int, int]]:
    """Contiguous project-id ranges [lo, hi), one per rank, minimising the largest shard's
    session-row count (a giant project stays whole on one rank and is split across workgroups
    there).  The smallest capacity C for which a greedy left-to-right packing needs at most `world`
    ranges is found by bisection over the prefix sums (the linear-partition bound: with config 5's
    20.8 M-row Zipf giant the largest of 4 shards drops from 34.8 M rows - cuts at the equal-rows
    targets - to the packing optimum); the ranges are then cut at that C, and left empty only when
    there are fewer projects than ranks."""
    P = len(t.projects)
    rows = (np.bincount(t.b_project.astype(np.int64), minlength=P)
            + np.bincount(t.c_project.astype(np.int64), minlength=P)
            + np.bincount(t.i_project.astype(np.int64), minlength=P)).astype(np.int64)
    return partition_rows(rows, world)


def partition_rows(rows: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """shard_bounds over per-project row counts: min-max contiguous partition into `world` ranges."""
    P = len(rows)
    cum = np.concatenate([[0], np.cumsum(rows)]).astype(np.int64)
    total = int(cum[-1])
    if world <= 1 or P == 0:
        return [(0, P)] + [(P, P)] * (world - 1) if world > 1 else [(0, P)]

    def cuts_for(cap):  # greedy: each range as long as it stays <= cap (a project over cap alone)
        cuts, lo = [0], 0
        while lo < P and len(cuts) <= world:
            hi = int(np.searchsorted(cum, cum[lo] + cap, "right")) - 1
            hi = max(hi, lo + 1)
            cuts.append(min(hi, P))
            lo = cuts[-1]
        return cuts

    lo_c, hi_c = max(int(rows.max()), -(-total // world)), total
    while lo_c < hi_c:
        mid = (lo_c + hi_c) // 2
        if cuts_for(mid)[-1] >= P and len(cuts_for(mid)) - 1 <= world:
            hi_c = mid
        else:
            lo_c = mid + 1
    cuts = cuts_for(lo_c)
    while len(cuts) - 1 < world:  # fewer ranges than ranks: split the largest multi-project range
        sizes = [(cum[cuts[i + 1]] - cum[cuts[i]], i) for i in range(len(cuts) - 1) if cuts[i + 1] - cuts[i] > 1]
        if not sizes:
            cuts.append(P)  # (empty trailing ranges)
            continue
        _, i = max(sizes)
        a, b = cuts[i], cuts[i + 1]
        mid = int(np.searchsorted(cum, (cum[a] + cum[b]) // 2, "left"))
        mid = min(max(mid, a + 1), b - 1)
        cuts.insert(i + 1, mid)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


@dataclass
class ShardRows:
    """Global row ids of a shard's rows (shard row i == global row ids[i])."""
    lo: int
    hi: int
    builds: np.ndarray
    coverage: np.ndarray
    issues: np.ndarray


def take_shard(t: Tables, lo: int, hi: int) -> Tuple[Tables, ShardRows]:
    """The rows of projects [lo, hi) in their original (heap) order; project ids, vocabularies,
    string pools and the corpus CSV stay global."""
    def sel(p):
        p = p.astype(np.int64)
        return np.nonzero((p >= lo) & (p < hi))[0]
    b, c, i = sel(t.b_project), sel(t.c_project), sel(t.i_project)
    pi = sel(t.pi_project)
    s = dataclasses.replace(
        t, b_project=t.b_project[b], b_type=t.b_type[b], b_result=t.b_result[b], b_time=t.b_time[b],
        b_modules=t.b_modules[b], b_revisions=t.b_revisions[b], b_name=t.b_name[b],
        c_project=t.c_project[c], c_date=t.c_date[c], c_coverage=t.c_coverage[c],
        c_coverage_valid=t.c_coverage_valid[c], c_covered=t.c_covered[c], c_covered_valid=t.c_covered_valid[c],
        c_total=t.c_total[c], c_total_valid=t.c_total_valid[c],
        i_number=t.i_number[i], i_project=t.i_project[i], i_rts=t.i_rts[i], i_status=t.i_status[i],
        i_new_id=t.i_new_id[i], pi_project=t.pi_project[pi], pi_first_commit=t.pi_first_commit[pi])
    return s, ShardRows(lo, hi, b, c, i)


# ------------------------------------------------------------------------- giant projects split
# A project larger than one rank's share (config 5's Zipf giant: 20.8 M of 100 M rows) would make
# its rank the slowest whatever the cut.  Every analysis reads a coverage row only when it is dated
# before a bound (the latest is RQ3's DATE(date) < '2025-01-09', rq3:263; the others use
# '2025-01-08', queries1.py:3) or when it lies in RQ4b's coverage-delta window (the last 7 positive
# rows before the corpus day and the first 7 from it, rq4b_coverage.py:745-772).  So a giant's
# other coverage rows - "movable" - are read by no analysis: they can sit on any rank.  There
# their project has no row before the eligibility date bound, so it is never eligible (>= 365 rows,
# rq1:144-152) and enters no analysis, while the rank's store still holds and sorts them: the
# store's work follows the rows, the analyses' stay with the owner.  The owner keeps the giant's
# builds, issues, every coverage row before the bound and the delta window; the movable rows are
# spread over the ranks in date order to even out their row counts - the owner's share first, the
# earliest ones: its rows of the giant stay one run of dates.  (A gap in a segment's dates - the
# owner's pre-bound rows and a far-off movable range - packs most of the segment into a few of
# the store's time sub-buckets, which overflow into the merge sort: config 5's owner at eight
# ranks took 6.4 ms against 4.3-4.7 for the others.)
SPLIT_BOUND_US = int(max(LIMIT_US, RQ3_LIMIT_US))
DELTA_WINDOW = 7


@dataclass
class SplitPlan:
    """Per rank: its own project range [lo, hi) and the global row ids it holds of each table."""
    bounds: List[Tuple[int, int]]
    builds: List[np.ndarray]
    coverage: List[np.ndarray]
    issues: List[np.ndarray]
    info: List[np.ndarray]
    moved: int  # coverage rows placed on another rank than their project's owner


def _giant_must(t: Tables, rows: np.ndarray, p: int, corpus_us) -> np.ndarray:
    """Mask over a project's coverage rows (global ids `rows`, ascending): the rows an analysis may
    read - dated before SPLIT_BOUND_US, or in the delta window around the corpus day."""
    date = t.c_date[rows]
    must = date < SPLIT_BOUND_US
    cu = int(corpus_us[p])
    if cu != TS_NULL:
        pos = np.nonzero(t.c_coverage_valid[rows] & (t.c_coverage[rows] > 0))[0]
        if len(pos):
            o = pos[np.argsort(date[pos], kind="stable")]      # positive rows by (date, row)
            j = int(np.searchsorted(date[o], (cu // US_PER_DAY) * US_PER_DAY, "left"))
            w = o[max(0, j - DELTA_WINDOW):j + DELTA_WINDOW]
            must[w] = True
            if len(w):
                # every positive row sharing a date with the window's first or last row stays too:
                # which of equal-date rows the ORDER BY date ... LIMIT 7 picks is then irrelevant
                edge = (date[pos] == date[w[0]]) | (date[pos] == date[w[-1]])
                must[pos[edge]] = True
    return must


def split_plan(t: Tables, world: int) -> SplitPlan:
    """shard_bounds with the giants' movable coverage rows spread over the ranks (see above)."""
    from .rq.common import corpus_columns
    P = len(t.projects)
    nb = np.bincount(t.b_project.astype(np.int64), minlength=P)
    nc = np.bincount(t.c_project.astype(np.int64), minlength=P)
    ni = np.bincount(t.i_project.astype(np.int64), minlength=P)
    total = (nb + nc + ni).astype(np.int64)
    target = -(-int(total.sum()) // max(world, 1))
    # (projects over half a share: a contiguous cut around one of them leaves its range unbalanced -
    # config 5 at four ranks: largest share 1.17 of the mean with the 20.8 M-row giant whole)
    giants = np.nonzero(total > target // 2)[0] if world > 1 else np.zeros(0, np.int64)
    movable = {}
    if len(giants):
        corpus_us = corpus_columns(t)[1]
        sel = np.nonzero(np.isin(t.c_project, giants.astype(t.c_project.dtype)))[0]
        gp = t.c_project[sel].astype(np.int64)
        order = np.argsort(gp, kind="stable")
        sel, gp = sel[order], gp[order]
        starts = np.searchsorted(gp, giants)
        ends = np.searchsorted(gp, giants, "right")
        for p, a, b in zip(giants.tolist(), starts.tolist(), ends.tolist()):
            rows = sel[a:b]
            m = rows[~_giant_must(t, rows, p, corpus_us)]
            if len(m):
                movable[p] = m[np.argsort(t.c_date[m], kind="stable")]  # date order
    weight = total.copy()
    for p, m in movable.items():
        weight[p] -= len(m)
    bounds = partition_rows(weight, world)
    load = np.array([int(weight[a:b].sum()) for a, b in bounds], np.int64)
    incoming = [[] for _ in range(world)]
    out_of = {}
    for p, m in movable.items():
        owner = next(r for r, (a, b) in enumerate(bounds) if a <= p < b)
        k = min(len(m), max(0, target - int(load[owner])))  # the owner's share: the earliest rows
        load[owner] += k
        while k < len(m):
            # the least-loaded rank takes the next date range, up to the mean share
            r = int(np.argmin(load))
            take = max(1, min(len(m) - k, target - int(load[r]))) if load[r] < target else len(m) - k
            if r != owner:
                incoming[r].append(m[k:k + take])
                out_of.setdefault(p, []).append(m[k:k + take])
            load[r] += take
            k += take
    moved_out = np.sort(np.concatenate([x for v in out_of.values() for x in v])) if out_of else np.zeros(0, np.int64)

    def sel_rows(proj, lo, hi):
        p = proj.astype(np.int64)
        return np.nonzero((p >= lo) & (p < hi))[0]
    B, C, I, PI = [], [], [], []
    for r, (lo, hi) in enumerate(bounds):
        B.append(sel_rows(t.b_project, lo, hi))
        own = sel_rows(t.c_project, lo, hi)
        if len(moved_out):
            own = own[~np.isin(own, moved_out, assume_unique=True)]
        extra = np.concatenate(incoming[r]) if incoming[r] else np.zeros(0, np.int64)
        C.append(np.sort(np.concatenate([own, extra])) if len(extra) else own)
        I.append(sel_rows(t.i_project, lo, hi))
        PI.append(sel_rows(t.pi_project, lo, hi))
    return SplitPlan(bounds, B, C, I, PI, int(len(moved_out)))


def take_split(t: Tables, plan: SplitPlan, rank: int) -> Tuple[Tables, ShardRows]:
    """Rank `rank`'s table of a split plan (rows in their original order; ids, pools and the
    corpus CSV global) and the global ids of its rows."""
    b, c, i, pi = plan.builds[rank], plan.coverage[rank], plan.issues[rank], plan.info[rank]
    lo, hi = plan.bounds[rank]
    s = dataclasses.replace(
        t, b_project=t.b_project[b], b_type=t.b_type[b], b_result=t.b_result[b], b_time=t.b_time[b],
        b_modules=t.b_modules[b], b_revisions=t.b_revisions[b], b_name=t.b_name[b],
        c_project=t.c_project[c], c_date=t.c_date[c], c_coverage=t.c_coverage[c],
        c_coverage_valid=t.c_coverage_valid[c], c_covered=t.c_covered[c], c_covered_valid=t.c_covered_valid[c],
        c_total=t.c_total[c], c_total_valid=t.c_total_valid[c],
        i_number=t.i_number[i], i_project=t.i_project[i], i_rts=t.i_rts[i], i_status=t.i_status[i],
        i_new_id=t.i_new_id[i], pi_project=t.pi_project[pi], pi_first_commit=t.pi_first_commit[pi])
    return s, ShardRows(lo, hi, b, c, i)


# ------------------------------------------------------------- live split: a project cut in pieces
# split_plan above moves only rows no analysis reads.  When the rows of a project larger than one
# rank's share ARE read (config 5's live-row variant: every one of the giant's 20.8 M rows precedes
# the analysis limit), the project is cut into date ranges ("pieces") on consecutive ranks.  The
# reference reads it as one series (queries1.py:120-129), value i of session i
# (rq2_coverage_count.py:329-333, rq4b_coverage.py:917-931) and one shapiro / spearmanr
# (rq2_coverage_count.py:305-322); the sharded drivers keep all of that exact across the cut:
#   * eligibility (rq1:144-152): the pieces' counts summed every step (fix_cut_eligibility), the
#     project eligible on its first piece's rank only (its owner), ineligible on the others;
#   * sessions: every rank sends its runs - a project's values with the session index they start at
#     (a later piece starts where the earlier pieces' values end) - to the session owners, which
#     transpose the runs they receive (project-major exchange, _exchange_runs);
#   * the cut project's Spearman / Shapiro-Wilk: its values sorted in value buckets over the piece
#     ranks, per-bucket partial sums at their global sorted positions (_series_tests_cut).
# A project is cut only when no analysis needs its rows in one place beyond that: it has no builds
# and no issues (RQ1, RQ3, RQ2-add and RQ4a read nothing of it but its eligibility) and is not in
# rq4b's group 3 / 4 (whose delta window, rq4b_coverage.py:745-772, is a date range of the series).
@dataclass
class LivePlan:
    """Per rank r: bounds[r] = its own project range (a cut project belongs to its first piece's
    rank), the global row ids it holds of each table (builds / coverage / issues / info), cont[r] =
    the cut project whose later piece leads rank r's coverage rows (-1: none); cut = the cut
    projects (ascending) and ranks[p] = the ranks holding project p's pieces in date order."""
    bounds: List[Tuple[int, int]]
    builds: List[np.ndarray]
    coverage: List[np.ndarray]
    issues: List[np.ndarray]
    info: List[np.ndarray]
    cont: List[int]
    cut: List[int]
    ranks: dict
    moved: int  # coverage rows held by another rank than their project's owner


def live_plan(t: Tables, world: int) -> LivePlan:
    """Contiguous shards of about equal rows, a project larger than one share cut into pieces of
    about one share each (in (date, row) order) when the rules above allow it; then the min-max
    contiguous partition (partition_rows) over the sequence of whole projects and pieces."""
    from .rq.common import corpus_groups
    P = len(t.projects)
    cp = t.c_project.astype(np.int64)
    nb = np.bincount(t.b_project.astype(np.int64), minlength=P)
    nc = np.bincount(cp, minlength=P)
    ni = np.bincount(t.i_project.astype(np.int64), minlength=P)
    total = (nb + nc + ni).astype(np.int64)
    target = -(-int(total.sum()) // max(world, 1))
    pieces = {}  # p -> [row ids of each piece], date order
    if world > 1:
        big = np.nonzero((total > target) & (nb == 0) & (ni == 0))[0]
        if len(big):
            q = t.c_coverage_valid & (t.c_coverage > 0) & (t.c_date < LIMIT_US)
            elig = np.nonzero(np.bincount(cp[q], minlength=P) >= 365)[0]
            groups, _ = corpus_groups(t, elig, add_missing_to_g1=False)
            g34 = set(groups["group3"]) | set(groups["group4"])
            g12 = set(groups["group1"]) | set(groups["group2"])
            for p in big.tolist():
                if p in g34:
                    continue
                rows = np.nonzero(cp == p)[0]
                rows = rows[np.argsort(t.c_date[rows], kind="stable")]
                # pieces of an eighth of a share: the partition below balances the ranks to within
                # that, and a rank's consecutive pieces of the project are one piece
                k = -(-len(rows) // max(target // 8, 1))
                cuts = [len(rows) * j // k for j in range(k + 1)]
                if p in g12:  # rq4b's initial coverage (:230-240) is the first piece's first value
                    f = np.nonzero(q[rows])[0]
                    if len(f):
                        cuts = [0] + [c for c in cuts[1:] if c > f[0]]
                pieces[p] = [rows[cuts[j]:cuts[j + 1]] for j in range(len(cuts) - 1) if cuts[j + 1] > cuts[j]]
    # units: whole projects and pieces, in project order
    u_proj, u_w, u_piece = [], [], []
    for p in range(P):
        if p in pieces:
            for j, r in enumerate(pieces[p]):
                u_proj.append(p)
                u_w.append(len(r))
                u_piece.append(j)
        else:
            u_proj.append(p)
            u_w.append(int(total[p]))
            u_piece.append(-1)
    u_proj, u_piece = np.array(u_proj, np.int64), np.array(u_piece, np.int64)
    ub = partition_rows(np.array(u_w, np.int64), world)
    head_unit = np.searchsorted(u_proj, np.arange(P), "left")  # first unit of each project
    lo = [int(np.searchsorted(head_unit, a, "left")) for a, _ in ub]
    bounds = [(lo[r], lo[r + 1] if r + 1 < world else P) for r in range(world)]
    cont, ranks = [], {}
    for r, (a, b) in enumerate(ub):
        cont.append(int(u_proj[a]) if a < b and u_piece[a] > 0 else -1)
        for u in range(a, b):
            if u_piece[u] >= 0:
                ranks.setdefault(int(u_proj[u]), [])
                if r not in ranks[int(u_proj[u])]:
                    ranks[int(u_proj[u])].append(r)
    cut = sorted(p for p, rs in ranks.items() if len(rs) > 1)
    ranks = {p: ranks[p] for p in cut}

    def sel(proj, a, b):
        x = proj.astype(np.int64)
        return np.nonzero((x >= a) & (x < b))[0]
    is_cut = np.zeros(P, bool)
    is_cut[cut] = True
    # (pieces of a project that all landed on one rank: the project is whole there)
    for p in [p for p in pieces if p not in ranks]:
        del pieces[p]
    B, Cv, I, PI = [], [], [], []
    moved = 0
    for r, (a, b) in enumerate(bounds):
        B.append(sel(t.b_project, a, b))
        own = sel(t.c_project, a, b)
        own = own[~is_cut[cp[own]]]
        extra = []
        for u in range(*ub[r]):
            p = int(u_proj[u])
            if is_cut[p]:
                extra.append(pieces[p][int(u_piece[u])])
                if ranks[p][0] != r:
                    moved += len(extra[-1])
        Cv.append(np.sort(np.concatenate([own] + extra)) if extra else own)
        I.append(sel(t.i_project, a, b))
        PI.append(sel(t.pi_project, a, b))
    return LivePlan(bounds, B, Cv, I, PI, cont, cut, ranks, moved)


# ---------------------------------------------------------------------------------- collectives
import threading  # noqa: E402

_local = threading.local()


class use_group:
    """``with use_group(g):`` - this thread's collectives go to process group g (the sharded bench
    step runs each analysis' driver in its own thread, over its own group of all ranks: collectives
    of different drivers never interleave on one communicator)."""

    def __init__(self, group):
        self.group = group

    def __enter__(self):
        self.prev = getattr(_local, "group", None)
        _local.group = self.group
        return self

    def __exit__(self, *exc):
        _local.group = self.prev


def _group():
    return getattr(_local, "group", None)


def _dist():
    import torch.distributed as dist
    return dist


def _staged(x) -> bool:
    # RCCL ("nccl") takes device tensors directly; gloo (CPU tests, one-GPU rehearsals with several
    # ranks on one device) only host tensors for all_gather - stage device tensors through the host
    return x.is_cuda and _dist().get_backend() == "gloo"


def all_reduce(x, op=None):
    """In-place all-reduce (default SUM)."""
    dist = _dist()
    op = dist.ReduceOp.SUM if op is None else op
    if _staged(x):
        h = x.cpu()
        dist.all_reduce(h, op=op, group=_group())
        x.copy_(h)
    else:
        dist.all_reduce(x, op=op, group=_group())


def all_gather(x):
    """All-gather of equal-shape tensors -> list in rank order (on x's device)."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    if _staged(x):
        h = x.cpu()
        outs = [torch.empty_like(h) for _ in range(world)]
        dist.all_gather(outs, h, group=_group())
        return [o.to(x.device) for o in outs]
    outs = [torch.empty_like(x) for _ in range(world)]
    dist.all_gather(outs, x, group=_group())
    return outs


def _small(vals, dtype, device):
    """A few host numbers as a device tensor without a blocking copy: staged in pinned memory (torch's
    caching host allocator) and copied asynchronously on the current stream - torch.tensor(...,
    device=) from pageable memory waits for the stream's earlier work to finish first."""
    import torch
    t = torch.tensor(vals, dtype=dtype)
    if device is None or torch.device(device).type == "cpu":
        return t
    return t.pin_memory().to(device, non_blocking=True)


def _upload(a: np.ndarray, device):
    """A host numpy array to the device asynchronously (pinned staging, as _small)."""
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(device, non_blocking=True)


def all_gather_v(x):
    """All-gather of a 1-D tensor whose length differs per rank -> list (rank order) of tensors."""
    import torch
    n = _small([x.numel()], torch.int64, x.device)
    sizes = [int(v) for v in torch.cat(all_gather(n)).tolist()]
    m = max(max(sizes), 1)
    buf = torch.zeros(m, dtype=x.dtype, device=x.device)
    buf[:x.numel()] = x.reshape(-1)
    return [o[:k] for o, k in zip(all_gather(buf), sizes)]


def all_to_all_v(x, send_counts, recv_counts=None):
    """Variable all-to-all of a 1-D tensor: x holds the rows for rank 0, then rank 1, ...
    (send_counts[d] rows each) -> the rows every rank sent here, in source-rank order.
    recv_counts: what each rank sends here, when the caller knows it (no count exchange)."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    if recv_counts is None:
        sc = _small([int(v) for v in send_counts], torch.int64, x.device)
        rc = torch.cat(all_gather(sc)).reshape(world, world)[:, dist.get_rank()]
        recv_counts = rc.tolist()
    recv = [int(v) for v in recv_counts]
    send = [int(v) for v in send_counts]
    if _staged(x):
        h = x.cpu()
        out = torch.empty(sum(recv), dtype=x.dtype)
        dist.all_to_all_single(out, h, recv, send, group=_group())
        return out.to(x.device)
    out = torch.empty(sum(recv), dtype=x.dtype, device=x.device)
    dist.all_to_all_single(out, x.contiguous(), recv, send, group=_group())
    return out


_NP_DTYPES = {}
# above this many bytes a read goes through one concatenation and a DMA copy instead: kernel stores
# into host memory win for the small per-step reads, the copy engine for bulk (a Zipf giant's
# millions of session offsets)
_GATHER_MAX_BYTES = 4 << 20


def _host_many_dma(ts, dev):
    import torch

    def flat1(t):  # (1-D, unit stride: a one-element column slice can keep its row stride)
        x = t.reshape(-1)
        if x.stride(0) != 1 or not x.numel():
            x = torch.empty(x.numel(), dtype=x.dtype, device=x.device).copy_(x)
        return x.view(torch.uint8)
    flat = [flat1(t) for t in dev]
    h = torch.cat(flat).cpu().numpy()
    out, o, k = [], 0, 0
    for t in ts:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            nb = flat[k].numel()
            dt = _NP_DTYPES.get(t.dtype)
            if dt is None:
                dt = _NP_DTYPES[t.dtype] = torch.empty(0, dtype=t.dtype).numpy().dtype
            out.append(h[o:o + nb].view(dt).reshape(tuple(t.shape)))
            o += nb
            k += 1
        else:
            out.append(t.numpy().copy() if isinstance(t, torch.Tensor) else np.asarray(t))
    return out


def host_many(*ts):
    """Host numpy copies of several tensors (numpy arrays pass through) with ONE device->host read:
    each separate ``.cpu()`` would drain the stream once.  Device tensors go through libfz's
    fz_gather_to_host (one launch over every piece - strided 1-D slices read in place - into a
    pinned area, one sync); CPU tensors (the gloo tests' shards) are copied directly."""
    import torch
    dev = [t for t in ts if isinstance(t, torch.Tensor) and t.is_cuda]
    if not dev:
        return [t.numpy().copy() if isinstance(t, torch.Tensor) else np.asarray(t) for t in ts]
    if sum(t.numel() * t.element_size() for t in dev) > _GATHER_MAX_BYTES:
        return _host_many_dma(ts, dev)
    import ctypes as C
    from . import engine as E
    lib = E.load_library()
    keep, pieces, o = [], [], 0
    for t in dev:
        n, e = t.numel(), t.element_size()
        if n <= 1 or t.is_contiguous():
            stride = 1
        elif t.dim() == 1 and t.stride(0) > 0:
            stride = t.stride(0)
        else:  # (a strided block: one contiguous copy)
            t = t.contiguous()
            stride = 1
        keep.append(t)
        o = (o + 7) & ~7
        pieces.append(E.FzHostPiece(t.data_ptr() if n else None, n, max(stride, 1), o, e, 0))
        o += n * e
    buf = np.empty(max(o, 1), np.uint8)
    arr = (E.FzHostPiece * len(pieces))(*pieces)
    with torch.cuda.device(dev[0].device):
        stream = torch.cuda.current_stream(dev[0].device).cuda_stream
        E._check(lib, lib.fz_gather_to_host(C.c_void_p(stream), arr, len(pieces), C.c_void_p(buf.ctypes.data), o))
    out, k = [], 0
    for t in ts:
        if isinstance(t, torch.Tensor) and t.is_cuda:
            p = pieces[k]
            dt = _NP_DTYPES.get(t.dtype)
            if dt is None:
                dt = _NP_DTYPES[t.dtype] = torch.empty(0, dtype=t.dtype).numpy().dtype
            out.append(buf[p.dst_offset:p.dst_offset + p.n * p.elem_bytes].view(dt).reshape(tuple(t.shape)))
            k += 1
        else:
            out.append(t.numpy().copy() if isinstance(t, torch.Tensor) else np.asarray(t))
    return out


class Deferred:
    """A driver's result whose device values are copied to the host later, together with other
    drivers' (``finalize_all``): the sharded step then issues every driver's launches and
    collectives from one host thread in a fixed order - the same collective order on every rank -
    and drains the GPU once at the end instead of once per driver."""

    def __init__(self, tensors, finish):
        self.tensors, self.finish = list(tensors), finish

    def result(self):
        return self.finish(host_many(*self.tensors))


def finalize_all(ds):
    """The results of several Deferred (or plain values, passed through) with ONE device->host copy."""
    pend = [d for d in ds if isinstance(d, Deferred)]
    h = host_many(*[t for d in pend for t in d.tensors]) if pend else []
    out, o = [], 0
    for d in ds:
        if isinstance(d, Deferred):
            k = len(d.tensors)
            out.append(d.finish(h[o:o + k]))
            o += k
        else:
            out.append(d)
    return out


def _i64(x):
    """int64 image of a column for packing: float64 bit patterns travel unchanged."""
    import torch
    return x.view(torch.int64) if x.dtype == torch.float64 else x.to(torch.int64)


def _unpack(m, dtypes):
    import torch
    return [m[:, j].contiguous().view(torch.float64) if dt == torch.float64 else m[:, j].contiguous()
            for j, dt in enumerate(dtypes)]


def all_gather_cols(cols):
    """All-gather of k equal-length columns (int / float64) as ONE variable-size collective (a
    row-major [n, k] int64 block) -> per rank, the list of its k columns (dtypes restored)."""
    import torch
    dts = [c.dtype if c.dtype == torch.float64 else torch.int64 for c in cols]
    block = torch.stack([_i64(c) for c in cols], 1).reshape(-1)
    return [_unpack(p.reshape(-1, len(cols)), dts) for p in all_gather_v(block)]


def all_to_all_cols(cols, send_counts):
    """Variable all-to-all of k equal-length columns (rows grouped by destination rank) as ONE
    collective -> the k columns of the rows every rank sent here, in source-rank order."""
    import torch
    dts = [c.dtype if c.dtype == torch.float64 else torch.int64 for c in cols]
    k = len(cols)
    block = torch.stack([_i64(c) for c in cols], 1).reshape(-1)
    got = all_to_all_v(block, [int(v) * k for v in send_counts])
    return _unpack(got.reshape(-1, k), dts)


def agree_max(v: int, device=None) -> int:
    """MAX over ranks of a host integer (e.g. the RQ1 iteration-axis length, agreed once per load
    so every rank's per-iteration buffers have the same shape)."""
    import torch
    x = torch.tensor([int(v)], dtype=torch.int64, device=device)
    all_reduce(x, _dist().ReduceOp.MAX)
    return int(x.item())


# ----------------------------------------------------------------------------------------- RQ1
def rq1_sharded(shard, rank: int, world: int):
    """Exact RQ1 over project shards.  ``shard.run(ext)`` returns a dict of tensors (one device):
    counts[RQ1_NCOUNTS] int64, iter_total / iter_detected [M] int64 (M agreed across ranks),
    number / build_time int64 of this rank's matches (ORDER BY project, rts); ext is None or
    (number, build_time, before) tensors of competing matches from other ranks.
    ``shard.finish(counts, iter_total, iter_detected)`` recomputes the finishing counters in place.
    Returns (part, counts, iter_total, iter_detected, reran) - part = the final local run."""
    import torch
    dist = _dist()
    part = shard.run(None)
    reran = False
    if world > 1:
        if "number" not in part:  # (the GPU shard gathers the matches' numbers / times on demand)
            part.update(shard.numbers(part))
        got = all_gather_cols([part["number"], part["build_time"]])
        mine = part["number"]
        others = [r for r in range(world) if r != rank and got[r][0].numel()]
        if others and mine.numel():
            nums = torch.cat([got[r][0] for r in others])
            bts = torch.cat([got[r][1] for r in others])
            before = torch.cat([torch.full((got[r][0].numel(),), 1 if r < rank else 0, dtype=torch.uint8,
                                           device=mine.device) for r in others])
            hit = torch.isin(nums, mine)
            if bool(hit.any()):  # issue numbers shared with another shard: re-run with competitors
                part = shard.run((nums[hit], bts[hit], before[hit]))
                reran = True
    counts = part["counts"].clone()
    it, idt = part["iter_total"].clone(), part["iter_detected"].clone()
    if world > 1:  # one all-reduce: counters and both per-iteration tables
        M = it.numel()
        block = torch.cat([counts, it, idt])
        all_reduce(block)
        counts, it, idt = block[:RQ1_NCOUNTS].clone(), block[RQ1_NCOUNTS:RQ1_NCOUNTS + M].clone(), \
            block[RQ1_NCOUNTS + M:].clone()
        counts[RQ1_MAX_ITER] = (it > 0).sum()  # iter_total is non-increasing: its support is the max
    shard.finish(counts, it, idt)
    return part, counts, it, idt, reran


# ----------------------------------------------------------------------------------------- RQ3
RQ3_DET_F = ("det_pct",)
RQ3_DET_I = ("det_cov", "det_tot", "det_project", "det_issue")
RQ3_NON_F = ("non_pct",)
RQ3_NON_I = ("non_cov", "non_tot")


def rq3_sharded(shard, rank: int, world: int):
    """Exact RQ3 over project shards.  ``shard.run()`` runs with FZ_RQ3_FLUSH_LAST and returns
    counts[RQ3_NCOUNTS] int64 plus the det_* / non_* columns (sliced to their lengths);
    ``shard.stats(det_pct, det_tot, non_pct)`` runs the statistics over the gathered samples.
    Returns (counts, columns dict, stats) - columns in global project order.  At world 1 (one piece,
    no concatenation) the columns ALIAS the shard's persistent buffers: they are valid until the
    shard's next run; a caller that keeps a step's samples past that clones them."""
    import torch
    part = shard.run()
    counts = part["counts"]
    if world > 1:
        cl = host_many(*all_gather(counts))
        cols = {}
        for keys in (RQ3_DET_F + RQ3_DET_I, RQ3_NON_F + RQ3_NON_I):
            got = all_gather_cols([part[k] for k in keys])
            for j, k in enumerate(keys):
                cols[k] = [got[r][j] for r in range(world)]
    else:  # (a shard that read its counters already hands over the host copy)
        cl = [part["counts_h"]] if "counts_h" in part else host_many(counts)
        cols = {k: [part[k]] for k in RQ3_DET_F + RQ3_DET_I + RQ3_NON_F + RQ3_NON_I}
    with_issues = [r for r in range(world) if cl[r][RQ3_ISSUES] > 0]
    last = with_issues[-1] if with_issues else -1
    if last >= 0:  # the globally last issue-bearing project is never flushed (rq3:245-257)
        drop = int(cl[last][RQ3_NON_LAST])
        for k in RQ3_NON_F + RQ3_NON_I:
            v = cols[k][last]
            cols[k][last] = v[:v.numel() - drop]
    out = {k: (torch.cat(v) if len(v) > 1 else v[0]) for k, v in cols.items()}
    total = np.sum(np.stack(cl), axis=0)
    total[RQ3_DETECTED] = out["det_pct"].numel()
    total[RQ3_NON_DETECTED] = out["non_pct"].numel()
    total[RQ3_NON_LAST] = 0
    # NULL total_line pairs (rq3:253,297 raise TypeError): those of the never-flushed last project
    # do not count; the rest raise below (as compute.rq3_result does on one table)
    total[RQ3_NULL_TOTAL] -= int(cl[last][RQ3_NULL_LAST]) if last >= 0 else 0
    total[RQ3_NULL_LAST] = 0
    if total[RQ3_NULL_TOTAL] > 0:  # None > 0 (rq3:253,297): every rank holds the counters, all raise here
        raise TypeError("'>' not supported between instances of 'NoneType' and 'int'")
    st = shard.stats(out["det_pct"], out["det_tot"], out["non_pct"])
    return total, out, st


# ------------------------------------------------------------------------------------- RQ2 add
RQ2A_ROW_COLS = ("row_project", "row_first_build", "row_end_build", "row_start_build", "row_cov_i", "row_cov_i1",
                 "diff_total", "diff_coverage")
RQ2A_FLAGS = ("eligible", "covered_is_float", "total_is_float")


def rq2_add_sharded(shard, rank: int, world: int):
    """Exact RQ2 add over project shards.  rq2_coverage_and_added.py:73-238 runs one project at a
    time - a project's change rows read only its own Coverage builds and coverage rows - so the
    result is the shards' rows concatenated in rank (= project) order, and the per-project flags
    (eligible, the covered / total float upcasts) summed over disjoint project ranges (= OR).
    ``shard.run()`` returns the flags [P] and the RQ2A_ROW_COLS columns of this rank's rows (row ids
    in whatever id space the caller wants gathered).  Returns (flags dict of [P] int64, rows dict)."""
    import torch
    part = shard.run()
    flags = torch.stack([part[k].to(torch.int64) for k in RQ2A_FLAGS])
    if world > 1:
        all_reduce(flags)
    rows = gather_rows({k: part[k] for k in RQ2A_ROW_COLS}, world)
    return dict(zip(RQ2A_FLAGS, flags)), rows


# ------------------------------------------------------------------------------ session exchange
def merge_runs_torch(vals, runs):
    """fz_runs_merge on any device with torch ops (the CPU tests' shards): vals = R runs one after
    another, each grouped by segment; runs [R, S] their sizes -> (values segment by segment, run
    order inside a segment; offsets [S + 1])."""
    import torch
    R, S = runs.shape
    sz = runs.reshape(-1).tolist()
    st = np.concatenate([[0], np.cumsum(sz)]).astype(np.int64)
    pieces = [vals[st[r * S + s]:st[r * S + s] + sz[r * S + s]] for s in range(S) for r in range(R)]
    out = torch.cat(pieces) if pieces else vals[:0]
    offs = torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(runs.sum(0).to(torch.int64).cpu(), 0)])
    return out, offs.to(vals.device)


def exchange_grouped(shard, vals, offs_h, mat, mat_h, own, rank, k=1):
    """Send this rank's segment-grouped values (k segments per session: offs_h its host offsets) to
    the owners of their sessions and merge what arrives.  mat [world, k * M] (device) / mat_h (host):
    every rank's segment sizes; own: the owners' session ranges.  One all-to-all whose receive
    counts come from mat (no count exchange), then shard.merge_runs -> (values of the sessions
    [a, b) this rank owns, grouped by segment with the sources in rank order; offsets)."""
    n_loc = len(offs_h) - 1
    a, b = own[rank]
    send = [int(offs_h[min(k * hi, n_loc)] - offs_h[min(k * lo, n_loc)]) for lo, hi in own]
    recv = [int(v) for v in mat_h[:, k * a:k * b].sum(1)]
    got = all_to_all_v(vals, send, recv)
    return shard.merge_runs(got, mat[:, k * a:k * b].contiguous())


# ----------------------------------------------------------------------------------- RQ2 count
RQ2C_PROJECT_COLS = ("eligible", "raw_n", "n_trend", "sw_w", "sw_p", "corr")


def session_owners(sizes: np.ndarray, world: int) -> List[Tuple[int, int]]:
    """Contiguous session-index ranges, one per rank, with about equal numbers of values (session
    sizes are non-increasing, so equal index ranges would not balance)."""
    M = len(sizes)
    cum = np.concatenate([[0], np.cumsum(sizes)])
    cuts = [0]
    for r in range(1, world):
        k = int(np.searchsorted(cum, cum[-1] * r / world, "left"))
        cuts.append(min(max(k, cuts[-1]), M))
    cuts.append(M)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def _owner_cuts(lengths: np.ndarray, world: int, M: int) -> List[Tuple[int, int]]:
    """session_owners from the runs' lengths alone (O(projects), no per-session array): session i
    holds one value of every run longer than i, so the values of sessions [0, k) number
    cum(k) = sum(min(len, k)) - cut at the equal-values targets, as session_owners does."""
    L = np.sort(np.asarray(lengths, np.int64)[np.asarray(lengths) > 0])
    S = np.concatenate([[0], np.cumsum(L)]).astype(np.int64)

    def cum(k):
        j = int(np.searchsorted(L, k, "right"))
        return int(S[j]) + k * (len(L) - j)
    total = cum(M)
    cuts = [0]
    for r in range(1, world):
        x = total * r / world
        a, b = 0, M  # smallest k with cum(k) >= x
        while a < b:
            m = (a + b) // 2
            if cum(m) >= x:
                b = m
            else:
                a = m + 1
        cuts.append(min(max(a, cuts[-1]), M))
    cuts.append(M)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


@dataclass
class _Runs:
    """The project-major exchange of one analysis: every rank's runs (a project's values in date
    order and the session they start at), from per-project counts gathered once."""
    world: int
    bounds: List[Tuple[int, int]]   # each rank's own project range
    n_loc: np.ndarray                # [P] values of each project on its owner (its only / first piece)
    cont: np.ndarray                 # [world] the cut project leading each rank's rows (-1)
    cont_n: np.ndarray               # [world] that piece's values
    n: np.ndarray = None             # [P] global values per project
    cont_base: np.ndarray = None     # [world] the session the leading piece starts at

    def __post_init__(self):
        self.n = self.n_loc.copy()
        self.cont_base = np.zeros(self.world, np.int64)
        for r in range(self.world):
            p = int(self.cont[r])
            if p >= 0:
                # (the earlier pieces' values, owner's first; a one-GPU rehearsal of one shard has
                # no earlier piece: its leading piece starts at session 0, its runs are what it packs)
                self.cont_base[r] = self.n[p]
                self.n[p] += int(self.cont_n[r])

    def runs_of(self, r):
        """[R, 4] int64 rows (src, src_off, len, base) of rank r's runs in project order: its leading
        piece (src 1: fz_piece_values' buffer), then its own projects (src 0: the project-major
        values)."""
        a, b = self.bounds[r]
        nl = np.asarray(self.n_loc[a:b], np.int64)
        off = np.cumsum(nl) - nl
        k = np.nonzero(nl > 0)[0]
        out = np.zeros((len(k), 4), np.int64)
        out[:, 1], out[:, 2] = off[k], nl[k]
        if self.cont[r] >= 0 and self.cont_n[r] > 0:
            lead = np.array([[1, 0, int(self.cont_n[r]), int(self.cont_base[r])]], np.int64)
            out = np.concatenate([lead, out])
        return out

    @staticmethod
    def slices(runs, own):
        """[dest, run] values of each run in each destination's session range."""
        runs = np.asarray(runs, np.int64).reshape(-1, 4)
        if not len(runs):
            return np.zeros((len(own), 0), np.int64)
        base = runs[:, 3]
        end = base + runs[:, 2]
        a = np.array([o[0] for o in own], np.int64)[:, None]
        b = np.array([o[1] for o in own], np.int64)[:, None]
        return np.maximum(0, np.minimum(end[None], b) - np.maximum(base[None], a))


def _exchange_runs(shard, runs: _Runs, rank, own, a_vals, b_vals, group_of=None):
    """Send this rank's runs to the owners of their sessions (one all-to-all of packed slices,
    fz_pack_runs) and transpose what arrives (fz_transpose_runs) -> (the owner's values grouped by
    segment (session, group), offsets [S * G + 1]).  group_of: [P] run group (0 = G2, 1 = G1) or
    None (one group)."""
    import torch
    world = runs.world
    mine = runs.runs_of(rank)
    sl = _Runs.slices(mine, own)                      # [world, R]
    send = sl.sum(1)
    a, b = own[rank]
    recv = np.array([_Runs.slices(mine if s == rank else runs.runs_of(s), [own[rank]])[0].sum()
                     for s in range(world)], np.int64)
    if world > 1:
        packed = shard.pack(a_vals, b_vals, mine, sl, own, int(send.sum()))
        got = all_to_all_v(packed, send.tolist(), recv.tolist())
    elif not np.any(mine[:, 0]):  # (one rank, no leading piece: the project-major values ARE its runs)
        got = a_vals[:int(send.sum())]
    else:  # (one rank with a leading piece: that piece's run first, then its own projects')
        got = shard.pack(a_vals, b_vals, mine, sl, own, int(send.sum()))
    # the owner's runs: every project longer than its first session, in project order (a cut
    # project's pieces arrive one after another, in date order: one run)
    n = runs.n
    live = np.nonzero(n > a)[0]
    lens = np.minimum(n[live], b) - a
    roffs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    # (every rank derives the same runs from the same gathered counts: what arrives is exactly what
    # the owner's runs hold - checked before any kernel reads it)
    if int(recv.sum()) != int(roffs[-1]) or int(got.numel()) < int(roffs[-1]):
        raise RuntimeError(f"session exchange: {int(got.numel())} values received for runs of {int(roffs[-1])} "
                           f"(sessions [{a}, {b}))")
    grp = None if group_of is None else np.asarray(group_of)[live].astype(np.uint8)
    return shard.transpose(got, roffs, grp, b - a)


def _series_tests_cut(shard, p, holders, piece, base, n, rank, dev):
    """spearmanr(range(n), x) / shapiro(x) (rq2_coverage_count.py:305-322) of cut project p, whose
    n values lie in date-range pieces on the ranks `holders` (this rank's piece: `piece` from series
    index `base`, or None).  Value buckets over the holders from a sorted sample of every piece
    (ties never cross a bucket: a value goes to the first bucket whose upper splitter it does not
    exceed), one all-to-all of (value, series index), a sort per bucket, then the three passes of
    partial sums and their ordered combination (fz_series_dist_*) -> device [4] (rho, p, W, p) on
    every rank."""
    import torch
    k = len(holders)
    j = holders.index(rank) if rank in holders else -1
    f64 = torch.float64
    if j >= 0 and piece.numel():
        val, pos = shard.sort(piece)
        gidx = pos.to(torch.int64) + base
        m = val.numel()
        ns = min(256, m)
        samp = val[torch.div(torch.arange(ns, device=val.device) * m, ns, rounding_mode="floor")]
        head = _small([float(m)], f64, val.device)
    else:
        val = torch.zeros(0, dtype=f64, device=dev)
        gidx = torch.zeros(0, dtype=torch.int64, device=dev)
        samp = val
        head = torch.zeros(0, dtype=f64, device=dev)
    got = all_gather_v(torch.cat([head, samp.to(f64)]))
    gh = host_many(*got)
    xs, ws = [], []
    for g in gh:
        if len(g):
            m_r, s_r = int(g[0]), g[1:]
            xs.append(s_r)
            ws.append(np.full(len(s_r), m_r / max(len(s_r), 1)))
    xs = np.concatenate(xs) if xs else np.zeros(0)
    ws = np.concatenate(ws) if ws else np.zeros(0)
    o = np.argsort(xs, kind="stable")
    xs, cw = xs[o], np.cumsum(ws[o])
    tot = cw[-1] if len(cw) else 0.0
    spl = np.array([xs[min(int(np.searchsorted(cw, tot * q / k, "left")), len(xs) - 1)] for q in range(1, k)]
                   if len(xs) else np.zeros(0))
    # this piece's bucket boundaries, every rank's (the all-to-all's counts)
    if j >= 0 and val.numel():
        sd = torch.as_tensor(spl, dtype=f64, device=val.device)
        bnd = torch.searchsorted(val, sd, right=True) if len(spl) else torch.zeros(0, dtype=torch.int64, device=dev)
        bnd = torch.cat([torch.zeros(1, dtype=torch.int64, device=val.device), bnd.to(torch.int64),
                         _small([val.numel()], torch.int64, val.device)])
    else:
        bnd = torch.zeros(k + 1, dtype=torch.int64, device=dev)
    allb = host_many(*all_gather(bnd))                 # [world][k + 1]
    world = len(allb)
    cnt = np.stack([np.diff(x) for x in allb])          # [world, k]: source -> bucket
    sizes = cnt.sum(0)
    send = np.zeros(world, np.int64)
    recv = np.zeros(world, np.int64)
    for q, h in enumerate(holders):
        send[h] = cnt[rank, q] if j >= 0 else 0
    if j >= 0:
        recv[:] = cnt[:, j]
    rv = all_to_all_cols([val, gidx], send.tolist()) if world > 1 else [val, gidx]
    m = int(sizes[j]) if j >= 0 else 0
    g0 = int(sizes[:j].sum()) if j >= 0 else 0
    if j >= 0 and m:
        v2, p2 = shard.sort(rv[0])
        g2 = rv[1][p2.to(torch.int64)]
    else:
        v2, g2 = torch.zeros(0, dtype=f64, device=dev), torch.zeros(0, dtype=torch.int64, device=dev)
    # scipy's y -= x[N // 2]: the series value at index n // 2, from the piece holding it
    x0 = None
    if j >= 0 and piece is not None and base <= n // 2 < base + piece.numel():
        x0 = piece[n // 2 - base:n // 2 - base + 1]
    params, result = shard.dist_state()
    for ps in range(3):
        part = shard.dist_partials(ps, v2, g2, m, g0, n, params, x0 if ps == 0 else None) if j >= 0 else \
            torch.zeros(0, dtype=f64, device=dev)
        parts = torch.cat(all_gather_v(part)) if world > 1 else part
        shard.dist_combine(ps, parts, k, n, params, result, sizes)
    return result


def rq2_count_sharded(shard, rank: int, world: int, lo: int, hi: int, gather_values: bool = True,
                      finish_later: bool = False, cont: int = -1, host_sessions: bool = True):
    """Exact RQ2 count over project shards (rq2_coverage_count.py:244-483).
    ``shard.run()`` -> per-project columns over the global project axis (RQ2C_PROJECT_COLS), the
    local trend values project-major ("values": the eligible projects' values in (project, date)
    order, n_trend[p] each), "null_lines"; with a leading piece of cut project `cont`,
    "piece_values" / "piece_counts" (fz_piece_values).  Exchange (project-major, _exchange_runs):
    per-project columns and the pieces' counts gathered, each rank's runs sent to the owners of their
    sessions (one all-to-all), the owner's transpose + session statistics
    (``shard.session_stats_grouped``), per-session results gathered; a cut project's tests from its
    pieces (_series_tests_cut).  host_sessions=False leaves the per-session rows on their owners'
    devices ("sessions": the owner's session range and its average / median / percentile columns -
    config 5L's 20.8 M sessions are 1.2 GB) as the single-table step leaves its results in HBM; only
    the medians of sessions [0, K) the tail reads are gathered.  Returns a dict of host numpy arrays
    (every rank)."""
    import torch
    part = shard.run()
    vals_a = part["values"]
    dev = vals_a.device
    # (every rank's own range gathered into the global axis; one rank - a one-GPU rehearsal of one
    # shard too - keeps its columns over the global axis: the other ranks' projects are absent, zero)
    pc = [part[k][lo:hi] if world > 1 else part[k] for k in RQ2C_PROJECT_COLS]
    pc = [v.to(torch.float64) if v.is_floating_point() else v.to(torch.int64) for v in pc]
    nl = part.get("null_lines")
    nl = nl.to(torch.int64).reshape(-1)[:1] if nl is not None else torch.zeros(1, dtype=torch.int64, device=dev)
    vals_b = part.get("piece_values")
    pcnt = part.get("piece_counts")
    if pcnt is None or cont < 0:
        pcnt = torch.zeros(3, dtype=torch.int64, device=dev)
    info = torch.cat([_small([cont, lo, hi], torch.int64, dev), pcnt.to(torch.int64), nl])
    if world > 1:
        got = all_gather_cols(pc)
        pc = [torch.cat([got[r][j] for r in range(world)]) for j in range(len(pc))]
        info_all = torch.stack(all_gather(info))
    else:
        info_all = info[None]
    h = host_many(info_all, *pc)  # one device->host copy
    info_h = h[0]
    proj = dict(zip(RQ2C_PROJECT_COLS, h[1:]))
    bounds = [(int(x[1]), int(x[2])) for x in info_h]
    conts, cont_n, cont_raw = info_h[:, 0], info_h[:, 3], info_h[:, 4]
    null_lines = int(info_h[:, 5].sum() + info_h[:, 6].sum())
    if null_lines:  # float(None) (rq2_coverage_count.py:300-303): every rank holds the sum, all raise here
        raise TypeError("float() argument must be a string or a real number, not 'NoneType'")
    runs = _Runs(world, bounds, proj["n_trend"].astype(np.int64), conts.astype(np.int64), cont_n.astype(np.int64))
    # a cut project's columns: counts summed over its pieces, tests from all of its values
    cut = sorted({int(p) for p in conts.tolist() if p >= 0})
    for p in cut:
        proj["raw_n"][p] += int(cont_raw[conts == p].sum())
        proj["n_trend"][p] = runs.n[p]
    M = max(1, int(runs.n.max()) if len(runs.n) else 0)  # (sessions start as [[]], :285)
    own = _owner_cuts(runs.n, world, M)
    a, b = own[rank]
    S = b - a
    if getattr(shard, "session_major", False):
        # one rank, no leading piece (a one-GPU run of the sharded step): the local kernels wrote the
        # values session-major with their offsets (the single-table transpose, in the recorded local
        # phase) - no runs, no host-built transpose after the read
        if world != 1 or cont >= 0:
            raise ValueError("rq2_count_sharded: session-major shard output serves one rank without a cut project")
        vals, goffs = vals_a[:int(runs.n.sum())], part["session_offsets"][:M + 1]
    else:
        vals, goffs = _exchange_runs(shard, runs, rank, own, vals_a, vals_b)
    st = shard.session_stats_grouped(vals, goffs, S, len(proj["eligible"]))
    # sessions with >= 100 values: a prefix, as long as the 100th longest run (:390)
    srt = np.sort(runs.n)[::-1]
    K = int(srt[99]) if len(srt) >= 100 else 0
    K = min(K, M)
    med_k = None
    if host_sessions:
        block = torch.cat([st["average"][:S, None], st["median"][:S, None], st["percentiles"][:5 * S].reshape(S, 5)],
                          1)
        if world > 1:  # per-session rows (average, median, 5 percentiles) of every owner, session order
            block = torch.cat([m.reshape(-1, 7).view(torch.float64) for m in all_gather_v(block.reshape(-1).view(
                torch.int64))])
    else:
        # the per-session rows stay on their owners (session range own[rank]); the tail's median
        # trend needs sessions [0, K) only: each owner's part of that prefix gathered
        block = torch.zeros((0, 7), dtype=torch.float64, device=dev)
        if world > 1:
            kk = max(0, min(b, K) - a)
            med_k = torch.cat(all_gather_v(st["median"][:kk].contiguous().view(torch.int64))).view(torch.float64)
    for p in cut:  # its Spearman / Shapiro-Wilk over every piece (:305-322), patched on every rank
        holders = [r for r in range(world) if bounds[r][0] <= p < bounds[r][1] or conts[r] == p]
        if world == 1:
            holders = [0]
        if rank in holders:
            if bounds[rank][0] <= p < bounds[rank][1]:
                off = int(runs.n_loc[bounds[rank][0]:p].sum())
                piece, base = vals_a[off:off + int(runs.n_loc[p])], 0
            else:
                piece, base = vals_b[:int(cont_n[rank])], int(runs.cont_base[rank])
        else:
            piece, base = None, 0
        res = host_many(_series_tests_cut(shard, p, holders, piece, base, int(runs.n[p]), rank, dev))[0]
        proj["corr"][p], proj["sw_w"][p], proj["sw_p"][p] = res[0], res[2], res[3]
        for j, key in ((5, "corr"), (3, "sw_w"), (4, "sw_p")):
            pc[j][p] = float(proj[key][p])
        pc[1][p] = int(proj["raw_n"][p])
        pc[2][p] = int(proj["n_trend"][p])
    if hasattr(shard, "tail"):  # one library call (fz_rq2_count_tail), device in and out
        med = st["median"][:S] if world == 1 else (med_k if med_k is not None else block[:, 1].contiguous())
        tail = shard.tail(med, K, pc[5], pc[1], pc[0])
        tests, corr_mm = tail[:4], tail[4:6]
    else:
        med = st["median"][:S] if world == 1 else (med_k if med_k is not None else block[:, 1])
        tests = shard.series_tests(med[:K].contiguous())  # median trend of the sessions with >= 100 values
        elig = proj["eligible"] != 0
        corr = proj["corr"][elig][proj["raw_n"][elig] > 0]
        valid = corr[~np.isnan(corr)]
        corr_mm = shard.mean_median(torch.from_numpy(valid.copy()).to(dev))
    tensors = [block if host_sessions else block[:0], tests, corr_mm]
    if gather_values:  # coverage_by_session_index.csv: every value, session-major, project order
        tensors.append(torch.cat(all_gather_v(vals)) if world > 1 else vals)
    n_glob = runs.n

    def finish(h):  # (the one result copy)
        blk = h[0]
        out = {"proj": proj, "K": K, "average": blk[:, 0].copy(), "median": blk[:, 1].copy(),
               "percentiles": blk[:, 2:].reshape(-1).copy(), "tests": tuple(float(v) for v in h[1]),
               "corr_mm": tuple(float(v) for v in h[2]), "null_lines": null_lines}
        if not host_sessions:  # (this owner's sessions [a, b): device columns)
            out["sessions"] = {"range": (a, b), "average": st["average"][:S], "median": st["median"][:S],
                               "percentiles": st["percentiles"][:5 * S]}
        if gather_values:
            out["session_values"] = h[3]
            sizes = np.zeros(M + 1, np.int64)  # session i holds one value of every run longer than i
            np.add.at(sizes, np.minimum(n_glob, M), 1)
            per = np.cumsum(sizes[::-1])[::-1][1:]
            out["session_offsets"] = np.concatenate([[0], np.cumsum(per)]).astype(np.int64)
        return out
    d = Deferred(tensors, finish)
    return d if finish_later else d.result()


# ----------------------------------------------------------------------------------------- RQ4a
RQ4A_MAX_ITER, RQ4A_HAS_WINDOW = 0, 6
RQ4A_TABLES = ("g1_total", "g1_det", "g2_total", "g2_det")


def rq4a_sharded(shard, rank: int, world: int, lo: int, hi: int, finish_later: bool = False):
    """Exact RQ4a over project shards (rq4a_bug.py:653-884).  ``shard.run()`` -> counts, the four
    per-iteration tables (length agreed across ranks), member / intro over the global project axis,
    g4_steps[30], g4_transition[4]; ``shard.finish(tables, intro, steps, counts)`` -> scalars (and
    the recomputed counters, in place).  Group sizes, counters and step/transition counts add over
    disjoint projects; the iteration axis is a MAX; HAS_WINDOW is an OR."""
    import torch
    part = shard.run()
    counts = part["counts"].clone()
    tables = [part[k].clone() for k in RQ4A_TABLES]
    steps, trans = part["g4_steps"].clone(), part["g4_transition"].clone()
    member = part["member"][lo:hi].to(torch.int64)
    intro = part["intro"][lo:hi].clone()
    if world > 1:  # one all-reduce (counters, tables, step and transition counts), one gather
        parts = [counts] + tables + [steps, trans]
        block = torch.cat(parts)
        all_reduce(block)
        out, o = [], 0
        for x in parts:
            out.append(block[o:o + x.numel()].clone())
            o += x.numel()
        counts, tables, steps, trans = out[0], out[1:5], out[5], out[6]
        # the longest G1/G2 build axis is the support of the summed totals; HAS_WINDOW is an OR
        counts[RQ4A_MAX_ITER] = ((tables[0] + tables[2]) > 0).sum()
        counts[RQ4A_HAS_WINDOW] = (counts[RQ4A_HAS_WINDOW] > 0).to(counts.dtype)
        got = all_gather_cols([member, intro])
        member = torch.cat([g[0] for g in got])
        intro = torch.cat([g[1] for g in got])
    sc = shard.finish(tables, intro, steps, counts)

    def finish(h):
        m = int(h[0][RQ4A_MAX_ITER])
        return {"counts": h[0], "scalars": np.asarray(h[1]), "member": h[2], "tables": [x[:m] for x in h[6:]],
                "intro": h[3], "g4_steps": h[4], "g4_transition": h[5]}
    d = Deferred([counts, sc, member, intro, steps, trans, *tables], finish)
    return d if finish_later else d.result()


# ----------------------------------------------------------------------------------------- RQ4b
(RQ4B_SESSIONS, RQ4B_LAST, RQ4B_DELTA_PROJECTS, RQ4B_INIT_G2, RQ4B_INIT_G1) = range(5)
RQ4B_VALUES = 9


def rq4b_sharded(shard, rank: int, world: int, lo: int = None, hi: int = None, finish_later: bool = False,
                 cont: int = -1, host_sessions: bool = True):
    """Exact RQ4b over project shards (rq4b_coverage.py:1209-1261).  ``shard.run()`` -> counts,
    member[P], the G1/G2 full coverage values project-major (trend_values, trend_offsets [P + 1]),
    the delta columns (pre_cov / post_cov step-major, delta_order = CSV row of each column; at least
    counts' lengths) and the initial-coverage samples; with a leading piece of cut project `cont`,
    "piece_values" / "piece_counts" (fz_piece_values, rq4b kind).  ``shard.session_stats_grouped``,
    ``shard.tail`` (or spearman_prefix / row_medians / two_sample) run the statistics.  Exchange:
    per-project members and series lengths over the rank's own range [lo, hi) gathered (default: the
    whole axis when world == 1), each rank's runs sent to their sessions' owners and transposed there
    by (session, group) (_exchange_runs), per-session results, delta columns (re-ordered by CSV row,
    :216, :744) and initial samples gathered.  Intermediates stay on the device; the results are
    copied to the host once (host_sessions=False: the per-session columns stay on their owners,
    "sessions"; only the prefix of sessions the trends read is gathered).  Returns a dict for rq/compute.rq4b_result (host arrays, every rank)."""
    import torch
    part = shard.run()
    counts = part["counts"].clone()
    dev = counts.device
    P = part["member"].numel()
    if lo is None:
        if world > 1:
            raise ValueError("rq4b_sharded: the rank's own project range (lo, hi) is needed at world > 1")
        lo, hi = 0, P
    heads = None
    if getattr(shard, "session_major", False):
        # one rank, no leading piece (a one-GPU run of the sharded step): the local kernels grouped
        # the values by (session, group) already (the single-table transpose, in the recorded local
        # phase) - no runs, no host-built transpose; one read of the sizes
        if world != 1 or cont >= 0:
            raise ValueError("rq4b_sharded: session-major shard output serves one rank without a cut project")
        head = torch.stack([counts[RQ4B_SESSIONS], counts[RQ4B_VALUES], counts[RQ4B_DELTA_PROJECTS],
                            counts[RQ4B_INIT_G2], counts[RQ4B_INIT_G1]])
        m_loc, nv, nd, n2, n1 = (int(v) for v in host_many(head)[0])
        heads = (nd, n2, n1)
        M = m_loc
        a, b = 0, M
        S = M
        st = shard.session_stats_grouped(part["trend_values"][:nv], part["trend_offsets"][:2 * M + 1], S, P)
    else:
        a = b = S = M = None
    if heads is None:
        M, a, b, S, st = _rq4b_exchange_stats(shard, part, rank, world, lo, hi, cont, counts, P, dev)
    # per-session rows (c2, c1, g2 quartiles, g1 quartiles, p_bm) of every owner, session order
    cols = [st["c2"][:S], st["c1"][:S]] + [st["g2_q"][:3 * S].reshape(S, 3)[:, j] for j in range(3)] + \
        [st["g1_q"][:3 * S].reshape(S, 3)[:, j] for j in range(3)] + [st["p_bm"][:S]]
    own_cols = cols
    if world > 1:
        if host_sessions:
            got = all_gather_cols(cols)
        else:
            # the trends read sessions with both groups >= 100 (:849-860): a prefix of length L, the
            # shorter of the two groups' 100th longest series - each owner's part of it gathered, the
            # per-session rows stay on their owners
            runs_n, group = shard._last_runs

            def hundredth(x):
                x = np.sort(x)[::-1]
                return int(x[99]) if len(x) >= 100 else 0
            L = min(hundredth(runs_n[group == 0]), hundredth(runs_n[group == 1]), M)
            kk = max(0, min(b, L) - a)
            got = all_gather_cols([x[:kk] for x in cols])
        cols = [torch.cat([g[j] for g in got]) for j in range(len(cols))]
    return _rq4b_finish(shard, part, world, counts, cols, own_cols, st, S, M, a, b, heads, finish_later,
                        host_sessions)


def _rq4b_exchange_stats(shard, part, rank, world, lo, hi, cont, counts, P, dev):
    """rq4b_sharded's project-major exchange: runs from the gathered series lengths, sent to the
    sessions' owners and transposed by (session, group) there, the owner's session statistics ->
    (M, a, b, S, stats).  (shard._last_runs: the global run lengths and groups, for the prefix the
    trends read.)"""
    import torch
    toffs = part["trend_offsets"][:P + 1]
    # (own ranges gathered into the global axis; one rank keeps its columns over the global axis)
    nloc = (toffs[1:] - toffs[:-1])[lo:hi] if world > 1 else toffs[1:] - toffs[:-1]
    nloc = nloc.to(torch.int64)
    member = (part["member"][lo:hi] if world > 1 else part["member"]).to(torch.int64)
    vals_a = part["trend_values"]
    vals_b = part.get("piece_values")
    pcnt = part.get("piece_counts")
    if pcnt is None or cont < 0:
        pcnt = torch.zeros(3, dtype=torch.int64, device=dev)
    info = torch.cat([_small([cont, lo, hi], torch.int64, dev), pcnt.to(torch.int64)])
    if world > 1:
        got = all_gather_cols([member, nloc])
        member = torch.cat([g[0] for g in got])
        nloc = torch.cat([g[1] for g in got])
        info_all = torch.stack(all_gather(info))
        all_reduce(counts)
    else:
        info_all = info[None]
    info_h, member_h, nloc_h = host_many(info_all, member, nloc)
    bounds = [(int(x[1]), int(x[2])) for x in info_h]
    conts, cont_n = info_h[:, 0].astype(np.int64), info_h[:, 3].astype(np.int64)
    # (a leading piece of a project outside G1 / G2 contributes no series)
    cont_n = np.where((conts >= 0) & ((member_h[np.maximum(conts, 0)] & 3) != 0), cont_n, 0)
    runs = _Runs(world, bounds, nloc_h.astype(np.int64), conts, cont_n)
    M = int(runs.n.max()) if len(runs.n) else 0
    own = _owner_cuts(runs.n, world, M) if world > 1 else [(0, M)]
    group = np.where((member_h & 2) != 0, 0, 1)  # G2 -> segment 2s, G1 -> 2s + 1
    vals, goffs = _exchange_runs(shard, runs, rank, own, vals_a, vals_b, group_of=group)
    shard._last_runs = (runs.n, group)
    a, b = own[rank]
    S = b - a
    return M, a, b, S, shard.session_stats_grouped(vals, goffs, S, P)


def _rq4b_finish(shard, part, world, counts, cols, own_cols, st, S, M, a, b, heads, finish_later, host_sessions):
    """rq4b_sharded after the per-session statistics: deltas, initial samples, the tail, the one
    result copy."""
    import torch
    # coverage deltas: columns of every rank (CSV row, 7 pre, 7 post), put in corpus CSV order below
    if heads is not None:
        nd, n2, n1 = heads
    else:
        nd, n2, n1 = (int(v) for v in host_many(torch.stack([part["counts"][RQ4B_DELTA_PROJECTS],
                                                              part["counts"][RQ4B_INIT_G2],
                                                              part["counts"][RQ4B_INIT_G1]]))[0])
    proj = part["delta_order"][:nd]
    pre = part["pre_cov"][:7 * nd].reshape(7, nd)
    post = part["post_cov"][:7 * nd].reshape(7, nd)
    if world > 1:  # one gather
        got = all_gather_cols([proj] + [pre[i] for i in range(7)] + [post[i] for i in range(7)])
        cat = [torch.cat([g[j] for g in got]) for j in range(15)]
        proj, pre, post = cat[0], torch.stack(cat[1:8]), torch.stack(cat[8:15])
    # initial coverage: samples in project order, tests once
    x, y = part["init_g2"][:n2], part["init_g1"][:n1]
    if world > 1:  # both samples in one variable gather: [len(x), x, y] per rank
        nx = _small([x.numel()], torch.int64, x.device)
        parts = all_gather_v(torch.cat([nx, x.contiguous().view(torch.int64), y.contiguous().view(torch.int64)]))
        heads = host_many(torch.stack([q[0] for q in parts]))[0]
        xs, ys = [], []
        for q, k in zip(parts, heads.tolist()):
            xs.append(q[1:1 + k].view(torch.float64))
            ys.append(q[1 + k:].view(torch.float64))
        x, y = torch.cat(xs), torch.cat(ys)
    if hasattr(shard, "tail"):
        # trends, delta columns in CSV order with their medians, initial-coverage tests: one library
        # call (fz_rq4b_tail), device in and out
        if world > 1:  # (the gathered quartile columns back to [session, 3] rows)
            g2q, g1q = torch.stack(cols[2:5], 1).reshape(-1), torch.stack(cols[5:8], 1).reshape(-1)
        else:
            g2q, g1q = st["g2_q"][:3 * S], st["g1_q"][:3 * S]
        last_d, sp, pre, post, med, tests = shard.tail(cols[0], cols[1], g2q, g1q, proj, pre, post, x, y)
    else:
        if hasattr(shard, "trends"):  # one library call (fz_rq4b_trends), device in and out
            last_d, sp = shard.trends(cols)
        else:
            c2d, c1d = cols[0], cols[1]
            # last session with both groups >= 100 (:849-860), on the device
            idx = torch.arange(c2d.numel(), dtype=torch.int64, device=c2d.device)
            ok = (c2d >= 100) & (c1d >= 100)
            last_d = torch.where(ok, idx, torch.full_like(idx, -1)).max() if c2d.numel() else torch.tensor(-1)
            # Spearman of G1 Q1 / Med / Q3, then G2 Q1 / Med / Q3 over sessions 0..last (:879-899)
            quart = torch.stack([cols[5], cols[6], cols[7], cols[2], cols[3], cols[4]]).to(torch.float64)
            sp = shard.spearman_prefix(quart, last_d + 1)
        order = torch.argsort(proj, stable=True)
        pre, post = pre[:, order], post[:, order]
        med = shard.row_medians(torch.cat([pre, post]).contiguous())
        tests = shard.two_sample(x, y)

    def finish(h):  # (the one result copy)
        counts_h, last, sp_h, pre_h, post_h, med_h, x_h, y_h, tests_h = h[:9]
        cols_h = h[9:] if host_sessions else [np.zeros(0)] * 9
        last = int(last)
        sp6 = np.asarray(sp_h, dtype=np.float64).reshape(-1) if last >= 0 else np.full(12, np.nan)
        counts_h[RQ4B_SESSIONS] = M
        counts_h[RQ4B_LAST] = last
        counts_h[RQ4B_DELTA_PROJECTS] = pre_h.shape[1]
        med_h = np.asarray(med_h, dtype=np.float64)
        out = {"counts": counts_h, "c2": cols_h[0], "c1": cols_h[1], "g2_q": np.stack(cols_h[2:5], 1).reshape(-1),
               "g1_q": np.stack(cols_h[5:8], 1).reshape(-1), "p_bm": cols_h[8], "sp6": sp6,
               "pre_cov": [pre_h[i].copy() for i in range(7)], "post_cov": [post_h[i].copy() for i in range(7)],
               "pre_median": [float(v) for v in med_h[:7]], "post_median": [float(v) for v in med_h[7:]],
               "init_g2": x_h, "init_g1": y_h, "tests": np.asarray(tests_h, dtype=np.float64)}
        if not host_sessions:  # (this owner's sessions [a, b): device columns)
            out["sessions"] = {"range": (a, b), "cols": own_cols}
        return out
    d = Deferred([counts, last_d, sp, pre, post, med, x, y, tests] + (list(cols) if host_sessions else []), finish)
    return d if finish_later else d.result()


# ------------------------------------------------------------------------- cut projects' eligibility
def fix_cut_eligibility(ctl, cut, lo: int, hi: int, world: int):
    """GROUP BY project HAVING COUNT(*) >= 365 (rq1:144-152) of the cut projects (ascending, every
    rank the same list) over all of their pieces: this store's counts summed over the ranks (one
    all-reduce), the project eligible on its owner (lo <= p < hi) when the sum allows, ineligible on
    a rank that holds only a later piece.  ctl: .elig_counts(ids) -> device int64 counts,
    .set_eligible(ids, flags).  Run after every store build, before the analyses."""
    import torch
    if not cut:
        return
    ids = np.asarray(cut, np.int64)
    cnt = ctl.elig_counts(ids)
    if world > 1:
        all_reduce(cnt)
    own = torch.as_tensor(((ids >= lo) & (ids < hi)).astype(np.uint8), device=cnt.device)
    ctl.set_eligible(ids, ((cnt >= 365).to(torch.uint8) & own))


class GpuEligibility:
    """fix_cut_eligibility's store access on a GPU engine (fz_store_elig_counts /
    fz_store_set_eligible; device in, device out)."""

    def __init__(self, eng):
        import ctypes as C
        from . import engine as E
        self.E, self.C, self.eng = E, C, eng
        self._ids = None

    def _dev_ids(self, ids):
        torch = self.eng.torch
        if self._ids is None or self._ids[0] != tuple(ids.tolist()):
            self._ids = (tuple(ids.tolist()), torch.as_tensor(ids.astype(np.int32), device=self.eng.dev))
        return self._ids[1]

    def elig_counts(self, ids):
        torch = self.eng.torch
        d = self._dev_ids(ids)
        out = torch.empty(len(ids), dtype=torch.int64, device=self.eng.dev)
        self.E._check(self.eng.lib, self.eng.lib.fz_store_elig_counts(self.eng.ctx, self.C.c_void_p(d.data_ptr()),
                                                                      len(ids), self.C.c_void_p(out.data_ptr())))
        return out

    def set_eligible(self, ids, flags):
        d = self._dev_ids(ids)
        flags = flags.contiguous()
        self.E._check(self.eng.lib, self.eng.lib.fz_store_set_eligible(self.eng.ctx, self.C.c_void_p(d.data_ptr()),
                                                                       self.C.c_void_p(flags.data_ptr()), len(ids)))


# ------------------------------------------------------------------------------------ row gathers
def gather_rows(cols: dict, world: int) -> dict:
    """Concatenate per-rank row columns in rank (= project) order (RQ2 change rows, RQ1 raw rows)."""
    import torch
    if world == 1:
        return dict(cols)
    keys = list(cols)
    if len({int(cols[k].numel()) for k in keys}) == 1:  # equal-length columns: ONE gather
        got = all_gather_cols([cols[k] for k in keys])
        return {k: torch.cat([g[j] for g in got]) for j, k in enumerate(keys)}
    return {k: torch.cat(all_gather_v(v)) for k, v in cols.items()}


# --------------------------------------------------------------------------------- GPU shards
class GpuRQ1Shard:
    """RQ1 of one rank on its engine (libfz fz_rq1_ex / fz_rq1_finish)."""

    def __init__(self, eng, max_iter: int, threshold: int = 100):
        import ctypes as C
        from . import engine as E
        from .rq import compute
        self.E, self.C, self.eng, self.threshold = E, C, eng, threshold
        self.bufs = compute.RQ1Buffers(eng, max_iter=max_iter)
        self.b_time = eng.tables.cols["b_time"]
        self.i_number = eng.tables.cols["i_number"]

    pre = False  # launch() already enqueued the first run (a recorded local phase): run(None) reads it

    def launch(self, ext=None):
        """The first run's kernels alone (no host read: graph-capturable)."""
        E, C, eng, b = self.E, self.C, self.eng, self.bufs
        keep = None
        if ext is None:
            x = E.FzRq1Ext(0, None, None, None)
        else:
            keep = tuple(v.contiguous() for v in ext)
            x = E.FzRq1Ext(keep[0].numel(), C.c_void_p(keep[0].data_ptr()), C.c_void_p(keep[1].data_ptr()),
                           C.c_void_p(keep[2].data_ptr()))
        E._check(eng.lib, eng.lib.fz_rq1_ex(eng.ctx, self.threshold, C.byref(x), C.byref(b.out)))

    def run(self, ext):
        b = self.bufs
        if ext is not None or not self.pre:
            self.launch(ext)
        self.pre = False
        n = int(b.counts[RQ1_MATCHED].item())
        mi, mb = b.matched_issue[:n], b.matched_build[:n]
        return {"counts": b.counts, "iter_total": b.iter_total, "iter_detected": b.iter_detected,
                "matched_issue": mi, "matched_build": mb}

    def numbers(self, part):
        """The issue numbers / build times of a run's matches (the cross-shard exchange's columns)."""
        return {"number": self.i_number[part["matched_issue"]], "build_time": self.b_time[part["matched_build"]]}

    def finish(self, counts, it, idt):
        E, C, eng = self.E, self.C, self.eng
        E._check(eng.lib, eng.lib.fz_rq1_finish(eng.ctx, self.threshold, C.c_void_p(it.data_ptr()),
                                                C.c_void_p(idt.data_ptr()), it.numel(),
                                                C.c_void_p(counts.data_ptr()), C.c_void_p(self.bufs.late.data_ptr())))


class _GpuExchange:
    """The project-major session exchange and a cut project's tests on one engine (fz_piece_values,
    fz_pack_runs, fz_transpose_runs, fz_sort_f64, fz_series_dist_*): the shard methods the drivers
    call (the CPU tests' oracle shards implement the same with numpy)."""

    def _piece(self, kind):
        """This rank's leading piece of cut project self.cont: its filtered values (device)."""
        E, C, eng = self.E, self.C, self.eng
        torch = eng.torch
        st = eng.stats
        cap = max(int(st.max_cov_per_project), 1)
        if getattr(self, "_pv", None) is None or self._pv.numel() < cap:
            self._pv = torch.empty(cap, dtype=torch.float64, device=eng.dev)
            self._pc = torch.zeros(3, dtype=torch.int64, device=eng.dev)
        E._check(eng.lib, eng.lib.fz_piece_values(eng.ctx, int(self.cont), kind, C.c_void_p(self._pv.data_ptr()),
                                                  C.c_void_p(self._pc.data_ptr())))

    def pack(self, a, b, runs, sl, own, n):
        """fz_pack_runs: this rank's runs (src, src_off, len, base) sliced by the owners' session
        ranges (sl [world, R] values per slice) -> one buffer, destination-major."""
        E, C, eng = self.E, self.C, self.eng
        torch = eng.torch
        out = torch.empty(max(n, 1), dtype=torch.float64, device=eng.dev)
        runs = np.asarray(runs, np.int64).reshape(-1, 4)
        R = len(runs)
        if n == 0 or R == 0:
            return out[:0]
        # fz_run_desc rows: src_off, len, base, src (int32, pad 0: one little-endian int64)
        desc = np.ascontiguousarray(runs[:, [1, 2, 3, 0]])
        in_off = np.concatenate([[0], np.cumsum(desc[:, 1])[:-1]]).astype(np.int64)
        W = sl.shape[0]
        dst = np.concatenate([[0], np.cumsum(sl.sum(1))[:-1]]).astype(np.int64)
        table = np.zeros((W, R + 1), np.int64)
        table[:, 1:] = np.cumsum(sl, 1)
        table += dst[:, None]
        cuts = np.array([o[0] for o in own] + [own[-1][1]], np.int64)
        h = np.concatenate([desc.reshape(-1), in_off, cuts, table.reshape(-1)])
        d = _upload(h, eng.dev)
        o1 = desc.size
        o2 = o1 + R
        o3 = o2 + W + 1
        P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        a = a if a is not None and a.numel() else None
        b = b if b is not None and b.numel() else None
        E._check(eng.lib, eng.lib.fz_pack_runs(eng.ctx, P(a) if a is not None else None,
                                               P(b) if b is not None else None, P(d), P(d[o1:]), R, P(d[o2:]), W,
                                               P(d[o3:]), n, P(out)))
        return out[:n]

    def transpose(self, vals, roffs, grp, S):
        """fz_transpose_runs: the owner's runs (offsets roffs, host) -> (values grouped by (session,
        group) segment, offsets [S * G + 1]) over its S sessions (device)."""
        E, C, eng = self.E, self.C, self.eng
        torch = eng.torch
        G = 1 if grp is None else 2
        R = len(roffs) - 1
        n = int(roffs[-1])
        if vals.numel() < n or (G == 2 and len(grp) != R) or np.any(np.diff(roffs) > S):
            raise ValueError("transpose: runs exceed the values or the session range")
        out = torch.empty(max(n, 1), dtype=torch.float64, device=eng.dev)
        offs = torch.empty(max(S, 1) * G + 1, dtype=torch.int64, device=eng.dev)
        ro = _upload(np.asarray(roffs, np.int64), eng.dev)
        gd = _upload(np.asarray(grp, np.uint8), eng.dev) if G == 2 and R else None
        vals = vals.contiguous()
        P = lambda t: C.c_void_p(t.data_ptr()) if t is not None and t.numel() else None  # noqa: E731
        E._check(eng.lib, eng.lib.fz_transpose_runs(eng.ctx, P(vals), P(ro), P(gd), R, G, S, n, P(out), P(offs)))
        return out[:n], offs[:S * G + 1]

    def sort(self, x):
        return self.eng.sort_f64(x.contiguous())

    def dist_state(self):
        torch = self.eng.torch
        return (torch.zeros(self.E.FZ_DIST_PARAMS, dtype=torch.float64, device=self.eng.dev),
                torch.full((4,), float("nan"), dtype=torch.float64, device=self.eng.dev))

    def dist_partials(self, ps, v, g, m, g0, n, params, x0):
        E, C, eng = self.E, self.C, self.eng
        torch = eng.torch
        part = torch.empty(E.DIST_PART_WIDTH[ps], dtype=torch.float64, device=eng.dev)
        P = lambda t: C.c_void_p(t.data_ptr()) if t is not None and t.numel() else None  # noqa: E731
        E._check(eng.lib, eng.lib.fz_series_dist_partials(eng.ctx, ps, P(v.contiguous()), P(g.contiguous()), m, g0, n,
                                                          P(params), P(x0), P(part)))
        return part

    def dist_combine(self, ps, parts, k, n, params, result, sizes=None):
        E, C, eng = self.E, self.C, self.eng
        E._check(eng.lib, eng.lib.fz_series_dist_combine(eng.ctx, ps, C.c_void_p(parts.contiguous().data_ptr()), k, n,
                                                         C.c_void_p(params.data_ptr()),
                                                         C.c_void_p(result.data_ptr())))


class GpuRQ2CountShard(_GpuExchange):
    """RQ2 count of one rank on its engine (fz_rq2_count_ex project-major, fz_piece_values for a
    leading piece of a cut project, the exchange primitives, fz_rq2_session_stats_grouped,
    fz_rq2_count_tail)."""

    def __init__(self, eng, cont: int = -1, session_major: bool = False):
        """session_major: (one rank, no cut project) the local kernels write the values session-major
        (the single-table transpose) and rq2_count_sharded skips the run exchange."""
        import ctypes as C
        from . import engine as E
        from .rq import compute
        self.E, self.C, self.eng, self.cont = E, C, eng, int(cont)
        if session_major and self.cont >= 0:
            raise ValueError("GpuRQ2CountShard: a leading piece needs the project-major output")
        self.session_major = bool(session_major)
        self.bufs = compute.rq2_count_buffers(eng)

    pre = False  # launch() already enqueued this step's local kernels (a recorded local phase)

    def launch(self):
        E, C, eng, b = self.E, self.C, self.eng, self.bufs
        flags = E.FZ_RQ2C_SKIP_SESSION_STATS | (0 if self.session_major else E.FZ_RQ2C_PROJECT_MAJOR)
        E._check(eng.lib, eng.lib.fz_rq2_count_ex(eng.ctx, flags, C.byref(b.out)))
        if self.cont >= 0:
            self._piece(E.FZ_PIECE_RQ2)

    def run(self):
        E, b = self.E, self.bufs
        if not self.pre:
            self.launch()
        self.pre = False
        out = {k: getattr(b, k) for k in RQ2C_PROJECT_COLS}
        out["null_lines"] = b.counts[E.RQ2C_NULL_LINES:E.RQ2C_NULL_LINES + 1]
        out["values"] = b.session_values
        out["session_offsets"] = b.session_offsets
        if self.cont >= 0:
            out["piece_values"], out["piece_counts"] = self._pv, self._pc
        return out

    def session_stats_grouped(self, vals, offs, S, max_len):
        return gpu_session_stats_grouped(self.eng, vals, offs, S, max_len)

    def merge_runs(self, vals, runs):
        return gpu_merge_runs(self.eng, vals, runs)

    def series_tests(self, x):
        return gpu_series_tests(self.eng, x)

    def mean_median(self, x):
        return gpu_mean_median(self.eng, x)

    def tail(self, median, k, corr, raw_n, eligible):
        """fz_rq2_count_tail: the median-trend tests over median[:k] and the valid correlations'
        (mean, median) -> device [6] (rho, p, W, p, mean, median)."""
        E, C, eng = self.E, self.C, self.eng
        torch = eng.torch
        out = torch.empty(6, dtype=torch.float64, device=eng.dev)
        median, corr = median.contiguous(), corr.to(torch.float64).contiguous()
        raw_n, eligible = raw_n.to(torch.int64).contiguous(), eligible.to(torch.int64).contiguous()
        P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
        E._check(eng.lib, eng.lib.fz_rq2_count_tail(eng.ctx, P(median), k, P(corr), P(raw_n), P(eligible), corr.numel(),
                                                    P(out)))
        return out


def gpu_merge_runs(eng, vals, runs):
    """fz_runs_merge: R runs of segment-grouped values (runs [R, S] device sizes) -> (values
    segment by segment, offsets [S + 1]); device."""
    import ctypes as C
    from . import engine as E
    torch = eng.torch
    R, S = runs.shape
    vals, runs = vals.contiguous(), runs.to(torch.int64).contiguous()
    out = torch.empty(max(vals.numel(), 1), dtype=torch.float64, device=eng.dev)
    offs = torch.empty(S + 1, dtype=torch.int64, device=eng.dev)
    P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
    E._check(eng.lib, eng.lib.fz_runs_merge(eng.ctx, P(vals), P(runs), R, S, P(out), P(offs)))
    return out[:vals.numel()], offs


def gpu_session_stats_grouped(eng, vals, offs, S, max_len):
    """fz_rq2_session_stats_grouped: per-session mean / median / percentiles of values grouped by
    session (offsets [S + 1])."""
    import ctypes as C
    from . import engine as E
    torch = eng.torch
    avg = torch.empty(max(S, 1), dtype=torch.float64, device=eng.dev)
    med = torch.empty_like(avg)
    pct = torch.empty(max(5 * S, 1), dtype=torch.float64, device=eng.dev)
    ge = torch.zeros(1, dtype=torch.int64, device=eng.dev)
    vals, offs = vals.contiguous(), offs.contiguous()
    P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
    E._check(eng.lib, eng.lib.fz_rq2_session_stats_grouped(eng.ctx, P(vals), P(offs), vals.numel(), S, max_len,
                                                           P(avg), P(med), P(pct), P(ge)))
    return {"average": avg, "median": med, "percentiles": pct, "ge100": ge}


def gpu_session_stats(eng, vals, sids, S, max_len):
    """fz_rq2_session_stats: per-session mean / median / percentiles of (session id, value) pairs."""
    import ctypes as C
    from . import engine as E
    torch = eng.torch
    avg = torch.empty(max(S, 1), dtype=torch.float64, device=eng.dev)
    med = torch.empty_like(avg)
    pct = torch.empty(max(5 * S, 1), dtype=torch.float64, device=eng.dev)
    ge = torch.zeros(1, dtype=torch.int64, device=eng.dev)
    vals, sids = vals.contiguous(), sids.contiguous()
    P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
    E._check(eng.lib, eng.lib.fz_rq2_session_stats(eng.ctx, P(vals), P(sids), vals.numel(), S, max_len, P(avg), P(med),
                                                   P(pct), P(ge)))
    return {"average": avg, "median": med, "percentiles": pct, "ge100": ge}


def gpu_series_tests(eng, x):
    """fz_series_tests: (spearman rho, p, shapiro W, p) of one device series."""
    import ctypes as C
    from . import engine as E
    out = eng.torch.empty(4, dtype=eng.torch.float64, device=eng.dev)
    x = x.contiguous()
    E._check(eng.lib, eng.lib.fz_series_tests(eng.ctx, C.c_void_p(x.data_ptr()) if x.numel() else None, x.numel(),
                                              C.c_void_p(out.data_ptr())))
    return out  # device [4]: read with the other results (host_many)


def gpu_spearman_prefix(eng, rows, n):
    """fz_spearman_index_seg over the first n (a device scalar) entries of every row of a [k, M]
    device block -> device [k, 2] (rho, p); no host round trip."""
    import ctypes as C
    from . import engine as E
    torch = eng.torch
    k, M = rows.shape
    n = n.to(torch.int64).reshape(()).clamp(min=0, max=M)
    j = torch.arange(k * M, dtype=torch.int64, device=eng.dev)
    nn = torch.clamp(n, min=1)
    src = torch.where(j < k * n, (j // nn) * M + j % nn, torch.zeros_like(j))  # row-major prefixes, packed
    x = rows.reshape(-1).to(torch.float64)[src].contiguous()
    offs = (torch.arange(k + 1, dtype=torch.int64, device=eng.dev) * n).contiguous()
    out = torch.empty(2 * k, dtype=torch.float64, device=eng.dev)
    P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
    if k * M > 0:
        E._check(eng.lib, eng.lib.fz_spearman_index_seg(eng.ctx, P(x), x.numel(), P(offs), k, M, P(out[:k]),
                                                        P(out[k:])))
    else:
        out.fill_(float("nan"))
    return torch.stack([out[:k], out[k:]], 1)


def gpu_rq4b_session_stats(eng, vals, sids, grp, S, max_len):
    """fz_rq4b_session_stats: per-session G2 (group 0) / G1 (group 1) counts, quartiles and
    Brunner-Munzel p of (value, session id, group) triples."""
    import ctypes as C
    from . import engine as E
    torch = eng.torch
    z = lambda n, dt: torch.zeros(max(n, 1), dtype=dt, device=eng.dev)  # noqa: E731
    out = {"c2": z(S, torch.int64), "c1": z(S, torch.int64), "g2_q": z(3 * S, torch.float64),
           "g1_q": z(3 * S, torch.float64), "p_bm": z(S, torch.float64)}
    vals, sids, grp = vals.contiguous(), sids.contiguous(), grp.contiguous()
    P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
    E._check(eng.lib, eng.lib.fz_rq4b_session_stats(eng.ctx, P(vals), P(sids), P(grp), vals.numel(), S, max_len,
                                                    *[P(out[k]) for k in ("c2", "c1", "g2_q", "g1_q", "p_bm")]))
    return out


def gpu_rq4b_session_stats_grouped(eng, vals, offs2, S, max_len):
    """fz_rq4b_session_stats_grouped: the same from values grouped by (session, group) segment
    (offsets [2 * S + 1])."""
    import ctypes as C
    from . import engine as E
    torch = eng.torch
    # (every session's counts, quartiles and p are written by the library: no zero fill - config
    # 5L's 20.8 M sessions made the five fills 1.5 GB of memsets per step)
    z = lambda n, dt: torch.empty(max(n, 1), dtype=dt, device=eng.dev)  # noqa: E731
    out = {"c2": z(S, torch.int64), "c1": z(S, torch.int64), "g2_q": z(3 * S, torch.float64),
           "g1_q": z(3 * S, torch.float64), "p_bm": z(S, torch.float64)}
    vals, offs2 = vals.contiguous(), offs2.contiguous()
    P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
    E._check(eng.lib, eng.lib.fz_rq4b_session_stats_grouped(eng.ctx, P(vals), P(offs2), vals.numel(), S, max_len,
                                                            *[P(out[k]) for k in ("c2", "c1", "g2_q", "g1_q", "p_bm")]))
    return out


def gpu_mean_median(eng, x):
    """(mean, median) of one device vector through fz_describe_f64_dev (NaN when empty): a device
    [2] view, copied with the driver's other results."""
    import ctypes as C
    from . import engine as E
    if x.numel() == 0:
        return np.array([np.nan, np.nan])
    x = x.contiguous()
    d = eng.torch.empty(E.DESCRIBE_DOUBLES, dtype=eng.torch.float64, device=eng.dev)
    E._check(eng.lib, eng.lib.fz_describe_f64_dev(eng.ctx, C.c_void_p(x.data_ptr()), x.numel(),
                                                  C.c_void_p(d.data_ptr())))
    return d[4:6]  # fz_describe: count, n_pos, n_zero, n_neg, mean, median, ...


class GpuRQ4aShard:
    """RQ4a of one rank on its engine (fz_rq4a / fz_rq4a_finish)."""

    def __init__(self, eng, max_iter: int):
        import ctypes as C
        from . import engine as E
        from .rq import compute
        self.E, self.C, self.eng = E, C, eng
        self.bufs = compute.rq4a_buffers(eng, max_iter=max_iter)

    pre = False  # launch() already enqueued this step's local kernels (a recorded local phase)

    def launch(self):
        E, C, eng, b = self.E, self.C, self.eng, self.bufs
        E._check(eng.lib, eng.lib.fz_rq4a(eng.ctx, C.byref(eng.groups), C.byref(b.out)))

    def run(self):
        b = self.bufs
        if not self.pre:
            self.launch()
        self.pre = False
        return {k: getattr(b, k) for k in ("counts", "member", "intro", "g4_steps", "g4_transition") + RQ4A_TABLES}

    def finish(self, tables, intro, steps, counts):
        E, C, eng, b = self.E, self.C, self.eng, self.bufs
        P = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
        tables = [x.contiguous() for x in tables]
        intro = intro.contiguous()
        E._check(eng.lib, eng.lib.fz_rq4a_finish(eng.ctx, *[P(x) for x in tables], tables[0].numel(), P(intro),
                                                 intro.numel(), P(steps), P(counts), P(b.scalars)))
        return b.scalars  # device: copied with the other results (parallel.host_many)


class GpuRQ2AddShard:
    """RQ2 add of one rank on its engine (fz_rq2_add): the flags and the change rows, sliced on the
    device to the row count (one host read of the counter)."""

    def __init__(self, eng):
        from . import engine as E
        from .rq import compute
        self.E, self.eng, self.compute = E, eng, compute
        self.bufs = compute.rq2_add_buffers(eng)

    pre = False  # launch() already enqueued this step's kernels (a recorded local phase)

    def launch(self):
        self.compute.rq2_add_launch(self.eng, self.bufs)

    def run(self):
        b, P = self.bufs, self.eng.tables.fz.n_projects
        if not self.pre:
            self.launch()
        self.pre = False
        n = int(host_many(b.counts[self.E.RQ2A_ROWS])[0])
        out = {k: getattr(b, k)[:P] for k in RQ2A_FLAGS}
        out.update({k: getattr(b, k)[:n] for k in RQ2A_ROW_COLS})
        return out


class GpuRQ4bShard(_GpuExchange):
    """RQ4b of one rank on its engine (fz_rq4b_ex project-major, fz_piece_values for a leading piece
    of a cut project, the exchange primitives, fz_rq4b_session_stats_grouped, fz_rq4b_tail)."""

    def __init__(self, eng, cont: int = -1, session_major: bool = False):
        """session_major: as GpuRQ2CountShard (values grouped by (session, group) locally)."""
        import ctypes as C
        from . import engine as E
        from .rq import compute
        self.E, self.C, self.eng, self.cont = E, C, eng, int(cont)
        if session_major and self.cont >= 0:
            raise ValueError("GpuRQ4bShard: a leading piece needs the project-major output")
        self.session_major = bool(session_major)
        self.bufs = compute.rq4b_buffers(eng, shard=True)

    pre = False  # launch() already enqueued this step's local kernels (a recorded local phase)

    def launch(self):
        E, C, eng, b = self.E, self.C, self.eng, self.bufs
        flags = E.FZ_RQ4B_SKIP_SESSION_STATS | (0 if self.session_major else E.FZ_RQ4B_PROJECT_MAJOR)
        E._check(eng.lib, eng.lib.fz_rq4b_ex(eng.ctx, C.byref(eng.groups), flags, C.byref(b.out)))
        if self.cont >= 0:
            self._piece(E.FZ_PIECE_RQ4B)

    def run(self):
        eng, b = self.eng, self.bufs
        if not self.pre:
            self.launch()
        self.pre = False
        P = eng.tables.fz.n_projects  # column lengths stay on the device (counts); rq4b_sharded slices
        out = {"counts": b.counts, "member": b.member[:P], "trend_values": b.trend_values,
               "trend_offsets": b.trend_offsets, "pre_cov": b.pre_cov, "post_cov": b.post_cov,
               "delta_order": b.delta_order, "init_g2": b.init_g2, "init_g1": b.init_g1}
        if self.cont >= 0:
            out["piece_values"], out["piece_counts"] = self._pv, self._pc
        return out

    def session_stats_grouped(self, vals, offs2, S, max_len):
        return gpu_rq4b_session_stats_grouped(self.eng, vals, offs2, S, max_len)

    def merge_runs(self, vals, runs):
        return gpu_merge_runs(self.eng, vals, runs)

    def series_tests(self, x):
        return gpu_series_tests(self.eng, x)

    def spearman_prefix(self, rows, n):
        return gpu_spearman_prefix(self.eng, rows, n)

    def trends(self, cols):
        """fz_rq4b_trends over the per-session columns (c2, c1, G2 Q1..Q3, G1 Q1..Q3, p_bm) -> (last
        session with both groups >= 100 as a device scalar, (rho, p) x 6 device)."""
        E, C, eng = self.E, self.C, self.eng
        torch = eng.torch
        n = cols[0].numel()
        c2, c1 = cols[0].to(torch.int64).contiguous(), cols[1].to(torch.int64).contiguous()
        g2 = torch.stack(cols[2:5], 1).reshape(-1).to(torch.float64).contiguous()
        g1 = torch.stack(cols[5:8], 1).reshape(-1).to(torch.float64).contiguous()
        last = torch.empty(1, dtype=torch.int64, device=eng.dev)
        sp = torch.empty(12, dtype=torch.float64, device=eng.dev)
        P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
        E._check(eng.lib, eng.lib.fz_rq4b_trends(eng.ctx, P(c2), P(c1), P(g2), P(g1), n, P(last), P(sp)))
        return last[0], sp

    def mean_median(self, x):
        return gpu_mean_median(self.eng, x)

    def row_medians(self, rows):
        """statistics.median of every row of a [k, n] device block (NaN for n == 0), one call; device."""
        k, n = rows.shape
        offs = self.eng.torch.arange(k + 1, dtype=self.eng.torch.int64, device=self.eng.dev) * n
        out = gpu_session_stats_grouped(self.eng, rows.reshape(-1).contiguous(), offs, k, n)
        return out["median"][:k]

    def tail(self, c2, c1, g2q, g1q, order, pre, post, x, y):
        """fz_rq4b_tail: trends over the per-session columns, the delta columns ([7, nd] each) in CSV
        order by `order` with the medians of their 14 rows, the initial-coverage tests -> device
        (last, spearman6 [12], pre [7, nd], post [7, nd], medians [14], tests)."""
        E, C, eng = self.E, self.C, self.eng
        torch = eng.torch
        M, nd = c2.numel(), order.numel()
        c2, c1 = c2.to(torch.int64).contiguous(), c1.to(torch.int64).contiguous()
        g2q, g1q = g2q.to(torch.float64).contiguous(), g1q.to(torch.float64).contiguous()
        order = order.to(torch.int64).contiguous()
        pre, post = pre.to(torch.float64).contiguous(), post.to(torch.float64).contiguous()
        x, y = x.contiguous(), y.contiguous()
        last = torch.empty(1, dtype=torch.int64, device=eng.dev)
        res = torch.empty(12 + 14 + E.FZ_RQ4B_NTESTS + 14 * max(nd, 1), dtype=torch.float64, device=eng.dev)
        sp, med, tests = res[:12], res[12:26], res[26:26 + E.FZ_RQ4B_NTESTS]
        po = res[26 + E.FZ_RQ4B_NTESTS:]
        pre_o, post_o = po[:7 * nd].view(7, nd), po[7 * nd:14 * nd].view(7, nd)
        P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
        E._check(eng.lib, eng.lib.fz_rq4b_tail(eng.ctx, P(c2), P(c1), P(g2q), P(g1q), M, P(order), P(pre), P(post), nd,
                                               int(eng.groups.n_order), P(x), x.numel(), P(y), y.numel(), P(last),
                                               P(sp), P(pre_o), P(post_o), P(med), P(tests)))
        return last[0], sp, pre_o, post_o, med, tests

    def two_sample(self, x, y):
        E, C, eng = self.E, self.C, self.eng
        out = eng.torch.full((E.FZ_RQ4B_NTESTS,), float("nan"), dtype=eng.torch.float64, device=eng.dev)
        x, y = x.contiguous(), y.contiguous()
        P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
        if x.numel() and y.numel():
            E._check(eng.lib, eng.lib.fz_two_sample_tests(eng.ctx, P(x), x.numel(), P(y), y.numel(), P(out)))
        return out  # device: copied with the other results


class GpuRQ3Shard:
    """RQ3 of one rank on its engine (libfz fz_rq3_ex with FZ_RQ3_FLUSH_LAST / fz_rq3_stats)."""

    def __init__(self, eng):
        import ctypes as C
        from . import engine as E
        from .rq import compute
        self.E, self.C, self.eng = E, C, eng
        self.bufs = compute.rq3_buffers(eng)

    pre = False  # launch() already enqueued this step's local kernels (a recorded local phase)

    def launch(self):
        E, C, eng, b = self.E, self.C, self.eng, self.bufs
        E._check(eng.lib, eng.lib.fz_rq3_ex(eng.ctx, E.FZ_RQ3_FLUSH_LAST | E.FZ_RQ3_SKIP_STATS, C.byref(b.out)))

    def run(self):
        b = self.bufs
        if not self.pre:
            self.launch()
        self.pre = False
        cnt = b.counts.cpu()
        nd, nn = int(cnt[RQ3_DETECTED]), int(cnt[RQ3_NON_DETECTED])
        out = {"counts": b.counts, "counts_h": cnt.numpy()}
        for k in RQ3_DET_F + RQ3_DET_I:
            out[k] = getattr(b, k)[:nd]
        for k in RQ3_NON_F + RQ3_NON_I:
            out[k] = getattr(b, k)[:nn]
        return out

    def stats(self, det_pct, det_tot, non_pct):
        E, C, eng, b = self.E, self.C, self.eng, self.bufs
        P = lambda t: C.c_void_p(t.data_ptr()) if t.numel() else None  # noqa: E731
        E._check(eng.lib, eng.lib.fz_rq3_stats(eng.ctx, P(det_pct), P(det_tot), det_pct.numel(), P(non_pct),
                                               non_pct.numel(), C.c_void_p(b.describe.data_ptr()),
                                               C.c_void_p(b.tests.data_ptr())))
        return {"describe": b.describe, "tests": b.tests}
