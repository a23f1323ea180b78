"""GPU compute path: each function runs one reference script's analysis through ``libfz`` and
returns the same result object the CPU oracle produces (``tse_amd.rq.results``).

Only O(iterations) / O(projects) bookkeeping happens here on the host (unpacking counts,
building Python lists for the renderer); every per-row computation is a HIP kernel.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import engine as E
from .results import Describe, RQ1Result


def _describe(d: E.FzDescribe, with_min_nonzero=False) -> Describe:
    return Describe(count=int(d.count), n_pos=int(d.n_pos), n_zero=int(d.n_zero), n_neg=int(d.n_neg),
                    mean=float(d.mean), median=float(d.median), std=float(d.std), min=float(d.min),
                    max=float(d.max), q1=float(d.q1), q3=float(d.q3),
                    min_nonzero=(float(d.min_nonzero) if (with_min_nonzero and d.has_nonzero) else None))


class RQ1Buffers:
    """Device outputs of fz_rq1, allocated once per store (re-used across bench steps)."""

    def __init__(self, eng: E.Engine):
        torch = eng.torch
        fz = eng.tables.fz
        M = max(int(eng.stats.max_fuzz_per_project), 1)
        self.counts = eng.zeros(E.FZ_RQ1_NCOUNTS, torch.int64)
        self.eligible = eng.zeros(fz.n_projects, torch.uint8)
        self.iter_total = eng.zeros(M, torch.int64)
        self.iter_detected = eng.zeros(M, torch.int64)
        self.matched_issue = eng.zeros(fz.n_issues, torch.int64)
        self.matched_build = eng.zeros(fz.n_issues, torch.int64)
        self.late = eng.zeros(E.DESCRIBE_DOUBLES, torch.float64)
        self.out = E.FzRq1Out(*[C.c_void_p(b.data_ptr()) for b in (
            self.counts, self.eligible, self.iter_total, self.iter_detected, self.matched_issue,
            self.matched_build, self.late)])


def rq1_launch(eng: E.Engine, bufs: RQ1Buffers, threshold: int = 100):
    """Enqueue RQ1 on the engine stream (no host synchronisation)."""
    E._check(eng.lib, eng.lib.fz_rq1(eng.ctx, threshold, C.byref(bufs.out)))


def rq1_collect(eng: E.Engine, bufs: RQ1Buffers, threshold: int = 100) -> RQ1Result:
    cnt = bufs.counts.cpu().numpy()
    n_match = int(cnt[E.RQ1_MATCHED])
    M = int(cnt[E.RQ1_MAX_ITER])
    late = None
    if cnt[E.RQ1_LATE] > 0:
        d = _describe(E.describe_from_doubles(bufs.late.cpu().numpy()), with_min_nonzero=True)
        # rq1_detection_rate.py:256-268 reports only these numbers (no sign split, no std)
        late = Describe(count=d.count, n_zero=d.n_zero, min=d.min, max=d.max, q1=d.q1, q3=d.q3,
                        median=d.median, mean=d.mean, min_nonzero=d.min_nonzero)
    elig = np.nonzero(bufs.eligible.cpu().numpy()[:eng.tables.fz.n_projects])[0]
    return RQ1Result(
        n_issues_lim=int(cnt[E.RQ1_ISSUES_LIM]), n_issues_lim_projects=int(cnt[E.RQ1_ISSUES_LIM_PROJECTS]),
        n_fixed_lim=int(cnt[E.RQ1_FIXED_LIM]), n_fixed_lim_projects=int(cnt[E.RQ1_FIXED_LIM_PROJECTS]),
        eligible=elig, n_without_matching=int(cnt[E.RQ1_WITHOUT_MATCHING]),
        n_target=int(cnt[E.RQ1_TARGET]), n_target_projects=int(cnt[E.RQ1_TARGET_PROJECTS]),
        total_fuzz_builds=int(cnt[E.RQ1_TOTAL_FUZZ]),
        matched_issue=bufs.matched_issue[:n_match].cpu().numpy(),
        matched_build=bufs.matched_build[:n_match].cpu().numpy(),
        n_matched_projects=int(cnt[E.RQ1_MATCHED_PROJECTS]),
        iter_total=bufs.iter_total[:M].cpu().numpy(), iter_detected=bufs.iter_detected[:M].cpu().numpy(),
        min_project_threshold=threshold, late=late)


def rq1(eng: E.Engine, threshold: int = 100) -> RQ1Result:
    """rq1_detection_rate.collect_and_analyze_data (rq1_detection_rate.py:101-269) on the GPU."""
    bufs = RQ1Buffers(eng)
    rq1_launch(eng, bufs, threshold)
    return rq1_collect(eng, bufs, threshold)
