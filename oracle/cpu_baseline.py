"""CPU BASELINE (test infrastructure only - see oracle/__init__.py).

ctypes front of ``oracle/cpu/libfzcpu.so`` (``oracle/cpu/fz_cpu.cpp``): the multi-core C++
restatement of the six analyses over the same host columns the engine uploads (``fz_tables`` /
``fz_rq4_groups`` of include/fz.h, host pointers).  bench.py's ``cpu_baseline`` leg times it with
the host's cores; tests/test_cpu_baseline.py checks its outputs against ``rq_oracle``.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "cpu", "libfzcpu.so")
STAGES = {"rq1": 1, "rq2_count": 2, "rq2_add": 4, "rq3": 8, "rq4a": 16, "rq4b": 32}
TIMES = ("store", "rq1", "rq2_count", "rq2_add", "rq3", "rq4a", "rq4b")

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle` (or __graft_entry__.build())")
        lib = C.CDLL(LIB_PATH)
        lib.fzcpu_run.restype = C.c_void_p
        lib.fzcpu_run.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_int, C.POINTER(C.c_double)]
        for n, t in (("fzcpu_get_f64", C.c_double), ("fzcpu_get_i64", C.c_int64)):
            f = getattr(lib, n)
            f.restype = C.c_int64
            f.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.POINTER(t))]
        lib.fzcpu_free.argtypes = [C.c_void_p]
        lib.fzcpu_max_threads.restype = C.c_int
        lib.fzcpu_limit_us.restype = C.c_int64
        lib.fzcpu_limit_us.argtypes = [C.c_int]
        _lib = lib
    return _lib


class HostTables:
    """The engine's upload image (engine.Engine.upload) as host arrays + fz_tables / fz_rq4_groups
    structs pointing at them (kept alive by this object)."""

    def __init__(self, t):
        from tse_amd import engine as E
        from tse_amd.rq.common import corpus_columns
        P = len(t.projects)
        c_valid = (t.c_coverage_valid.astype(np.uint8) * E.VALID_COVERAGE
                   | t.c_covered_valid.astype(np.uint8) * E.VALID_COVERED
                   | t.c_total_valid.astype(np.uint8) * E.VALID_TOTAL)
        member, corpus_us, order = corpus_columns(t)
        cols = {
            "b_project": t.b_project, "b_type": t.b_type, "b_result": t.b_result, "b_time": t.b_time,
            "b_group": t.group_key(), "b_rev_canon": t.rev_canon(), "c_project": t.c_project,
            "c_date": t.c_date, "c_coverage": t.c_coverage, "c_covered": t.c_covered, "c_total": t.c_total,
            "c_valid": c_valid, "i_number": t.i_number, "i_project": t.i_project, "i_rts": t.i_rts,
            "i_status": t.i_status,
            "pi_count": np.bincount(t.pi_project.astype(np.int64), minlength=P).astype(np.int32),
        }
        want = {"b_project": np.uint32, "c_project": np.uint32, "i_project": np.uint32, "b_group": np.int32,
                "b_rev_canon": np.int32}
        self.cols = {k: np.ascontiguousarray(v, dtype=want.get(k, np.asarray(v).dtype)) for k, v in cols.items()}
        self.g = {"member": np.ascontiguousarray(member, np.uint8),
                  "corpus_us": np.ascontiguousarray(corpus_us, np.int64),
                  "order": np.ascontiguousarray(order, np.int32)}
        ptr = {k: C.c_void_p(v.ctypes.data) for k, v in self.cols.items()}
        self.fz = E.FzTables(n_projects=P, n_builds=len(t.b_project), n_cov=len(t.c_project),
                             n_issues=len(t.i_project), **ptr)
        self.groups = E.FzRq4Groups(member=C.c_void_p(self.g["member"].ctypes.data),
                                    corpus_us=C.c_void_p(self.g["corpus_us"].ctypes.data),
                                    order=C.c_void_p(self.g["order"].ctypes.data), n_order=len(order))
        self.n_rows = t.n_rows


def run(host: HostTables, stages=tuple(STAGES), threads: int = 0):
    """Index build + ``stages`` with ``threads`` OpenMP threads (0: all).  Returns (outputs dict of
    numpy arrays, per-stage seconds dict)."""
    lib = load()
    mask = 0
    for s in stages:
        mask |= STAGES[s]
    secs = (C.c_double * 7)()
    h = lib.fzcpu_run(C.byref(host.fz), C.byref(host.groups), mask, int(threads), secs)
    if not h:
        raise RuntimeError("fzcpu_run rejected its arguments")
    try:
        return _outputs(lib, h), dict(zip(TIMES, list(secs)))
    finally:
        lib.fzcpu_free(h)


_F64 = ("rq1_late", "rq2c_sw_w", "rq2c_sw_p", "rq2c_corr", "rq2c_session_values", "rq2c_scalars", "rq2c_average",
        "rq2c_median", "rq2c_pct", "rq2c_dist_mean", "rq2a_diff_total", "rq2a_diff_coverage", "rq3_det_pct",
        "rq3_non_pct", "rq3_describe", "rq3_tests", "rq4a_scalars", "rq4b_g2_q", "rq4b_g1_q", "rq4b_p_bm",
        "rq4b_spearman6", "rq4b_pre", "rq4b_post", "rq4b_medians", "rq4b_init_g2", "rq4b_init_g1", "rq4b_tests")
_I64 = ("rq1_counts", "rq1_iter_total", "rq1_iter_detected", "rq1_matched_issue", "rq1_matched_build",
        "rq2c_raw_n", "rq2c_n_trend", "rq2c_session_offsets", "rq2a_rows", "rq2a_flags", "rq3_counts",
        "rq3_det_cols", "rq3_non_cols", "rq4a_g1_total", "rq4a_g1_det", "rq4a_g2_total", "rq4a_g2_det", "rq4a_intro",
        "rq4a_steps", "rq4a_transition", "rq4b_c2", "rq4b_c1", "rq4b_last")


def _outputs(lib, h):
    out = {}
    for names, ctype, fn, dt in ((_F64, C.c_double, lib.fzcpu_get_f64, np.float64),
                                 (_I64, C.c_int64, lib.fzcpu_get_i64, np.int64)):
        for n in names:
            p = C.POINTER(ctype)()
            k = fn(h, n.encode(), C.byref(p))
            if k < 0:
                continue
            out[n] = np.ctypeslib.as_array(p, shape=(k,)).astype(dt, copy=True) if k else np.zeros(0, dt)
    return out
