"""ctypes binding of ``libfz.so`` (C ABI: ``include/fz.h``) and the device-resident tables.

This is the drop-in for ``program/__module/dbFile.py:5-38`` (``DB.connect`` /
``DB.executeQuery``): instead of one SQL round trip per project, the columnar tables are
uploaded to HBM once (``DeviceTables``), sorted once into the store (``Engine.build_store``,
the replacement for PostgreSQL's tables + indexes) and every RQ computation runs as HIP
kernels over it.  PyTorch-ROCm is used only to allocate device buffers and to provide the
stream; all compute goes through ``libfz``.  There is no CPU fallback: without the built
library or without a GPU every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import LIB_PATH
from .schema import Tables

FZ_RQ1_NCOUNTS = 16
(RQ1_ISSUES_LIM, RQ1_ISSUES_LIM_PROJECTS, RQ1_FIXED_LIM, RQ1_FIXED_LIM_PROJECTS, RQ1_ELIGIBLE,
 RQ1_WITHOUT_MATCHING, RQ1_TARGET, RQ1_TARGET_PROJECTS, RQ1_TOTAL_FUZZ, RQ1_MATCHED,
 RQ1_MATCHED_PROJECTS, RQ1_MAX_ITER, RQ1_KEPT_ITERS, RQ1_FIRST_DOWN, RQ1_LATE) = range(15)

VALID_COVERAGE, VALID_COVERED, VALID_TOTAL = 1, 2, 4

_P = C.c_void_p
_I64 = C.c_int64


class FzTables(C.Structure):
    _fields_ = [("n_projects", _I64),
                ("n_builds", _I64), ("b_project", _P), ("b_type", _P), ("b_result", _P), ("b_time", _P),
                ("b_group", _P), ("b_rev_canon", _P),
                ("n_cov", _I64), ("c_project", _P), ("c_date", _P), ("c_coverage", _P), ("c_covered", _P),
                ("c_total", _P), ("c_valid", _P),
                ("n_issues", _I64), ("i_number", _P), ("i_project", _P), ("i_rts", _P), ("i_status", _P),
                ("pi_count", _P)]


class FzStoreStats(C.Structure):
    _fields_ = [("n_projects", _I64), ("n_fuzz", _I64), ("n_coverage_builds", _I64),
                ("max_fuzz_per_project", _I64), ("max_cov_per_project", _I64), ("sort_passes", _I64)]


class FzDescribe(C.Structure):
    _fields_ = [("count", _I64), ("n_pos", _I64), ("n_zero", _I64), ("n_neg", _I64),
                ("mean", C.c_double), ("median", C.c_double), ("std", C.c_double), ("min", C.c_double),
                ("max", C.c_double), ("q1", C.c_double), ("q3", C.c_double), ("min_nonzero", C.c_double),
                ("has_nonzero", _I64)]


DESCRIBE_DOUBLES = 13  # sizeof(fz_describe) / 8


class FzRq1Out(C.Structure):
    _fields_ = [("counts", _P), ("eligible", _P), ("iter_total", _P), ("iter_detected", _P),
                ("matched_issue", _P), ("matched_build", _P), ("late", _P)]


class FzRq1Ext(C.Structure):
    _fields_ = [("n", _I64), ("number", _P), ("build_time", _P), ("before", _P)]


FZ_RQ2C_NCOUNTS, FZ_RQ2C_NSCALARS = 8, 8
RQ2C_ELIGIBLE, RQ2C_SESSIONS, RQ2C_GE100, RQ2C_VALUES, RQ2C_NULL_LINES = range(5)
RQ2C_CORR_MEAN, RQ2C_CORR_MEDIAN, RQ2C_SP_RHO, RQ2C_SP_P, RQ2C_SW_MEDIAN_P = range(5)
FZ_RQ2C_SKIP_SESSION_STATS = 1
FZ_RQ2C_PROJECT_MAJOR = 2


class FzRq2CountOut(C.Structure):
    _fields_ = [(n, _P) for n in ("counts", "scalars", "eligible", "raw_n", "n_trend", "sw_w", "sw_p", "corr",
                                  "session_offsets", "session_values", "average_trend", "median_trend",
                                  "dist_percentiles", "dist_mean")]


FZ_RQ2A_NCOUNTS = 4
RQ2A_ELIGIBLE, RQ2A_ROWS, RQ2A_RUNS = range(3)


class FzRq2AddOut(C.Structure):
    _fields_ = [(n, _P) for n in ("counts", "eligible", "row_project", "row_first_build", "row_end_build",
                                  "row_start_build", "row_cov_i", "row_cov_i1", "diff_total", "diff_coverage",
                                  "covered_is_float", "total_is_float")]


FZ_RQ3_NCOUNTS, FZ_RQ3_NTESTS = 8, 16
RQ3_ISSUES, RQ3_DETECTED, RQ3_NON_DETECTED, RQ3_ELIGIBLE, RQ3_NON_LAST, RQ3_NULL_TOTAL, RQ3_NULL_LAST = range(7)
FZ_RQ3_FLUSH_LAST, FZ_RQ3_SKIP_STATS = 1, 2
RQ3_AD_DET, RQ3_AD_NON, RQ3_LEVENE_W, RQ3_LEVENE_P, RQ3_BM_STAT, RQ3_BM_P = 0, 6, 12, 13, 14, 15


class FzRq3Out(C.Structure):
    _fields_ = [(n, _P) for n in ("counts", "eligible", "det_pct", "det_cov", "det_tot", "det_project", "det_issue",
                                  "non_pct", "non_cov", "non_tot", "describe", "tests")]


class FzHostPiece(C.Structure):  # fz_host_piece (fz_gather_to_host)
    _fields_ = [("src", _P), ("n", _I64), ("stride", _I64), ("dst_offset", _I64), ("elem_bytes", C.c_int32),
                ("pad_", C.c_int32)]


class FzRq4Groups(C.Structure):
    _fields_ = [("member", _P), ("corpus_us", _P), ("order", _P), ("n_order", _I64)]


FZ_RQ4A_NCOUNTS, FZ_RQ4A_NSCALARS = 12, 12
(RQ4A_MAX_ITER, RQ4A_ROWS, RQ4A_G1, RQ4A_G2, RQ4A_G3, RQ4A_G4, RQ4A_HAS_WINDOW, RQ4A_AFTER_G1, RQ4A_AFTER_G2,
 RQ4A_INTRO_POS) = range(10)
(RQ4A_AFTER_G1_MEDIAN, RQ4A_AFTER_G1_IQR, RQ4A_AFTER_G2_MEDIAN, RQ4A_AFTER_G2_IQR, RQ4A_INTRO_MEAN,
 RQ4A_INTRO_MEDIAN, RQ4A_INTRO_MIN, RQ4A_INTRO_MAX, RQ4A_PRE_RATE, RQ4A_POST_RATE) = range(10)


class FzRq4aOut(C.Structure):
    _fields_ = [(n, _P) for n in ("counts", "scalars", "eligible", "member", "g1_total", "g1_det", "g2_total",
                                  "g2_det", "intro", "g4_steps", "g4_transition")]


FZ_RQ4B_NCOUNTS, FZ_RQ4B_NTESTS = 12, 8
(RQ4B_SESSIONS, RQ4B_LAST, RQ4B_DELTA_PROJECTS, RQ4B_INIT_G2, RQ4B_INIT_G1, RQ4B_G1, RQ4B_G2, RQ4B_G3,
 RQ4B_G4, RQ4B_VALUES) = range(10)
RQ4B_MWU_P, RQ4B_CLIFF, RQ4B_BM_STAT, RQ4B_BM_P, RQ4B_LEVENE_W, RQ4B_LEVENE_P = range(6)
FZ_RQ4B_SKIP_SESSION_STATS = 1
FZ_RQ4B_PROJECT_MAJOR = 2
FZ_PIECE_RQ2, FZ_PIECE_RQ4B = 0, 1
FZ_DIST_PARAMS = 10
DIST_PART_WIDTH = (14, 4, 6)  # FZ_DIST_PART_WIDTH(pass)


class FzRq4bOut(C.Structure):
    _fields_ = [(n, _P) for n in ("counts", "eligible", "member", "c2", "c1", "g2_q", "g1_q", "p_bm", "spearman6",
                                  "pre_cov", "post_cov", "pre_median", "post_median", "init_g2", "init_g1",
                                  "tests", "trend_values", "trend_offsets", "delta_order")]


class FzBuildlogOut(C.Structure):
    _fields_ = [("log_type", _P), ("log_result", _P), ("log_status", _P), ("log_proj_off", _P), ("log_proj_len", _P),
                ("log_line0", _P), ("n_lines", _P), ("ev_line", _P), ("ev_start", _P), ("ev_len", _P),
                ("ev_flags", _P), ("event_cap", _I64), ("n_events", _P)]


# every symbol include/fz.h declares, with its ctypes signature
SIGNATURES = {
    "fz_abi_version": (C.c_int, []),
    "fz_last_error": (C.c_char_p, []),
    "fz_ctx_create": (C.c_int, [C.c_int, _P, C.POINTER(_P)]),
    "fz_ctx_create_child": (C.c_int, [_P, _P, C.POINTER(_P)]),
    "fz_ctx_destroy": (C.c_int, [_P]),
    "fz_ctx_set_stream": (C.c_int, [_P, _P]),
    "fz_store_build": (C.c_int, [_P, C.POINTER(FzTables), C.POINTER(FzStoreStats)]),
    "fz_store_set_helpers": (C.c_int, [_P, C.POINTER(_P), C.c_int]),
    "fz_rq1": (C.c_int, [_P, _I64, C.POINTER(FzRq1Out)]),
    "fz_rq1_ex": (C.c_int, [_P, _I64, C.POINTER(FzRq1Ext), C.POINTER(FzRq1Out)]),
    "fz_rq1_finish": (C.c_int, [_P, _I64, _P, _P, _I64, _P, _P]),
    "fz_rq2_count": (C.c_int, [_P, C.POINTER(FzRq2CountOut)]),
    "fz_rq2_count_ex": (C.c_int, [_P, C.c_uint32, C.POINTER(FzRq2CountOut)]),
    "fz_rq2_session_stats": (C.c_int, [_P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P]),
    "fz_rq2_session_stats_grouped": (C.c_int, [_P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P]),
    "fz_runs_merge": (C.c_int, [_P, _P, _P, _I64, _I64, _P, _P]),
    "fz_series_tests": (C.c_int, [_P, _P, _I64, _P]),
    "fz_spearman_index_seg": (C.c_int, [_P, _P, _I64, _P, _I64, _I64, _P, _P]),
    "fz_rq2_add": (C.c_int, [_P, C.POINTER(FzRq2AddOut)]),
    "fz_rq3": (C.c_int, [_P, C.POINTER(FzRq3Out)]),
    "fz_rq3_ex": (C.c_int, [_P, C.c_uint32, C.POINTER(FzRq3Out)]),
    "fz_rq3_stats": (C.c_int, [_P, _P, _P, _I64, _P, _I64, _P, _P]),
    "fz_rq3_stats_dn": (C.c_int, [_P, _P, _P, _I64, _P, _P, _I64, _P, _P, _P]),
    "fz_rq4a": (C.c_int, [_P, C.POINTER(FzRq4Groups), C.POINTER(FzRq4aOut)]),
    "fz_rq4a_finish": (C.c_int, [_P, _P, _P, _P, _P, _I64, _P, _I64, _P, _P, _P]),
    "fz_rq4b": (C.c_int, [_P, C.POINTER(FzRq4Groups), C.POINTER(FzRq4bOut)]),
    "fz_rq4b_ex": (C.c_int, [_P, C.POINTER(FzRq4Groups), C.c_uint32, C.POINTER(FzRq4bOut)]),
    "fz_rq4b_session_stats": (C.c_int, [_P, _P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P]),
    "fz_rq4b_session_stats_grouped": (C.c_int, [_P, _P, _P, _I64, _I64, _I64, _P, _P, _P, _P, _P]),
    "fz_rq4b_trends": (C.c_int, [_P, _P, _P, _P, _P, _I64, _P, _P]),
    "fz_describe_f64_dev": (C.c_int, [_P, _P, _I64, _P]),
    "fz_two_sample_tests": (C.c_int, [_P, _P, _I64, _P, _I64, _P]),
    "fz_rq2_count_tail": (C.c_int, [_P, _P, _I64, _P, _P, _P, _I64, _P]),
    "fz_gather_to_host": (C.c_int, [_P, _P, C.c_int, _P, _I64]),
    "fz_rq4b_tail": (C.c_int, [_P, _P, _P, _P, _P, _I64, _P, _P, _P, _I64, _I64, _P, _I64, _P, _I64,
                              _P, _P, _P, _P, _P, _P]),
    "fz_buildlog": (C.c_int, [_P, _P, _I64, _P, _P, _I64, C.POINTER(FzBuildlogOut)]),
    "fz_probe_begin": (C.c_int, [_P, C.c_char_p]),
    "fz_probe_end": (C.c_int, [_P, C.POINTER(_I64), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "fz_probe_get": (C.c_int, [_P, C.c_char_p, C.POINTER(_I64), C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    "fz_capture_begin": (C.c_int, [_P]),
    "fz_capture_end": (C.c_int, [_P, C.POINTER(_P)]),
    "fz_graph_launch": (C.c_int, [_P, _P]),
    "fz_graph_destroy": (C.c_int, [_P]),
    "fz_radix_sort_u64": (C.c_int, [_P, _P, _P, _I64, C.c_int]),
    "fz_sort_f64": (C.c_int, [_P, _P, _I64, _P, _P]),
    "fz_describe_f64": (C.c_int, [_P, _P, _I64, C.POINTER(FzDescribe)]),
    "fz_eligibility_count": (C.c_int, [_P, C.POINTER(FzTables), _I64, _P]),
    "fz_store_elig_counts": (C.c_int, [_P, _P, _I64, _P]),
    "fz_store_set_eligible": (C.c_int, [_P, _P, _P, _I64]),
    "fz_piece_values": (C.c_int, [_P, _I64, C.c_int, _P, _P]),
    "fz_pack_runs": (C.c_int, [_P, _P, _P, _P, _P, _I64, _P, C.c_int, _P, _I64, _P]),
    "fz_transpose_runs": (C.c_int, [_P, _P, _P, _P, _I64, C.c_int, _I64, _I64, _P, _P]),
    "fz_series_dist_partials": (C.c_int, [_P, C.c_int, _P, _P, _I64, _I64, _I64, _P, _P, _P]),
    "fz_series_dist_combine": (C.c_int, [_P, C.c_int, _P, _I64, _I64, _P, _P]),
}

_lib = None


def load_library(path: str = LIB_PATH):
    """dlopen libfz and bind every exported symbol (works without a GPU: no HIP call is made)."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"libfz not built: {path} is missing (run __graft_entry__.build())")
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.fz_abi_version() != 1:
        raise RuntimeError("libfz ABI version mismatch")
    if path == LIB_PATH:
        _lib = lib
    return lib


class FzError(RuntimeError):
    pass


def _check(lib, rc):
    if rc != 0:
        raise FzError(f"libfz error {rc}: {lib.fz_last_error().decode(errors='replace')}")


def _torch():
    import torch
    if not torch.cuda.is_available():
        raise RuntimeError("the fz engine needs a ROCm GPU (torch.cuda.is_available() is False); "
                           "there is no CPU fallback - use oracle/ only as a test checker")
    return torch


@dataclass
class DeviceTables:
    """The four session tables as device columns (HBM), plus the host ``Tables`` they came from
    (text pools stay on the host: the renderer needs them, the kernels never do)."""
    host: Tables
    cols: dict
    fz: FzTables

    @property
    def n_rows(self):
        return self.host.n_rows


class Graph:
    """A recorded analysis sequence of one engine (Engine.record)."""

    def __init__(self, eng, handle):
        self.eng, self.handle = eng, handle

    def launch(self):
        _check(self.eng.lib, self.eng.lib.fz_graph_launch(self.eng.ctx, self.handle))

    def close(self):
        if self.handle:
            self.eng.lib.fz_graph_destroy(self.handle)
            self.handle = None


class Engine:
    """One engine per GPU: a ``fz_ctx`` bound to torch's current stream on ``device``."""

    def __init__(self, device: int = 0, lib_path: str = LIB_PATH):
        self.torch = _torch()
        self.lib = load_library(lib_path)
        self.device = device
        self.dev = self.torch.device("cuda", device)
        self.stream = self.torch.cuda.current_stream(self.dev)
        ctx = _P()
        _check(self.lib, self.lib.fz_ctx_create(device, _P(self.stream.cuda_stream), C.byref(ctx)))
        self.ctx = ctx
        self.tables: Optional[DeviceTables] = None
        self.stats: Optional[FzStoreStats] = None

    def child(self) -> "Engine":
        """An engine for one analysis thread: its own HIP stream and fz context over THIS engine's
        store (fz_ctx_create_child) - the analyses of one store run concurrently, one child each.
        Its stream waits for the parent's work enqueued so far (the store build); call
        ``join_children`` on the parent before it rebuilds the store."""
        ch = Engine.__new__(Engine)
        ch.torch, ch.lib, ch.device, ch.dev = self.torch, self.lib, self.device, self.dev
        ch.stream = self.torch.cuda.Stream(device=self.dev)
        ctx = _P()
        _check(self.lib, self.lib.fz_ctx_create_child(self.ctx, _P(ch.stream.cuda_stream), C.byref(ctx)))
        ch.ctx = ctx
        ch._parent = self
        ch._share()
        self.__dict__.setdefault("_children", []).append(ch)
        return ch

    def follow_parent(self):
        """(child) order this child's next work after everything enqueued on the parent stream."""
        self.stream.wait_stream(self._parent.stream)
        self._share()

    _SHARED = ("tables", "stats", "groups")

    def _share(self):
        for k in self._SHARED:
            if k in self._parent.__dict__:
                setattr(self, k, getattr(self._parent, k))

    def record(self, fn) -> "Graph":
        """Record ``fn(self)`` - a fixed sequence of analysis launches on this engine (no host
        sync; warm: run once before) - as a HIP graph (fz_capture_begin/end); ``Graph.launch()``
        replays it on this engine's stream."""
        _check(self.lib, self.lib.fz_capture_begin(self.ctx))
        try:
            fn(self)
        finally:
            g = _P()
            rc = self.lib.fz_capture_end(self.ctx, C.byref(g))
        _check(self.lib, rc)
        return Graph(self, g)

    def set_store_helpers(self, helpers):
        """Let build_store fork its independent sorts onto these children's streams / contexts
        (fz_store_set_helpers; they must be idle while the store is built - join_children /
        follow_parent order them as usual).  [] turns it off."""
        arr = (_P * max(len(helpers), 1))(*[h.ctx for h in helpers])
        _check(self.lib, self.lib.fz_store_set_helpers(self.ctx, arr, len(helpers)))
        self._helpers = list(helpers)

    def join_children(self):
        """(parent) order the parent stream after all its children's enqueued work."""
        for ch in self.__dict__.get("_children", []):
            self.stream.wait_stream(ch.stream)

    def close(self):
        for ch in self.__dict__.pop("_children", []):
            ch.close()
        parent = self.__dict__.get("_parent")
        if parent is not None and self in parent.__dict__.get("_children", []):
            parent._children.remove(self)
        if getattr(self, "ctx", None):
            self.lib.fz_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- columnar loader: host columns -> HBM -------------------------------------------------
    _TORCH_DT = {np.dtype(np.int64): "int64", np.dtype(np.int32): "int32", np.dtype(np.uint8): "uint8",
                 np.dtype(np.float64): "float64"}

    def upload(self, t: Tables) -> DeviceTables:
        """Stream the typed columns to HBM: every column is copied (host memcpy) into ONE reusable
        pinned staging buffer at a 256-byte aligned offset, then ONE async H2D copy on the engine
        stream moves the whole image into a device buffer whose typed slices are the columns.  The
        dictionary encodings (group key, canonical revisions, corpus columns) come from the table's
        cache (persisted by store.save_columnar), so a re-upload does no per-row Python work.
        ``self.upload_ms`` = {"host": staging memcpy, "h2d": the copy's device time}."""
        import time as _time
        torch = self.torch
        h0 = _time.perf_counter()
        P = len(t.projects)
        c_valid = (t.c_coverage_valid.astype(np.uint8) * VALID_COVERAGE
                   | t.c_covered_valid.astype(np.uint8) * VALID_COVERED
                   | t.c_total_valid.astype(np.uint8) * VALID_TOTAL)
        pi_count = np.bincount(t.pi_project.astype(np.int64), minlength=P).astype(np.int32)
        from .rq.common import corpus_columns
        member, corpus_us, order = corpus_columns(t)
        host = {
            "b_project": t.b_project.view(np.int32), "b_type": t.b_type, "b_result": t.b_result,
            "b_time": t.b_time, "b_group": t.group_key(), "b_rev_canon": t.rev_canon(),
            "c_project": t.c_project.view(np.int32), "c_date": t.c_date, "c_coverage": t.c_coverage,
            "c_covered": t.c_covered, "c_total": t.c_total, "c_valid": c_valid,
            "i_number": t.i_number, "i_project": t.i_project.view(np.int32), "i_rts": t.i_rts,
            "i_status": t.i_status, "pi_count": pi_count,
            "g_member": member, "g_corpus_us": corpus_us, "g_order": order,
        }
        layout, total = {}, 0
        for k, a in host.items():
            nbytes = int(a.size) * a.dtype.itemsize
            layout[k] = (total, int(a.size), a.dtype)
            total += (nbytes + 255) // 256 * 256 or 256
        stage = self._staging(total)
        sn = stage.numpy()
        for k, a in host.items():
            off, n, dt = layout[k]
            if n:
                sn[off:off + n * dt.itemsize] = np.ascontiguousarray(a).reshape(-1).view(np.uint8)
        h1 = _time.perf_counter()
        dbuf = torch.empty(total, dtype=torch.uint8, device=self.dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self.stream):
            e0.record(self.stream)
            dbuf.copy_(stage[:total], non_blocking=True)
            e1.record(self.stream)
        self._stage_event = e1  # the staging buffer is reused only after this copy has finished
        cols = {}
        for k, (off, n, dt) in layout.items():
            tdt = getattr(torch, self._TORCH_DT[np.dtype(dt)])
            cols[k] = dbuf[off:off + max(n, 1) * dt.itemsize].view(tdt)
        cols["_image"] = dbuf
        ptr = {k: _P(v.data_ptr()) for k, v in cols.items() if not k.startswith(("g_", "_"))}
        fz = FzTables(n_projects=P, n_builds=len(t.b_project), n_cov=len(t.c_project), n_issues=len(t.i_project),
                      **ptr)
        self.tables = DeviceTables(host=t, cols=cols, fz=fz)
        self.groups = FzRq4Groups(member=_P(cols["g_member"].data_ptr()),
                                  corpus_us=_P(cols["g_corpus_us"].data_ptr()),
                                  order=_P(cols["g_order"].data_ptr()), n_order=len(order))
        self._upload_events = (e0, e1)
        self._upload_host_ms = (h1 - h0) * 1e3
        self._upload_bytes = total
        return self.tables

    def upload_timing(self):
        """After an upload has completed: {"host_ms": staging memcpy + encode lookups, "h2d_ms":
        device time of the copy, "bytes": image size, "h2d_gbs": its PCIe rate}."""
        e0, e1 = self._upload_events
        e1.synchronize()
        ms = e0.elapsed_time(e1)
        return {"host_ms": round(self._upload_host_ms, 3), "h2d_ms": round(ms, 3), "bytes": self._upload_bytes,
                "h2d_gbs": round(self._upload_bytes / (ms * 1e-3) / 1e9, 2) if ms > 0 else None}

    def _staging(self, nbytes):
        """The pinned host staging buffer (grown, never shrunk; waits for the last copy out of it)."""
        ev = getattr(self, "_stage_event", None)
        if ev is not None:
            ev.synchronize()
        st = getattr(self, "_stage", None)
        if st is None or st.numel() < nbytes:
            st = self.torch.empty(max(nbytes, 1), dtype=self.torch.uint8, pin_memory=True)
            self._stage = st
        return st

    # ---- store ---------------------------------------------------------------------------------
    def build_store(self, dt: Optional[DeviceTables] = None) -> FzStoreStats:
        dt = dt or self.tables
        if dt is None:
            raise FzError("no tables uploaded")
        st = FzStoreStats()
        _check(self.lib, self.lib.fz_store_build(self.ctx, C.byref(dt.fz), C.byref(st)))
        self.tables = dt
        self.stats = st
        return st

    # ---- helpers ------------------------------------------------------------------------------
    def empty(self, n, dtype):
        return self.torch.empty(max(int(n), 1), dtype=dtype, device=self.dev)

    def zeros(self, n, dtype):
        return self.torch.zeros(max(int(n), 1), dtype=dtype, device=self.dev)

    def synchronize(self):
        self.stream.synchronize()

    def radix_sort(self, keys, vals=None, bits=64):
        n = keys.numel()
        _check(self.lib, self.lib.fz_radix_sort_u64(self.ctx, _P(keys.data_ptr()),
                                                   _P(vals.data_ptr()) if vals is not None else None, n, bits))

    def sort_f64(self, x):
        """Stable sort of a device float64 vector: (values ascending, int32 positions)."""
        n = x.numel()
        val = self.torch.empty(max(n, 1), dtype=self.torch.float64, device=self.dev)
        pos = self.torch.empty(max(n, 1), dtype=self.torch.int32, device=self.dev)
        _check(self.lib, self.lib.fz_sort_f64(self.ctx, _P(x.data_ptr()) if n else None, n,
                                              _P(val.data_ptr()), _P(pos.data_ptr())))
        return val[:n], pos[:n]

    def probe_begin(self, kernel: str):
        _check(self.lib, self.lib.fz_probe_begin(self.ctx, kernel.encode()))

    def probe_end(self):
        """-> (launches, total device ms, algorithmic bytes) of the probed kernel."""
        n, ms, b = _I64(), C.c_double(), C.c_double()
        _check(self.lib, self.lib.fz_probe_end(self.ctx, C.byref(n), C.byref(ms), C.byref(b)))
        return int(n.value), float(ms.value), float(b.value)

    def probe_get(self, kernel: str):
        """After probe_end: (launches, total device ms, algorithmic bytes) of any probed kernel."""
        n, ms, b = _I64(), C.c_double(), C.c_double()
        _check(self.lib, self.lib.fz_probe_get(self.ctx, kernel.encode(), C.byref(n), C.byref(ms), C.byref(b)))
        return int(n.value), float(ms.value), float(b.value)

    def describe(self, x):
        d = FzDescribe()
        _check(self.lib, self.lib.fz_describe_f64(self.ctx, _P(x.data_ptr()), x.numel(), C.byref(d)))
        return d

    # ---- finishing entry points over caller-supplied tables (no store needed) ------------------
    def _dev(self, a, dtype):
        t = self.torch.as_tensor(np.ascontiguousarray(a), dtype=dtype)
        return t.to(self.dev) if t.numel() else self.torch.zeros(1, dtype=dtype, device=self.dev)

    def rq1_finish(self, iter_total, iter_detected, threshold: int = 100):
        """fz_rq1_finish (rq1_detection_rate.py:233-268) on host per-iteration tables ->
        (counts[FZ_RQ1_NCOUNTS], late fz_describe as 13 doubles), host copies."""
        torch = self.torch
        it = self._dev(iter_total, torch.int64)
        idt = self._dev(iter_detected, torch.int64)
        counts = self.zeros(FZ_RQ1_NCOUNTS, torch.int64)
        late = self.zeros(DESCRIBE_DOUBLES, torch.float64)
        _check(self.lib, self.lib.fz_rq1_finish(self.ctx, threshold, _P(it.data_ptr()), _P(idt.data_ptr()),
                                                len(iter_total), _P(counts.data_ptr()), _P(late.data_ptr())))
        return counts.cpu().numpy(), late.cpu().numpy()

    def rq4a_finish(self, g1_total, g1_det, g2_total, g2_det, intro, g4_steps):
        """fz_rq4a_finish (rq4a_bug.py:156-207, :698-747, :246-299, :412-510) on host tables
        (intro[n_projects]: -1 = not a G4 project) -> (counts, scalars), host copies."""
        torch = self.torch
        tabs = [self._dev(x, torch.int64) for x in (g1_total, g1_det, g2_total, g2_det)]
        it = self._dev(intro, torch.int64)
        st = self._dev(np.asarray(g4_steps, np.int64).reshape(30), torch.int64)
        counts = self.zeros(FZ_RQ4A_NCOUNTS, torch.int64)
        sc = self.zeros(FZ_RQ4A_NSCALARS, torch.float64)
        _check(self.lib, self.lib.fz_rq4a_finish(self.ctx, *[_P(x.data_ptr()) for x in tabs], len(g1_total),
                                                 _P(it.data_ptr()), len(intro), _P(st.data_ptr()),
                                                 _P(counts.data_ptr()), _P(sc.data_ptr())))
        return counts.cpu().numpy(), sc.cpu().numpy()

    def rq3_stats(self, det_pct, det_tot, non_pct):
        """fz_rq3_stats (rq3_diff_coverage_at_detection.py:25-66, :321-352) on host samples ->
        (describe [3 x 13 doubles], tests[FZ_RQ3_NTESTS]), host copies."""
        torch = self.torch
        dp, dt, nn = (self._dev(det_pct, torch.float64), self._dev(det_tot, torch.int64),
                      self._dev(non_pct, torch.float64))
        desc = self.zeros(3 * DESCRIBE_DOUBLES, torch.float64)
        tests = self.torch.full((FZ_RQ3_NTESTS,), float("nan"), dtype=torch.float64, device=self.dev)
        P = lambda t, n: _P(t.data_ptr()) if n else None  # noqa: E731
        _check(self.lib, self.lib.fz_rq3_stats(self.ctx, P(dp, len(det_pct)), P(dt, len(det_pct)), len(det_pct),
                                               P(nn, len(non_pct)), len(non_pct), _P(desc.data_ptr()),
                                               _P(tests.data_ptr())))
        return desc.cpu().numpy().reshape(3, DESCRIBE_DOUBLES), tests.cpu().numpy()

    def eligibility_counts(self, limit_us):
        out = self.zeros(self.tables.fz.n_projects, self.torch.int32)
        _check(self.lib, self.lib.fz_eligibility_count(self.ctx, C.byref(self.tables.fz), limit_us,
                                                      _P(out.data_ptr())))
        return out


def describe_from_doubles(a: np.ndarray):
    """fz_describe laid out as 13 x 8 bytes -> field dict."""
    b = np.asarray(a).view(np.uint8).tobytes()
    d = FzDescribe.from_buffer_copy(b[:C.sizeof(FzDescribe)])
    return d
