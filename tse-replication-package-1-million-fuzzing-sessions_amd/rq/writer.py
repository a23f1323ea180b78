"""Native byte-exact CSV writers (csrc/fz_write.cpp, ``lib/libfzwrite.so``; include/fz_write.h).

The reference writes its large result tables with ``csv.writer``: coverage_by_session_index.csv
(rq2_coverage_count.py:347-352, one ``repr(float)`` per coverage value - 1e8 of them at config 3)
and the change-point tables (rq2_coverage_and_added.py:221-238: 13 mixed cells per row, every row
twice - its project's file and the all-projects file).  These wrappers format the same bytes in
C++ worker threads; ``rq/render.py`` uses them when the library is built and its own
``csv.writer`` path otherwise (both are held to each other by tests/test_writer.py)."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lib", "libfzwrite.so")
_lib = None
_tried = False


class _ChangeCols(C.Structure):
    _fields_ = [(k, C.c_void_p) for k in ("project", "t_end", "mod_f", "rev_f", "t_start", "mod_s", "rev_s",
                                          "cov_i", "cov_i1", "diff_total", "diff_coverage", "c_covered", "c_total",
                                          "c_covered_valid", "c_total_valid", "covered_is_float", "total_is_float",
                                          "proj_blob", "proj_off", "mod_blob", "mod_off", "rev_blob", "rev_off")]


def lib():
    """The loaded libfzwrite, or None when it is not built (FZ_WRITER=python forces None)."""
    global _lib, _tried
    if os.environ.get("FZ_WRITER") == "python":
        return None
    if not _tried:
        _tried = True
        if os.path.exists(_LIB):
            L = C.CDLL(_LIB)
            P, I64 = C.c_void_p, C.c_int64
            L.fzw_float_rows.restype = I64
            L.fzw_float_rows.argtypes = [P, P, I64, P, I64, C.c_int]
            L.fzw_float_rows_cap.restype = I64
            L.fzw_float_rows_cap.argtypes = [P, I64]
            L.fzw_change_rows.restype = I64
            L.fzw_change_rows.argtypes = [C.POINTER(_ChangeCols), I64, P, I64, P, C.c_int]
            L.fzw_change_rows_cap.restype = I64
            L.fzw_change_rows_cap.argtypes = [C.POINTER(_ChangeCols), I64]
            L.fzw_repr.restype = C.c_int
            L.fzw_repr.argtypes = [C.c_double, C.c_char_p]
            _lib = L
    return _lib


def _threads() -> int:
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    return max(1, min(32, n))


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data) if a.size else None


def repr_float(v: float) -> str:
    """repr(float) through the native formatter (tests)."""
    buf = C.create_string_buffer(40)
    n = lib().fzw_repr(float(v), buf)
    return buf.raw[:n].decode()


def float_rows(vals: np.ndarray, offs: np.ndarray) -> bytes:
    """csv.writer rows of floats: row i = vals[offs[i]:offs[i + 1]] ("\\r\\n" after every row)."""
    L = lib()
    vals = np.ascontiguousarray(vals, dtype=np.float64)
    offs = np.ascontiguousarray(offs, dtype=np.int64)
    nrows = len(offs) - 1
    if nrows <= 0:
        return b""
    cap = int(L.fzw_float_rows_cap(_ptr(offs), nrows))
    out = np.empty(max(cap, 1), dtype=np.uint8)
    n = int(L.fzw_float_rows(_ptr(vals), _ptr(offs), nrows, _ptr(out), cap, _threads()))
    if n < 0:
        raise RuntimeError("fzw_float_rows: output bound exceeded")
    return out[:n].tobytes()


def _pool_blob(pool):
    """(bytes, offsets[len + 1]) of a string pool (None -> empty; never read: ids < 0 mean None)."""
    enc = [(s or "").encode("utf-8") for s in pool]
    off = np.zeros(len(enc) + 1, dtype=np.int64)
    if enc:
        off[1:] = np.cumsum([len(b) for b in enc])
    blob = np.frombuffer(b"".join(enc) or b"\0", dtype=np.uint8)
    return blob, off


def pool_blobs(t):
    """The tables' project / modules / revisions pools as blobs (cached on the tables)."""
    return t.cached("writer_pools", (t.projects, t.modules_pool, t.revisions_pool),
                    lambda: (_pool_blob(t.projects), _pool_blob(t.modules_pool), _pool_blob(t.revisions_pool)))


def change_rows(r, t):
    """The rq2_coverage_and_added.py change rows of result r (RQ2AddResult) over tables t, every row
    formatted once -> (bytes of all rows, row_end[k] = byte offset after row k)."""
    L = lib()
    n = len(r.row_project)
    if n == 0:
        return b"", np.zeros(0, dtype=np.int64)
    i64 = lambda a: np.ascontiguousarray(a, dtype=np.int64)  # noqa: E731
    u8 = lambda a: np.ascontiguousarray(a, dtype=np.uint8)  # noqa: E731
    f, e, s = i64(r.row_first_build), i64(r.row_end_build), i64(r.row_start_build)
    keep = {
        "project": i64(r.row_project), "t_end": i64(t.b_time[e]), "mod_f": i64(t.b_modules[f]),
        "rev_f": i64(t.b_revisions[f]), "t_start": i64(t.b_time[s]), "mod_s": i64(t.b_modules[s]),
        "rev_s": i64(t.b_revisions[s]), "cov_i": i64(r.row_cov_i), "cov_i1": i64(r.row_cov_i1),
        "diff_total": np.ascontiguousarray(r.diff_total, dtype=np.float64),
        "diff_coverage": np.ascontiguousarray(r.diff_coverage, dtype=np.float64),
        "c_covered": i64(t.c_covered), "c_total": i64(t.c_total), "c_covered_valid": u8(t.c_covered_valid),
        "c_total_valid": u8(t.c_total_valid), "covered_is_float": u8(r.covered_is_float),
        "total_is_float": u8(r.total_is_float)}
    (pb, po), (mb, mo), (rb, ro) = pool_blobs(t)
    keep.update(proj_blob=pb, proj_off=po, mod_blob=mb, mod_off=mo, rev_blob=rb, rev_off=ro)
    cols = _ChangeCols(**{k: (v.ctypes.data if v.size else None) for k, v in keep.items()})
    cap = int(L.fzw_change_rows_cap(C.byref(cols), n))
    out = np.empty(max(cap, 1), dtype=np.uint8)
    row_end = np.empty(n, dtype=np.int64)
    m = int(L.fzw_change_rows(C.byref(cols), n, _ptr(out), cap, _ptr(row_end), _threads()))
    if m < 0:
        raise RuntimeError("fzw_change_rows: output bound exceeded")
    return out[:m].tobytes(), row_end
