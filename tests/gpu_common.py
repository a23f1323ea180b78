"""Shared helpers for the GPU parity tests: result-object comparison (integers / index arrays
bit-exact, floating point within the north-star tolerance 1e-9 relative)."""
from __future__ import annotations

import dataclasses
import math

import numpy as np

RTOL = 1e-9
# Far-tail p-values (config 4's 1e5-1e6-point series) are ill-conditioned: p = Q(z(W)) amplifies
# the last-ulp difference of a statistic by about |ln p|, so below TAIL they are compared as -ln p
# (1e-9 relative there is still 1e-9 relative on the statistic's own scale).
TAIL = 1e-30


def _close(a, b, rtol=RTOL):
    if a is None or b is None:
        return a is b
    if isinstance(a, float) or isinstance(b, float):
        a, b = float(a), float(b)
        if math.isnan(a) or math.isnan(b):
            return math.isnan(a) and math.isnan(b)
        if math.isinf(a) or math.isinf(b):
            # non-finite values compare exactly: +inf == +inf only, never inf vs a finite value
            return a == b
        if 0.0 < a < TAIL and 0.0 < b < TAIL:
            a, b = -math.log(a), -math.log(b)
        return a == b or abs(a - b) <= rtol * max(abs(a), abs(b))
    return a == b


def assert_same(ours, ref, path="result", rtol=RTOL):
    """Field-by-field comparison of two result objects (dataclasses, dicts, arrays, scalars)."""
    if dataclasses.is_dataclass(ref):
        for f in dataclasses.fields(ref):
            assert_same(getattr(ours, f.name), getattr(ref, f.name), f"{path}.{f.name}", rtol)
        return
    if isinstance(ref, dict):
        assert set(ours) == set(ref), f"{path}: keys {sorted(ours)} != {sorted(ref)}"
        for k in ref:
            assert_same(ours[k], ref[k], f"{path}[{k!r}]", rtol)
        return
    scalar = (int, float, np.number)
    if isinstance(ref, (list, tuple)) and not (len(ref) and all(isinstance(x, scalar) and not isinstance(x, bool)
                                                                for x in ref)):
        assert len(ours) == len(ref), f"{path}: len {len(ours)} != {len(ref)}"
        for i, (a, b) in enumerate(zip(ours, ref)):
            assert_same(a, b, f"{path}[{i}]", rtol)
        return
    if isinstance(ref, (np.ndarray, list, tuple)):
        a, b = np.asarray(ours), np.asarray(ref)
        assert a.shape == b.shape, f"{path}: shape {a.shape} != {b.shape}"
        if b.dtype.kind in "iub" and a.dtype.kind in "iub":
            bad = np.nonzero(a != b)[0] if a.ndim == 1 else None
            assert np.array_equal(a, b), f"{path}: integer mismatch at {bad[:10] if bad is not None else '?'}"
        else:
            a, b = a.astype(np.float64), b.astype(np.float64)
            # non-finite values compare exactly (NaN only with NaN, +-inf only with the same
            # infinity); the tolerance applies to finite pairs only
            fin = np.isfinite(a) & np.isfinite(b)
            tail = (a > 0) & (a < TAIL) & (b > 0) & (b < TAIL)
            if tail.any():
                a, b = np.where(tail, -np.log(np.where(tail, a, 1.0)), a), np.where(tail, -np.log(np.where(tail, b, 1.0)), b)
            with np.errstate(invalid="ignore", over="ignore"):
                near = np.abs(a - b) <= rtol * np.maximum(np.abs(a), np.abs(b))
            ok = (a == b) | (np.isnan(a) & np.isnan(b)) | (fin & near)
            assert ok.all(), f"{path}: float mismatch at {np.nonzero(~ok.ravel())[0][:10]}"
        return
    assert _close(ours, ref, rtol), f"{path}: {ours!r} != {ref!r}"
