"""The GPU parity comparator (`tests/gpu_common.py`) itself: non-finite values compare exactly.

Statistics that can legitimately be infinite (rq3_diff_coverage_at_detection.py:321-352's
Anderson / Levene on degenerate samples, rq2_coverage_count.py:316-322's Spearman t on perfectly
monotone series) must match the reference's infinity with the same sign; a finite value never
matches an infinity and NaN only matches NaN."""
import numpy as np
import pytest

from gpu_common import assert_same


@pytest.mark.parametrize("a,b", [
    (float("inf"), 5.0), (5.0, float("inf")), (float("-inf"), float("inf")),
    (float("nan"), 1.0), (1.0, float("nan")), (float("inf"), float("nan")),
    (1e300, float("inf")), (1.0, 1.0 + 1e-6),
])
def test_scalar_mismatch_fails(a, b):
    with pytest.raises(AssertionError):
        assert_same(a, b)


@pytest.mark.parametrize("a,b", [
    ([np.inf, -np.inf], [1e300, np.inf]), ([np.inf], [5.0]), ([-np.inf], [np.inf]),
    ([np.nan], [0.0]), ([0.0], [np.nan]), ([np.inf, 1.0], [np.nan, 1.0]),
    ([1.0, 2.0], [1.0, 2.0 + 1e-6]),
])
def test_array_mismatch_fails(a, b):
    with pytest.raises(AssertionError):
        assert_same(np.array(a), np.array(b))


def test_matches_pass():
    assert_same(float("inf"), float("inf"))
    assert_same(float("-inf"), float("-inf"))
    assert_same(float("nan"), float("nan"))
    assert_same(1.0, 1.0 + 1e-12)
    assert_same(np.array([np.inf, -np.inf, np.nan, 1.0, 1e-40]),
                np.array([np.inf, -np.inf, np.nan, 1.0 + 1e-12, 1e-40 * (1 + 1e-12)]))
    assert_same({"x": [np.inf, 2.0]}, {"x": [np.inf, 2.0]})


def test_no_warnings_on_infinities():
    with np.errstate(all="raise"):
        assert_same(np.array([np.inf, -np.inf, np.nan]), np.array([np.inf, -np.inf, np.nan]))
