"""CPU: the verify tile's batch latency histograms use fd_histf's bucket
edges (src/util/hist/fd_histf.h:40-118).  fd_verify_hip_hist_edges against
the worked example in that header's comment (min 1, max 100), against the
edge rule restated here over a spread of ranges, and its argument checks."""
import numpy as np
import pytest

from firedancer_amd import verify_tile as V


def ref_edges(lo, hi, n=16):
    """fd_histf_new's rule: [0, lo), then each interior edge spreads the
    remaining ratio hi/edge over the buckets left (rounded, strictly
    increasing), then [hi, inf)."""
    lo = max(lo, 1)
    hi = max(hi, lo + n - 2)
    e = [0, lo]
    for i in range(2, n - 1):
        x = int(0.5 + e[-1] * (hi / e[-1]) ** (1.0 / (n - i)))
        e.append(max(x, e[-1] + 1))
    return e + [hi]


def test_edges_match_the_header_example():
    assert V.hist_edges(1, 100).tolist() == [0, 1, 2, 3, 4, 5, 7, 9, 12, 16, 22, 30, 41, 55, 74, 100]


@pytest.mark.parametrize("lo,hi", [(1, 2), (1, 15), (3, 20), (10, 10_000), (10_000, 1_000_000_000),
                                   (1_000, 50_000_000), (7, 2**40), (0, 100), (100, 101)])
def test_edges_rule(lo, hi):
    got = V.hist_edges(lo, hi)
    assert got.tolist() == ref_edges(lo, hi)
    assert np.all(np.diff(got.astype(np.int64)) > 0)             # no empty bucket


def test_edges_reject_empty_range():
    for lo, hi in ((5, 5), (9, 3)):
        with pytest.raises(ValueError):
            V.hist_edges(lo, hi)
