"""CPU: the bench tile leg's drop-free rate search (tools/svc_link_sweep.py:
drop_free_search, judge_rate) on a synthetic stage whose loss is a step
function of the offered rate, with and without a one-off collapse."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import svc_link_sweep as SL   # noqa: E402


def stage(limit, collapse_at=()):
    """run(rate): loses frags above limit; the k-th call in collapse_at loses frags regardless."""
    calls = [0]

    def run(rate):
        calls[0] += 1
        bad = rate > limit or calls[0] in collapse_at
        return {"offered_rate": rate, "overrun": 1000 if bad else 0, "lapped": 0, "unseen": 0}
    return run, calls


def test_single_vote_follows_every_run():
    run, _ = stage(20e6)
    best, tried = SL.drop_free_search(run, 29e6, 2e6, 4)
    assert best is not None and best["offered_rate"] <= 20e6
    assert len(tried) == 5
    # one collapse on the first bisection step sends a single-vote search low
    run, _ = stage(20e6, collapse_at={2})
    best1, _ = SL.drop_free_search(run, 29e6, 2e6, 4)
    assert best1["offered_rate"] < 7.7e6


def test_majority_vote_outlasts_one_collapse():
    run, _ = stage(20e6)
    clean, _ = SL.drop_free_search(run, 29e6, 2e6, 4, votes=3)
    run, _ = stage(20e6, collapse_at={3})          # the first run at the first mid-rate collapses
    best, tried = SL.drop_free_search(run, 29e6, 2e6, 4, votes=3)
    assert best["offered_rate"] == clean["offered_rate"]
    assert best["offered_rate"] <= 20e6
    assert sum(1 for _, r in tried if SL.lost(r)) >= 3       # every run is kept, lossy ones too


def test_judge_rate_stops_once_decided():
    run, calls = stage(10e6)
    tried = []
    assert SL.judge_rate(run, 5e6, tried, 3)[0] and calls[0] == 2
    assert not SL.judge_rate(run, 15e6, tried, 3)[0] and calls[0] == 4
    assert len(tried) == 4


def test_nothing_passes():
    run, _ = stage(1e6)
    best, tried = SL.drop_free_search(run, 29e6, 2e6, 3, votes=3)
    assert best is None and all(SL.lost(r) for _, r in tried)
