"""CPU checks of the half-size scalar model (tools/halfsize_model.py), the
reference the GPU test (test_gpu_halfsize.py) holds the device reduction to:
k1 == k*k2 (mod 8L), k2 odd and positive, the fallback pair (k, 1) for
scalars whose first quotients overflow 32 bits, and the window counts the
DSM kernel is sized for (W is the reference's; this is the
executed work)."""
import os
import random
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import halfsize_model as HM  # noqa: E402


def test_invariants_random_and_edges():
    rng = random.Random(11)
    ks = [rng.randrange(HM.L) for _ in range(3000)]
    ks += [0, 1, 2, 2**127, 2**128 - 1, 2**128, HM.L - 1, HM.M // 2**40, HM.M // (2**32 + 1)]
    for k in ks:
        r, t, b, _ = HM.halfsize(k)
        assert t > 0 and t % 2 == 1 and t < HM.L
        assert (r - k * t) % HM.M == 0
        assert b == max(abs(r).bit_length(), t.bit_length())


def test_fallback_on_large_quotient():
    k = HM.M // 2**40                       # first quotient ~2^40
    r, t, b, _ = HM.halfsize(k)
    assert (r, t) == (k, 1) and b == k.bit_length()


def test_window_counts():
    rng = random.Random(12)
    bits = [HM.halfsize(rng.randrange(HM.L))[2] for _ in range(64 * 40)]
    wins = [max(31, HM.windows(b)) for b in bits]
    waves = [max(wins[i:i + 64]) for i in range(0, len(wins), 64)]
    assert max(bits) <= 150
    assert 33 <= sum(waves) / len(waves) <= 34.5      # vs 64 windows for the full-length scalar
