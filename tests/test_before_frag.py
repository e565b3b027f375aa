"""CPU: fd_verify_hip_before_frag == before_frag (fd_verify_tile.c:37-58),
restated here as the truth table it is, over every in-link kind, a spread of
seq values, round-robin shapes and mcache sigs (gossip: the update tag)."""
import itertools

from firedancer_amd import verify_tile as V


def ref_before_frag(kind, seq, sig, cnt, idx):
    is_bundle_packet = kind == V.IN_BUNDLE and not sig
    if is_bundle_packet or kind == V.IN_QUIC:
        return (seq % cnt) != idx
    if kind == V.IN_BUNDLE:
        return idx != 0
    if kind == V.IN_GOSSIP:
        return (seq % cnt) != idx or sig != V.GOSSIP_UPDATE_TAG_VOTE
    return False


def test_before_frag_truth_table():
    n = 0
    for kind, seq, sig, (cnt, idx) in itertools.product(
            (V.IN_QUIC, V.IN_BUNDLE, V.IN_GOSSIP, V.IN_SEND), (0, 1, 5, 6, 41, 2**40 + 3, 2**64 - 1),
            (0, 1, 2, 3, 4, 5, 2**63), ((1, 0), (6, 0), (6, 5), (42, 17))):
        assert V.before_frag(kind, seq, sig, cnt, idx) == ref_before_frag(kind, seq, sig, cnt, idx), \
            (kind, seq, sig, cnt, idx)
        n += 1
    assert n == 4 * 7 * 7 * 4
