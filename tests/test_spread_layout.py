"""The one-state-per-wave Keccak layout (mk::spread, keccak_dev.hpp) as a
lane-by-lane CPU emulation (tools/spread_emu.py: DPP row shifts/rotates
with row masks, v_permlane16/32_swap, ds_bpermute) against the oracle's
textbook Keccak-f[1600] (oracle.py_keccak_f): both word forms, random
states.  The GPU side of the same layout is checked bit-exact by
tools/lat_probe.hip and by every trie / merkleHash parity test."""
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_spread_layout_matches_keccak_f():
    import spread_emu as E
    from oracle import oracle as O

    rng = random.Random(0x5EED)
    for _ in range(3):
        A = [rng.getrandbits(64) for _ in range(25)]
        want = O.py_keccak_f(list(A))
        assert E.keccak_f(A) == want
        assert E.run_ilv(A) == want
        assert E.run_lh(A) == want


def test_spread_lane_constants():
    """Every Keccak lane has exactly one canonical GPU lane; pi sources are
    canonical lanes; the mirrors (groups 5-7) carry row 4."""
    import spread_emu as E

    canon = {}
    for L, c in enumerate(E.CS):
        g, q = L >> 3, L & 7
        if g < 5 and q < 5:
            assert c["i"] not in canon
            canon[c["i"]] = L
        if g >= 5:
            assert c["i"] // 5 == 4
        src = c["src"] // 4
        assert (src >> 3) < 5 and (src & 7) < 5
    assert sorted(canon) == list(range(25))
