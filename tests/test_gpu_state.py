"""State tree hash: TreeHash of a synthetic, SSZ-legal
pb.BeaconState (proto/beacon/p2p/v1/types.pb.go:50-79) through the engine's
batched path (prysm_amd/state.py) and the reflective mirror
(prysm_amd.ssz.tree_hash), both against the oracle's restatement of the
reference's reflective hasher (oracle/ssz_ref.py, shared/ssz/hash.go:23-239)."""
import json
import os

import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 700
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    assert _lib.device_count() >= 1
    return torch.device("cuda:0")


@pytest.mark.parametrize("nv,natt,nb,nvotes,lists", [(1000, 128, 16, 4, 8192), (0, 0, 0, 0, 8192),
                                                      (37, 3, 1, 1, 5), (4099, 257, 33, 9, 1000)])
def test_state_root_vs_oracle(gpu, nv, natt, nb, nvotes, lists):
    from oracle import ssz_ref as OS
    from prysm_amd import ssz
    from prysm_amd import state as ST
    from tests.ssz_types import to_ref_type

    st = ST.synthetic_state(nv, SEED + nv, n_attestations=natt, n_batched=nb, n_votes=nvotes, lists_len=lists,
                            shards=min(1024, lists))
    val = st.as_value()
    want = OS.tree_hash(to_ref_type(ST.STATE_SSZ), val)
    assert st.tree_hash_ssz() == want
    assert ssz.tree_hash(val, ST.STATE_SSZ) == want


def test_state_nil_fork_is_the_reference_error(gpu):
    from prysm_amd import ssz
    from prysm_amd import state as ST

    val = ST.synthetic_state(10, SEED, n_attestations=2).as_value()
    val["Fork"] = None
    with pytest.raises(ssz.HashError) as ei:
        ssz.tree_hash(val, ST.STATE_SSZ)
    assert str(ei.value) == ("hash error: failed to hash field of struct: nil is not supported "
                             "for input type pb.BeaconState")


def test_full_size_state_root(gpu):
    """1,000,000 validators, 8192-entry root arrays, 1024 crosslinks, 128
    attestations: the golden root of tests/golden/full_size_roots.json."""
    from prysm_amd import state as ST

    with open(os.path.join(ROOT, "tests", "golden", "full_size_roots.json")) as f:
        g = json.load(f)["c3_state"]
    st = ST.synthetic_state(g["n"], g["seed"])
    assert st.tree_hash_ssz().hex() == g["state_root"]
