"""The latency form of a small list's tree (capi.cpp dev_list_tree_32:
k_spread_leaf<8> + k_merkle_top_fused in spans of 16 nodes) for the TreeHash
of a []ValidatorRecord (hash.go:118-139 -> merkleHash, hash.go:194-239),
device records, at every boundary of the form: the first size that takes it
(17 windows), ragged last windows / workgroups / groups, one group exactly,
C1's 16,384, the last size (2^12 windows) and the first after it (general
plan).  Checked against the oracle's struct roots + merkleHash restatement."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000C1


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    assert _lib.device_count() >= 1, "libprysm_merkle.so sees no gfx950 device"
    _lib.init(0)
    return torch.device("cuda:0")


@pytest.mark.parametrize("n", [129, 130, 131, 256, 511, 1000, 4097, 8191, 16_383, 16_385, 32_767, 32_768, 32_769])
def test_dev_struct_list_root_latency_form(gpu, n):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd import registry as R

    reg = R.synthetic_registry(n, SEED + n)
    raw = reg.records.view(np.uint8).reshape(-1)
    spec = [(k, o, l) for k, o, l in R.VALIDATOR_FIELDS]
    roots = O.struct_roots(raw, n, 160, spec, nthreads=16)
    want = O.merkle_hash_flat(roots.reshape(-1), n, 32, nthreads=16)
    drec = torch.from_numpy(raw.copy()).to("cuda:0")
    for _ in range(3):  # back to back: the arrival counters reset between launches
        got = D.struct_list_root(drec, n, 160, R.VALIDATOR_FIELDS)
        torch.cuda.synchronize()
        assert bytes(got.cpu().numpy()) == want
    assert reg.tree_hash_ssz() == want  # the host-records entry, same plan
