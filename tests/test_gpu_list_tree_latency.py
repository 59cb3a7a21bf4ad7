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


# item sizes that pack 32 / 16 / 8 / 4 items per 128-B chunk, one item per
# chunk (48, 128, 200 B) and odd sizes (7, 24: a chunk of whole items short
# of 128 B); n at the form's first (17) and last (4,096) window counts, one
# either side of them, and ragged in between
_ITEM_CASES = [(8, 16 * 32 + 15), (8, 16 * 33), (8, 16 * 33 + 1), (8, 16 * 8192), (8, 16 * 8192 + 1), (16, 300),
               (32, 4097), (32, 8 * 4096 + 1), (4, 2000), (48, 35), (48, 8191), (128, 4000), (200, 33), (200, 999),
               (24, 5000), (7, 3333)]


@pytest.mark.parametrize("item_len,n", _ITEM_CASES)
def test_dev_merkle_hash_latency_form(gpu, item_len, n):
    """mk_dev_ssz_merkle_hash and the host entry through the latency form
    (and just outside it) against the oracle's merkleHash restatement."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd import ssz

    raw = O.splitmix_bytes(n * item_len, SEED + 7 * item_len + n)
    want = O.merkle_hash_flat(raw, n, item_len, nthreads=16)
    dev = torch.from_numpy(raw.copy()).to("cuda:0")
    for _ in range(2):
        got = D.merkle_hash(dev, n, item_len)
        torch.cuda.synchronize()
        assert bytes(got.cpu().numpy()) == want
    assert ssz.merkle_hash_flat(raw, n, item_len) == want
    if n > 1:  # unaligned start: the byte-wise sponge
        dev2 = torch.from_numpy(np.concatenate([np.zeros(3, np.uint8), raw])).to("cuda:0")[3:]
        got = D.merkle_hash(dev2, n, item_len)
        torch.cuda.synchronize()
        assert bytes(got.cpu().numpy()) == want
