"""GPU parity of the segmented (many-lists) merkleHash, mk_ssz_merkle_many /
mk_dev_ssz_merkle_many: every list's root equals the oracle's merkleHash of
that list (shared/ssz/hash.go:194-239), for empty, one-chunk, ragged, odd
item sizes, unaligned offsets and lists long enough to take their own fused
plan (> 2^15 chunks)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 600


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    assert _lib.device_count() >= 1
    return torch.device("cuda:0")


_SHAPES = [(0, 32), (1, 32), (4, 32), (5, 32), (8, 32), (9, 32), (37, 32), (1000, 32), (4099, 32),
           (0, 8), (1, 8), (16, 8), (17, 8), (100_003, 8), (3, 1), (129, 1), (7, 2), (1000, 4),
           (11, 48), (5, 128), (6, 200), (2, 300), (70_001, 32), ((1 << 17) + 3, 32), (1 << 18, 32)]


def _lists(shapes, seed):
    from oracle import oracle as O

    return [O.splitmix_bytes(max(8, n * il + (-(n * il)) % 8), seed + i)[:n * il] for i, (n, il) in enumerate(shapes)]


def test_host_many_vs_oracle(gpu):
    from oracle import oracle as O
    from prysm_amd import ssz

    for il in sorted({il for _, il in _SHAPES}):
        shapes = [s for s in _SHAPES if s[1] == il]
        data = _lists(shapes, SEED + il)
        got = ssz.merkle_many(data, [n for n, _ in shapes], il)
        for (n, _), a, r in zip(shapes, data, got):
            assert r == O.merkle_hash_flat(a, n, il, nthreads=8), (n, il)


@pytest.mark.parametrize("align", [16, 4, 1])
def test_dev_many_mixed_item_sizes(gpu, align):
    """One call over lists of different item sizes at `align`-aligned offsets
    (unaligned lists take the generic sponge windows)."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    shapes = _SHAPES
    data = _lists(shapes, SEED + 1000 + align)
    offs, pos, parts = [], 0, []
    for a in data:
        pad = (-pos) % align + (3 if align == 1 else 0)
        parts.append(np.zeros(pad, np.uint8))
        pos += pad
        offs.append(pos)
        parts.append(a)
        pos += a.size
    buf = np.concatenate(parts + [np.zeros(16, np.uint8)])
    items = torch.from_numpy(buf).to(gpu)
    roots = D.merkle_many(items, offs, [n for n, _ in shapes], [il for _, il in shapes])
    torch.cuda.synchronize()
    got = roots.cpu().numpy().reshape(-1, 32)
    for i, ((n, il), a) in enumerate(zip(shapes, data)):
        assert bytes(got[i]) == O.merkle_hash_flat(a, n, il, nthreads=8), (i, n, il)


def test_many_16k_small_lists(gpu):
    """16,384 lists of 0..40 uint32 (a [][]uint32 field of a 16k registry):
    one leaf launch + one launch per level for all of them."""
    from oracle import oracle as O
    from prysm_amd import ssz

    rng = np.random.default_rng(9)
    ns = rng.integers(0, 41, 16_384)
    data = [rng.integers(0, 1 << 32, int(n), dtype=np.uint32).view(np.uint8) for n in ns]
    got = ssz.merkle_many(data, [int(n) for n in ns], 4)
    for i in range(0, 16_384, 97):
        assert got[i] == O.merkle_hash_flat(data[i], int(ns[i]), 4), i


def test_many_zero_item_len_panics(gpu):
    from prysm_amd import ssz

    with pytest.raises(ZeroDivisionError):
        ssz.merkle_many([np.zeros(0, np.uint8)], [3], 0)
