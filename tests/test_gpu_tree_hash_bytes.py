"""ssz.TreeHash of a list of byte strings on the device in one call
(mk_ssz_tree_hash_bytes_list / mk_dev_ssz_tree_hash_bytes_list): every
element hashed as Keccak(le32(len) || element) (hashedEncoding,
shared/ssz/hash.go:100-107) and merkleHash over those digests
(makeSliceHasher, hash.go:118-139).  32-B elements above 2^20 run the fused
leaf kernel (k_reduce_elem: digests never reach HBM); everything else the
two-phase form.  Oracle: oracle.tree_hash_bytes_list (the pinned Keccak and
merkleHash restatements composed) and, at small sizes, the reflective
restatement oracle/ssz_ref.py; the full 2^28 root against
tests/golden/full_size_roots.json (c4tree)."""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SEED = 0x5EED000000000000 + 0x7E
FUSED_MIN = 8 * (1 << 17) + 1  # more than 2^17 windows: the leaf pass is a throughput pass


@pytest.fixture(scope="module")
def gpu():
    import torch

    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _dev_root(items_host: np.ndarray, n: int, L: int, gpu, offset: int = 0) -> bytes:
    import torch

    from prysm_amd import device as D

    buf = torch.zeros(items_host.size + offset + 16, dtype=torch.uint8, device=gpu)
    if items_host.size:
        buf[offset:offset + items_host.size] = torch.from_numpy(items_host.copy()).to(gpu)
    out = D.tree_hash_bytes_list(buf[offset:], n, L)
    torch.cuda.synchronize()
    return bytes(out.cpu().numpy())


@pytest.mark.parametrize("n", [0, 1, 2, 3, 4, 5, 7, 8, 9, 12, 13, 16, 17, 31, 33, 100, 1000, 4099, 65_536 + 3,
                               FUSED_MIN - 1, FUSED_MIN, FUSED_MIN + 7, 1 << 21, (1 << 21) + 5, 3_000_017])
def test_tree_hash_32b_elements(gpu, n):
    from oracle import oracle as O

    items = O.splitmix_bytes(n * 32, SEED + n % 1000)
    want = O.tree_hash_bytes_list(items, n, 32, nthreads=16)
    assert _dev_root(items, n, 32, gpu) == want
    if n in (1000, FUSED_MIN + 7):  # host-buffer entry point (the cgo TreeHash path)
        from prysm_amd import ssz

        assert ssz.tree_hash_bytes_list(items, n, 32) == want


@pytest.mark.parametrize("L", [0, 1, 4, 31, 33, 48, 96, 131, 132, 133, 200, 300])
@pytest.mark.parametrize("n", [1, 6, 9, 1001, FUSED_MIN + 3])
def test_tree_hash_other_lengths(gpu, L, n):
    """Element lengths other than 32 (pubkeys: 48; multi-block messages from
    132 bytes on) run the two-phase form, any alignment."""
    from oracle import oracle as O

    if n > 100_000 and L > 48:
        pytest.skip("large n checked at L <= 48")
    items = O.splitmix_bytes(n * L + 8, SEED + L)[:n * L]
    want = O.tree_hash_bytes_list(items, n, L, nthreads=16)
    assert _dev_root(items, n, L, gpu) == want
    assert _dev_root(items, n, L, gpu, offset=1) == want  # unaligned elements


def test_tree_hash_unaligned_32b_fused_size(gpu):
    """32-B elements at an odd address above the fused threshold: the
    two-phase form (the fused kernel needs 16-B aligned windows)."""
    from oracle import oracle as O

    n = FUSED_MIN + 11
    items = O.splitmix_bytes(n * 32, SEED + 5)
    want = O.tree_hash_bytes_list(items, n, 32, nthreads=16)
    for off in (4, 8, 3):
        import torch

        from prysm_amd import _lib
        from prysm_amd import device as D

        buf = torch.zeros(n * 32 + 64, dtype=torch.uint8, device=gpu)
        buf[off:off + n * 32] = torch.from_numpy(items.copy()).to(gpu)
        ws = torch.empty(n * 32 + _lib.load().mk_ssz_tree_hash_bytes_list_workspace_bytes(n, 32) + 512,
                         dtype=torch.uint8, device=gpu)
        out = D.tree_hash_bytes_list(buf[off:], n, 32, ws=ws)
        torch.cuda.synchronize()
        assert bytes(out.cpu().numpy()) == want, off
        # the default workspace covers the two-phase form's digest array
        out = D.tree_hash_bytes_list(buf[off:], n, 32)
        torch.cuda.synchronize()
        assert bytes(out.cpu().numpy()) == want, ("default ws", off)


def test_tree_hash_workspace_too_small(gpu):
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D

    n = 5000
    items = torch.zeros(n * 32, dtype=torch.uint8, device=gpu)
    ws = torch.empty(64, dtype=torch.uint8, device=gpu)
    with pytest.raises(_lib.MerkleError) as e:
        D.tree_hash_bytes_list(items, n, 32, ws=ws)
    assert e.value.code == _lib.MK_ENOMEM


def test_tree_hash_reflective_routes(gpu):
    """ssz.tree_hash(Slice(Bytes)) / Slice(ByteArray(32)) of one list goes
    through the one-call path and equals the reflective restatement."""
    from oracle import ssz_ref as OS
    from prysm_amd import ssz

    rng = np.random.default_rng(7)
    for n, L in ((1, 32), (5, 32), (37, 32), (300, 48), (77, 0), (9, 3)):
        vals = [bytes(rng.integers(0, 256, L, dtype=np.uint8)) for _ in range(n)]
        want = OS.tree_hash(("slice", ("bytes",)), vals)
        assert ssz.tree_hash(vals, ssz.Slice(ssz.Bytes())) == want, (n, L)
        if L:
            assert ssz.tree_hash(vals, ssz.Slice(ssz.ByteArray(L))) == want, (n, L)


# k_elem_lock (phase-locked element windows, n % 8 == 0 and n >= 2^23):
# 1024 groups; a partial last group + an odd window count; n not a multiple
# of 8 falls back to the fused form at the same size
@pytest.mark.parametrize("n", [1 << 23, (1 << 23) + 8 * (1024 * 37 + 5), (1 << 23) + 4])
def test_tree_hash_32b_locked_windows(gpu, n):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    items = torch.empty(n * 32, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 23)
    out = D.tree_hash_bytes_list(items, n, 32)
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()) == O.tree_hash_bytes_list(items.cpu().numpy(), n, 32, nthreads=16)


def test_tree_hash_2p28_golden(gpu):
    """The secondary C4 line's workload: TreeHash([][32]byte) of 2^28
    SplitMix64 elements (8 GiB generated on the device) vs the committed
    oracle root."""
    import torch

    from prysm_amd import device as D

    g = json.load(open(os.path.join(HERE, "golden", "full_size_roots.json")))["c4tree"]
    n, L = g["n"], g["elem_len"]
    items = torch.empty(n * L, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, g["seed"])
    out = D.tree_hash_bytes_list(items, n, L)
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()).hex() == g["root"]


@pytest.mark.parametrize("n,L", [((1 << 23) + 5, 32), (6_291_459, 48), ((1 << 21) + 1, 133)])
def test_tree_hash_host_overlap_path(gpu, n, L):
    """A host list of at least 2^28 bytes (the cgo TreeHash path) is hashed
    in shards on its one device: shard i+1's elements cross PCIe while shard
    i's digests and subtree are computed (multi_device_worker with elem_len)."""
    from oracle import oracle as O
    from prysm_amd import ssz

    assert n * L >= 1 << 28
    items = O.splitmix_bytes(n * L, SEED + L + 0x100)
    want = O.tree_hash_bytes_list(items, n, L, nthreads=16)
    assert ssz.tree_hash_bytes_list(items, n, L) == want
