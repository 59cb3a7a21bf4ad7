"""GPU parity of the phase-locked deposit-trie front (k_trie_rec_lock: the
leaf hashes of 280-B deposits plus trie levels 1..log2(DPT) in one launch,
DESIGN.md §5 "Locked trie front"), at the shapes where it hands over to the
free-running kernels: whole groups run locked, a persistent workgroup may
take several groups, and the rest (a partial group, an odd deposit count)
runs k_keccak_rec + k_trie_level on the suffix of each level.

Every level the front writes (0..4) and the root are checked bit-exactly
against a CPU restatement of deposit_trie.go:29-40 (leaf = Keccak(deposit),
node = Keccak(left || right-or-0^32)): the C oracle's batched Keccak composed
level by level, itself checked against the dict restatement of the
reference's per-deposit loop in tests/test_oracle.py."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 0x70
DEPTH = 32
DL = 280


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    _lib.init(0)
    return torch.device("cuda:0")


def ref_levels(host: np.ndarray, n: int, upto: int):
    """Levels 0..upto of the batch build (lists of (count, 32) uint8 arrays)
    and the depth-32 root."""
    from oracle import oracle as O

    lv = [O.keccak256_batch(host[:n * DL], DL, nthreads=16)]
    cur = lv[0]
    for _ in range(DEPTH):
        c = cur.shape[0]
        if c % 2:
            cur = np.concatenate([cur, np.zeros((1, 32), dtype=np.uint8)])
        cur = O.keccak256_batch(cur.reshape(-1), 64, nthreads=16)
        if len(lv) <= upto:
            lv.append(cur)
    return lv, bytes(cur[0])


def level_off(cap: int, d: int) -> int:
    return sum(-(-cap // (1 << i)) for i in range(d))


def device_levels(levels, cap: int, n: int, upto: int):
    host = levels.cpu().numpy()
    out = []
    for d in range(upto + 1):
        c = -(-n // (1 << d))
        o = level_off(cap, d)
        out.append(host[32 * o:32 * (o + c)].reshape(c, 32))
    return out


@pytest.mark.parametrize("n", [
    1 << 18,                      # 64 whole groups of 4096, nothing after
    (1 << 18) + 3,                # + 3 deposits: a partial group, odd count at every level
    1 << 20,                      # C5: 256 groups, one per workgroup
    (1 << 21) + 4096 * 5 + 1234,  # 517 groups over 259 persistent workgroups (uneven) + the rest
    3 * (1 << 19) + 1,            # odd n, every level's last node is padded
])
def test_trie_front_levels_vs_restatement(gpu, n):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    host = O.splitmix_bytes(n * DL, SEED + n % 977)
    data = torch.from_numpy(host.copy()).to(gpu)
    lv = torch.zeros(D.deposit_trie_levels_bytes(n, DEPTH), dtype=torch.uint8, device=gpu)
    root = torch.zeros(32, dtype=torch.uint8, device=gpu)
    D.deposit_trie_build(lv, n, data, n, DL, DEPTH, DEPTH, root)
    torch.cuda.synchronize()
    want, want_root = ref_levels(host, n, 4)
    got = device_levels(lv, n, n, 4)
    for d in range(5):
        assert np.array_equal(got[d], want[d]), f"level {d}"
    assert bytes(root.cpu().numpy()) == want_root


@pytest.mark.parametrize("d_to", [2, 3])
def test_trie_front_split_levels(gpu, d_to):
    """The stream-of-tries split (pipeline.TriePipeline): the front to d_to on
    one call, the rest of the levels on another; levels and root as one build."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n = (1 << 19) + 4096 + 17
    host = O.splitmix_bytes(n * DL, SEED + 1)
    data = torch.from_numpy(host.copy()).to(gpu)
    lv = torch.zeros(D.deposit_trie_levels_bytes(n, DEPTH), dtype=torch.uint8, device=gpu)
    root = torch.zeros(32, dtype=torch.uint8, device=gpu)
    D.deposit_trie_build(lv, n, data, n, DL, d_to, DEPTH)
    D.deposit_trie_levels(lv, n, n, d_to, DEPTH, DEPTH, root)
    torch.cuda.synchronize()
    want, want_root = ref_levels(host, n, 3)
    got = device_levels(lv, n, n, 3)
    for d in range(4):
        assert np.array_equal(got[d], want[d]), f"level {d}"
    assert bytes(root.cpu().numpy()) == want_root


def test_trie_front_capacity_layout_and_unaligned(gpu):
    """A trie with room for more deposits (capacity layout: level d at
    sum_{i<d} ceil(cap / 2^i)) and deposits at an 8-B aligned (not 16-B)
    address, which takes the free-running kernels: both equal the oracle."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n, cap = (1 << 18) + 77, 1 << 20
    host = O.splitmix_bytes(n * DL, SEED + 2)
    want, want_root = ref_levels(host, n, 3)
    raw = torch.zeros(n * DL + 16, dtype=torch.uint8, device=gpu)
    for off in (0, 8):
        raw[off:off + n * DL].copy_(torch.from_numpy(host))
        lv = torch.zeros(D.deposit_trie_levels_bytes(cap, DEPTH), dtype=torch.uint8, device=gpu)
        root = torch.zeros(32, dtype=torch.uint8, device=gpu)
        D.deposit_trie_build(lv, cap, raw[off:], n, DL, DEPTH, DEPTH, root)
        torch.cuda.synchronize()
        got = device_levels(lv, cap, n, 3)
        for d in range(4):
            assert np.array_equal(got[d], want[d]), (off, d)
        assert bytes(root.cpu().numpy()) == want_root, off


def test_trie_pipeline_stream_vs_oracle(gpu):
    """Three tries through pipeline.TriePipeline (the C5 bench's stream): each
    root equals the restatement."""
    import torch

    from oracle import oracle as O
    from prysm_amd.pipeline import TriePipeline

    n = (1 << 20) + 5
    pipe = TriePipeline(n, DL, DEPTH, gpu)
    roots = []
    for t in range(3):
        host = O.splitmix_bytes(n * DL, SEED + 10 + t)
        data = torch.from_numpy(host).to(gpu)
        r = pipe.submit(data)
        torch.cuda.synchronize()
        roots.append((bytes(r.cpu().numpy()), ref_levels(host, n, 0)[1]))
    for got, want in roots:
        assert got == want
