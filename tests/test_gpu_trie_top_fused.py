"""GPU parity of the fused trie top (k_trie_top_fused): a
whole trie built in one call (mk_dev_deposit_trie_build with d_to = depth)
takes every level from the first of <= 2^20 nodes to the root in one launch:
each workgroup reduces 1024 nodes by 10 levels, the last workgroup to arrive
(an agent-scope arrival counter) the rest, zero-sibling levels included.

EVERY level 0..depth the build writes (GenerateMerkleBranch reads them) and
the root are checked bit-exactly against the CPU restatement of
deposit_trie.go:29-40 (leaf = Keccak(deposit), node = Keccak(left ||
right-or-0^32)), at shapes that cover: one workgroup (the top alone), a
ragged last workgroup, a last workgroup holding a single node, the locked
front's level 2 as the start, a start level wider than 2^20 (one k_trie_level
first), shallow tries whose whole top fits one workgroup, and repeated builds
into one level buffer (the arrival slot reset by each launch's last
workgroup)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 0x7F
DL = 280


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    _lib.init(0)
    return torch.device("cuda:0")


def ref_levels(host: np.ndarray, n: int, depth: int):
    """Every level 0..depth of the batch build ((count, 32) uint8 arrays)."""
    from oracle import oracle as O

    lv = [O.keccak256_batch(host[:n * DL], DL, nthreads=16)]
    cur = lv[0]
    for _ in range(depth):
        if cur.shape[0] % 2:
            cur = np.concatenate([cur, np.zeros((1, 32), dtype=np.uint8)])
        cur = O.keccak256_batch(cur.reshape(-1), 64, nthreads=16)
        lv.append(cur)
    return lv


def device_levels(levels, cap: int, n: int, depth: int):
    host = levels.cpu().numpy()
    out, o = [], 0
    for d in range(depth + 1):
        c = -(-n // (1 << d))
        out.append(host[32 * o:32 * (o + c)].reshape(c, 32))
        o += -(-cap // (1 << d))
    return out


def build(gpu, n, depth, seed, cap=None, offset=0, lv=None):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    cap = cap or n
    host = O.splitmix_bytes(n * DL, seed)
    raw = torch.zeros(n * DL + 16, dtype=torch.uint8, device=gpu)
    raw[offset:offset + n * DL].copy_(torch.from_numpy(host))
    if lv is None:
        lv = torch.zeros(D.deposit_trie_levels_bytes(cap, depth), dtype=torch.uint8, device=gpu)
    root = torch.zeros(32, dtype=torch.uint8, device=gpu)
    D.deposit_trie_build(lv, cap, raw[offset:], n, DL, depth, depth, root)
    torch.cuda.synchronize()
    return host, lv, root


@pytest.mark.parametrize("n,depth,offset", [
    (1, 32, 0),                     # the zero-sibling tail alone
    (2, 32, 0),
    (7, 32, 8),                     # free-running leaves (8-B aligned), one workgroup
    (1000, 32, 0),                  # one ragged workgroup, then the tail
    (5000, 32, 8),                  # 5 workgroups, the last ragged (904 nodes)
    (1024 * 1024 + 5, 32, 8),       # level 0 wider than 2^20: one k_trie_level, then 513 workgroups
    ((1 << 18) + 3, 32, 0),         # locked front; level 2 = 65537 nodes: the last workgroup holds 1
    (1 << 20, 32, 0),               # C5: 256 workgroups
    (3 * (1 << 19) + 1, 32, 0),     # odd counts at every level
    (200, 8, 0),                    # shallow: the whole top in one workgroup, no hand-off
    (3000, 12, 8),                  # 3 workgroups to level 10, the top from there
    ((1 << 18) + 4096, 20, 0),      # locked front, depth 20
])
def test_fused_top_every_level(gpu, n, depth, offset):
    host, lv, root = build(gpu, n, depth, SEED + n % 1009 + depth, offset=offset)
    want = ref_levels(host, n, depth)
    got = device_levels(lv, n, n, depth)
    for d in range(depth + 1):
        assert np.array_equal(got[d], want[d]), f"n={n} depth={depth}: level {d}"
    assert bytes(root.cpu().numpy()) == bytes(want[depth][0])


def test_fused_top_capacity_layout(gpu):
    """Room for more deposits (capacity layout) and a second build into the
    same level buffer: both equal the restatement."""
    n, cap, depth = (1 << 18) + 77, 1 << 20, 32
    host, lv, root = build(gpu, n, depth, SEED + 5, cap=cap)
    want = ref_levels(host, n, depth)
    got = device_levels(lv, cap, n, depth)
    for d in range(depth + 1):
        assert np.array_equal(got[d], want[d]), f"level {d}"
    assert bytes(root.cpu().numpy()) == bytes(want[depth][0])
    host2, lv2, root2 = build(gpu, n, depth, SEED + 6, cap=cap, lv=lv)
    assert bytes(root2.cpu().numpy()) == bytes(ref_levels(host2, n, depth)[depth][0])


def test_fused_top_many_builds(gpu):
    """40 back-to-back builds on one stream (40 arrival slots, each reset by
    its launch's last workgroup), alternating two inputs: every root right."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n, depth = 4096 * 3 + 17, 32
    hosts = [O.splitmix_bytes(n * DL, SEED + 100 + k) for k in range(2)]
    wants = [bytes(ref_levels(h, n, depth)[depth][0]) for h in hosts]
    datas = [torch.from_numpy(h.copy()).to(gpu) for h in hosts]
    lv = torch.zeros(D.deposit_trie_levels_bytes(n, depth), dtype=torch.uint8, device=gpu)
    roots = torch.zeros(40, 32, dtype=torch.uint8, device=gpu)
    for k in range(40):
        D.deposit_trie_build(lv, n, datas[k % 2], n, DL, depth, depth, roots[k])
    torch.cuda.synchronize()
    got = roots.cpu().numpy()
    for k in range(40):
        assert bytes(got[k]) == wants[k % 2], k
