"""GPU parity of the fused list tops (k_merkle_top_fused,
mk_dev_ssz_merkle_top_fused): one or two lists' trees from a
complete node level to the roots in one launch -- per-workgroup subtrees
over the chip, an agent-scope arrival counter, the last workgroup of each
list its top and the length mix-in, and with two lists the pair block of
mk_dev_ssz_merkle_finish_nodes_pair (the second list to finish hashes the
struct root).  Checked bit-exactly against the reference level loop
(hash.go:225-238, restated in _finish_ref) at counts that cover one
workgroup, ragged last workgroups (the odd rule at count 1 inside a part),
a last part of one node, the C3 shapes (125,000 registry / 31,250 balances
level-1 nodes) and 2^20; plus epochs, a workspace too small and a count past
2^20."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 0x91


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    _lib.init(0)
    return torch.device("cuda:0")


def _finish_ref(nodes: np.ndarray, n_total: int) -> bytes:
    """merkleHash's level loop over (count, 32) nodes and its length mix-in
    (hash.go:225-237: an odd level appends the 128-B zero chunk)."""
    from oracle import oracle as O

    cur = nodes
    while cur.shape[0] > 1:
        c = cur.shape[0]
        pairs = cur[: c - (c % 2)].reshape(-1)
        out = O.keccak256_batch(pairs, 64, nthreads=16) if c >= 2 else np.zeros((0, 32), np.uint8)
        if c % 2:
            last = np.frombuffer(O.keccak256(bytes(cur[-1]) + bytes(128)), dtype=np.uint8).reshape(1, 32)
            out = np.concatenate([out, last])
        cur = out
    return O.keccak256(bytes(cur[0]) + n_total.to_bytes(8, "little") + bytes(24))


def _nodes(gpu, c, seed):
    import torch

    from oracle import oracle as O

    host = O.splitmix_bytes(32 * c, seed).reshape(c, 32)
    return host, torch.from_numpy(host.copy()).to(gpu)


@pytest.mark.parametrize("c", [1, 2, 3, 1000, 1024, 1025, 1100, 5000, 4096 * 3 + 1, 125_000, 31_250, 1 << 20])
def test_top_fused_one_list(gpu, c):
    import torch

    from prysm_amd import device as D

    host, d = _nodes(gpu, c, SEED + c)
    n = 8 * c - 3
    out = torch.zeros(32, dtype=torch.uint8, device=gpu)
    D.merkle_top_fused(d, c, n, out)
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()) == _finish_ref(host, n)


@pytest.mark.parametrize("c0,c1", [(125_000, 31_250), (5000, 3), (1, 1), (1 << 20, 1 << 20), (70_001, 8751)])
def test_top_fused_pair(gpu, c0, c1):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    h0, d0 = _nodes(gpu, c0, SEED + 7 * c0)
    h1, d1 = _nodes(gpu, c1, SEED + 11 * c1 + 1)
    n0, n1 = c0 * 8, c1 * 32
    r0, r1 = _finish_ref(h0, n0), _finish_ref(h1, n1)
    pb = torch.zeros(128, dtype=torch.uint8, device=gpu)
    for epoch in (1, 2, 3):  # the same pair block, a new epoch per pair
        D.merkle_top_fused(d0, c0, n0, pb, d1, c1, n1, epoch=epoch)
        torch.cuda.synchronize()
        got = pb.cpu().numpy().tobytes()
        assert got[:32] == r0 and got[32:64] == r1
        assert got[64:96] == O.keccak256(r0 + r1), epoch


def test_top_fused_many_launches(gpu):
    """50 launches back to back on one stream, two inputs alternating, each
    into its own output (50 arrival slots, each reset by its last workgroup)."""
    import torch

    from prysm_amd import device as D

    c = 4096 * 5 + 13
    hs = [_nodes(gpu, c, SEED + 500 + k) for k in range(2)]
    wants = [_finish_ref(h, c) for h, _ in hs]
    outs = torch.zeros(50, 32, dtype=torch.uint8, device=gpu)
    ws = D.top_fused_workspace(c, 0, gpu)
    for k in range(50):
        D.merkle_top_fused(hs[k % 2][1], c, c, outs[k], ws=ws)
    torch.cuda.synchronize()
    got = outs.cpu().numpy()
    for k in range(50):
        assert bytes(got[k]) == wants[k % 2], k


def test_top_fused_errors(gpu):
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D

    L = _lib.load()
    assert L.mk_ssz_merkle_top_fused_workspace_bytes(0, 0) == 0
    assert L.mk_ssz_merkle_top_fused_workspace_bytes((1 << 20) + 1, 0) == 0
    _, d = _nodes(gpu, 5000, SEED)
    out = torch.zeros(128, dtype=torch.uint8, device=gpu)
    small = torch.empty(16, dtype=torch.uint8, device=gpu)
    with pytest.raises(Exception):
        D.merkle_top_fused(d, 5000, 5000, out, ws=small)
    with pytest.raises(Exception):  # a pair needs an epoch >= 1
        D.merkle_top_fused(d, 5000, 5000, out, d, 5000, 5000, epoch=0)
