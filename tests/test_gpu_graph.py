"""The device-resident entry points enqueue kernels and device-to-device
copies only (include/prysm_merkle.h: "they never allocate and can be
captured into a hipGraph"): capture each into a HIP graph through
torch.cuda.graph, replay it, and check the replayed results against the
eager calls and the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 1300


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    assert _lib.device_count() >= 1
    return torch.device("cuda:0")


def _capture(fn):
    import torch

    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    return g


# (1 << 23) + 77: the phase-locked leaf pass (k_leaf_lock_sc) inside the graph
@pytest.mark.parametrize("n,item_len", [(1 << 20, 32), ((1 << 16) + 3, 32), (100_003, 8), (5, 32),
                                        ((1 << 23) + 77, 32)])
def test_graph_merkle_hash(gpu, n, item_len):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    items = torch.empty((n * item_len + 7) // 8 * 8, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + n)
    ws = D.merkle_workspace(n, item_len, gpu)
    out = torch.zeros(32, dtype=torch.uint8, device=gpu)
    g = _capture(lambda: D.merkle_hash(items, n, item_len, out=out, ws=ws))
    out.zero_()
    g.replay()
    torch.cuda.synchronize()
    want = O.merkle_hash_flat(items[:n * item_len].cpu().numpy(), n, item_len)
    assert bytes(out.cpu().numpy()) == want
    D.synth_fill(items, SEED + n + 1)  # a replay reads the buffers' current contents
    g.replay()
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()) == O.merkle_hash_flat(items[:n * item_len].cpu().numpy(), n, item_len)


def test_graph_hash_batch_and_struct_list_root(gpu):
    import torch

    from oracle import oracle as O
    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd import registry as R

    n = 4099
    msgs = torch.empty(n * 64, dtype=torch.uint8, device=gpu)
    D.synth_fill(msgs, SEED + 7)
    hout = torch.empty(n * 32, dtype=torch.uint8, device=gpu)
    reg = R.synthetic_registry(n, SEED + 8)
    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(gpu)
    f = R._fields(R.VALIDATOR_FIELDS)
    sws = torch.empty(_lib.load().mk_ssz_struct_list_workspace_bytes(n, f, len(R.VALIDATOR_FIELDS)) + 256,
                      dtype=torch.uint8, device=gpu)
    sout = torch.zeros(32, dtype=torch.uint8, device=gpu)

    def body():
        D.hash_batch(msgs, n, 64, out=hout)
        D.struct_list_root(rec, n, 160, R.VALIDATOR_FIELDS, out=sout, ws=sws)

    g = _capture(body)
    hout.zero_()
    g.replay()
    torch.cuda.synchronize()
    want = O.keccak256_batch(msgs.cpu().numpy(), 64)
    assert np.array_equal(hout.cpu().numpy().reshape(n, 32), want.reshape(n, 32))
    rr = O.struct_roots(reg.records.view(np.uint8).reshape(-1), n, 160, R.VALIDATOR_FIELDS)
    assert bytes(sout.cpu().numpy()) == O.merkle_hash_flat(rr.reshape(-1), n, 32)


def test_graph_deposit_trie_append(gpu):
    """A captured k = 1 append (leaf + right edge, one launch) replayed at a
    fixed count overwrites the same node: replaying it for deposit `count`
    equals the eager append; the batch build captures too."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    ln, depth, cap = 280, 32, 1 << 12
    n = 1000
    data = torch.empty(cap * ln, dtype=torch.uint8, device=gpu)
    D.synth_fill(data, SEED + 9)
    lv = torch.zeros(D.deposit_trie_levels_bytes(cap, depth), dtype=torch.uint8, device=gpu)
    root = torch.zeros(32, dtype=torch.uint8, device=gpu)
    g_build = _capture(lambda: D.deposit_trie_append(lv, cap, 0, data, n, ln, depth, root))
    g_build.replay()
    torch.cuda.synchronize()
    host = data.cpu().numpy()
    deps = [bytes(host[i * ln:(i + 1) * ln]) for i in range(n + 1)]
    assert bytes(root.cpu().numpy()) == O.deposit_trie_levels(deps[:n], depth)[0]
    g_one = _capture(lambda: D.deposit_trie_append(lv, cap, n, data[n * ln:], 1, ln, depth, root))
    root.zero_()
    g_one.replay()
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()) == O.deposit_trie_levels(deps, depth)[0]


def test_graph_capture_refused_by_merkle_many(gpu):
    """mk_dev_ssz_merkle_many plans its descriptors on the host and uploads
    them through a pinned ring on every call; a captured copy would replay a
    slot a later call overwrote, so a capturing stream gets MK_EINVAL (and the
    same call outside capture still works)."""
    import torch

    from oracle import oracle as O
    from prysm_amd import _lib
    from prysm_amd import device as D

    ns, ils = [300, 17, 1], [32, 8, 32]
    offs = [0, 300 * 32, 300 * 32 + 17 * 8 + 8]
    items = torch.empty(offs[-1] + 32, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 11)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    err = None
    with torch.cuda.graph(g):
        try:
            D.merkle_many(items, offs, ns, ils)
        except _lib.MerkleError as e:
            err = e
    assert err is not None and err.code == _lib.MK_EINVAL and "captured" in str(err)
    roots = D.merkle_many(items, offs, ns, ils)
    torch.cuda.synchronize()
    host = items.cpu().numpy()
    for i in range(3):
        want = O.merkle_hash_flat(host[offs[i]:offs[i] + ns[i] * ils[i]], ns[i], ils[i])
        assert bytes(roots[32 * i:32 * i + 32].cpu().numpy()) == want


def test_graph_hash_batch_locked(gpu):
    """2^18 + 5 64-B messages: k_keccak64_lock (a partial last group) captured
    and replayed over new contents."""
    import numpy as np
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n = (1 << 18) + 5
    msgs = torch.empty(n * 64, dtype=torch.uint8, device=gpu)
    D.synth_fill(msgs, SEED + 77)
    out = torch.zeros(n * 32, dtype=torch.uint8, device=gpu)
    g = _capture(lambda: D.hash_batch(msgs, n, 64, out=out))
    for seed in (SEED + 77, SEED + 78):
        D.synth_fill(msgs, seed)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        want = O.keccak256_batch(msgs.cpu().numpy(), 64, nthreads=16)
        assert np.array_equal(out.cpu().numpy().reshape(n, 32), want)
