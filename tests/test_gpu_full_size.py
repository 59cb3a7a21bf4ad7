"""Device path at the BASELINE.json full sizes against the CPU oracle's
results (tests/golden/full_size_roots.json, tests/golden/make_full_size.py):
the same seeded synthetic inputs bench.py measures, checked bit-exactly.

  c1  16,384-validator TreeHash (typed Hashable path, reflective mirror,
      device-resident records)
  c2  2^24 x 64-B Hash           (Keccak-256 of the 2^24 digests)
  c3  1,000,000-validator State  (registry root, balances root, state root)
  c4  2^28 x 32-B merkleHash     (8 GiB on the device), unsharded, as
      8 frontier shards finished on one device (one-piece and split per
      shard), and pipelined (bench.py's N=1 path)
  c5  2^20-deposit trie root
"""
import json
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "full_size_roots.json")))


@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.mark.gpu
def test_c4_full_2p28(gpu):
    import torch

    from prysm_amd import device as D
    from prysm_amd import parallel as P

    g = GOLD["c4"]
    n, il = g["n"], g["item_len"]
    items = torch.empty(n * il, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, g["seed"])
    root = D.merkle_hash(items, n, il)
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()).hex() == g["root"]
    # the 8-GPU decomposition on one device: frontier k=10 per shard, finisher
    world, k = 8, 10
    h, ne, begin = D.shard_plan(n, il, world)
    level = torch.empty(world << (k + 5), dtype=torch.uint8, device=gpu)
    ws = D.subtree_workspace(begin[1] - begin[0], il, gpu)
    for s in range(ne):
        sn = begin[s + 1] - begin[s]
        D.merkle_subtree_frontier(items[begin[s] * il:begin[s + 1] * il], sn, il, h, k, True,
                                  out=level[s << (k + 5):(s + 1) << (k + 5)], ws=ws)
    count = ((ne - 1) << k) + P.frontier_count(begin[ne] - begin[ne - 1], il, h, k)
    root2 = D.merkle_finish_nodes(level, count, n)
    torch.cuda.synchronize()
    assert bytes(root2.cpu().numpy()).hex() == g["root"]
    # the 8-GPU per-rank split of ShardedMerklePipeline on one device: every
    # shard's leaf pass (5 levels), then its node passes to the frontier
    for s in range(ne):
        sn = begin[s + 1] - begin[s]
        lvl = D.merkle_subtree_frontier(items[begin[s] * il:begin[s + 1] * il], sn, il, h, h - 5, True, ws=ws)
        D.merkle_node_frontier(lvl, lvl.numel() // 32, h - 5, k, True, out=level[s << (k + 5):(s + 1) << (k + 5)])
    root3 = D.merkle_finish_nodes(level, count, n)
    torch.cuda.synchronize()
    assert bytes(root3.cpu().numpy()).hex() == g["root"]
    # bench.py's N=1 path: pipelined back-to-back trees (top on a side stream)
    from prysm_amd.pipeline import MerklePipeline

    pipe = MerklePipeline(n, il, gpu)
    roots = [pipe.submit(items), pipe.submit(items)]
    torch.cuda.synchronize()
    assert pipe.k == 21 and [bytes(r.cpu().numpy()).hex() for r in roots] == [g["root"]] * 2
    del items


@pytest.mark.gpu
def test_c1_full_16384_validators(gpu):
    """BASELINE config 1 at its size: ssz.TreeHash([]*ValidatorRecord) of
    16,384 validators (shared/ssz/hash.go:118-159) through the typed Hashable
    path, the reflective mirror and the device-resident struct-list call."""
    import torch

    from prysm_amd import device as D
    from prysm_amd import registry as R
    from prysm_amd import ssz as S

    g = GOLD["c1"]
    reg = R.synthetic_registry(g["n"], g["seed"])
    assert reg.tree_hash_ssz().hex() == g["root"]
    assert S.tree_hash(reg, R.REGISTRY_HASHABLE).hex() == g["root"]
    assert S.tree_hash(reg.as_dicts(), S.Slice(S.Ptr(R.VALIDATOR_SSZ))).hex() == g["root"]
    drec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(gpu)
    root = D.struct_list_root(drec, g["n"], 160, R.VALIDATOR_FIELDS)
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()).hex() == g["root"]


@pytest.mark.gpu
def test_c2_full_2p24(gpu):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    g = GOLD["c2"]
    n, ln = g["n"], g["msg_len"]
    msgs = torch.empty(n * ln, dtype=torch.uint8, device=gpu)
    D.synth_fill(msgs, g["seed"])
    out = D.hash_batch(msgs, n, ln)
    torch.cuda.synchronize()
    assert O.keccak256(out.cpu().numpy().tobytes()).hex() == g["digest_of_digests"]


@pytest.mark.gpu
def test_c3_2p20_validators_device_generated(gpu):
    """SURVEY.md §8d's second C3 size, N = 2^20: the registry and balances
    generated in HBM (synthetic_registry_device: k_synth + the index rules),
    equal to the host generator, and the device-resident State root equal to
    the oracle's (C restatement, computed here on the host cores)."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd import registry as R

    n, seed = 1 << 20, GOLD["c3"]["seed"]
    reg = R.synthetic_registry(n, seed)
    bal = R.synthetic_balances(n, seed)
    drec = R.synthetic_registry_device(n, seed, gpu)
    dbal = R.synthetic_balances_device(n, seed, gpu)
    torch.cuda.synchronize()
    assert np.array_equal(drec.cpu().numpy(), reg.records.view(np.uint8).reshape(-1))
    assert np.array_equal(dbal.cpu().numpy(), bal.view(np.uint8))
    reg_root = D.struct_list_root(drec, n, 160, R.VALIDATOR_FIELDS)
    bal_root = D.merkle_hash(dbal, n, 8)
    torch.cuda.synchronize()
    roots = O.struct_roots(reg.records.view(np.uint8).reshape(-1), n, 160, R.VALIDATOR_FIELDS, nthreads=16)
    assert bytes(reg_root.cpu().numpy()) == O.merkle_hash_flat(roots.reshape(-1), n, 32, nthreads=16)
    assert bytes(bal_root.cpu().numpy()) == O.merkle_hash_flat(bal.view(np.uint8), n, 8, nthreads=16)


@pytest.mark.gpu
def test_c3_full_1m_validators(gpu):
    from prysm_amd import registry as R
    from prysm_amd import ssz as S

    g = GOLD["c3"]
    reg = R.synthetic_registry(g["n"], g["seed"])
    bal = R.synthetic_balances(g["n"], g["seed"])
    assert reg.tree_hash_ssz().hex() == g["registry_root"]
    assert S.merkle_hash_flat(bal.view(np.uint8), len(bal), 8).hex() == g["balances_root"]
    assert R.state_root(reg, bal).hex() == g["state_root"]
    # the device-resident two-stream schedule the C3 bench line times
    import torch

    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(gpu)
    dbal = torch.from_numpy(bal.view(np.uint8).copy()).to(gpu)
    hasher = R.DeviceStateHasher(g["n"], gpu)
    roots = [bytes(hasher.submit(rec, dbal).cpu().numpy()).hex() for _ in range(3)]
    assert roots == [g["state_root"]] * 3


@pytest.mark.gpu
def test_c5_full_2p20_deposits(gpu):
    import ctypes

    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D

    g = GOLD["c5"]
    n, dl, depth = g["n"], g["deposit_len"], g["depth"]
    data = torch.empty(n * dl, dtype=torch.uint8, device=gpu)
    D.synth_fill(data, g["seed"])
    L = _lib.load()
    lv = torch.empty(L.mk_deposit_trie_levels_bytes(n, depth), dtype=torch.uint8, device=gpu)
    root = torch.empty(32, dtype=torch.uint8, device=gpu)
    st = ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
    _lib.check(L.mk_dev_deposit_trie_append(None, ctypes.c_void_p(lv.data_ptr()), n, 0, ctypes.c_void_p(data.data_ptr()),
                                            None, n, dl, depth, ctypes.c_void_p(root.data_ptr()), st),
               "mk_dev_deposit_trie_append")
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()).hex() == g["root"]


@pytest.mark.gpu
def test_c5_full_2p20_pipelined_stream(gpu):
    """The C5 bench's stream form at full size: three 2^20-deposit tries
    through TriePipeline's pipelined front (each trie's levels 3-7 built in
    the next trie's lock-step slots, its top beside the front after that,
    the last one by flush); every root = the golden 2^20 root."""
    import torch

    from prysm_amd import device as D
    from prysm_amd.pipeline import TriePipeline

    g = GOLD["c5"]
    n, dl, depth = g["n"], g["deposit_len"], g["depth"]
    data = torch.empty(n * dl, dtype=torch.uint8, device=gpu)
    D.synth_fill(data, g["seed"])
    pipe = TriePipeline(n, dl, depth, gpu, front="pipe")
    roots = [pipe.submit(data) for _ in range(3)]
    torch.cuda.synchronize()
    got = [bytes(roots[0].cpu().numpy()).hex(), bytes(roots[1].cpu().numpy()).hex()]
    pipe.flush()
    torch.cuda.synchronize()
    got.append(bytes(roots[2].cpu().numpy()).hex())
    assert got == [g["root"]] * 3


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 8])
def test_c5_sharded_subtrees_on_one_device(gpu, world):
    """SURVEY §8e's C5 split at full size on one device: every shard's
    depth-h subtree (parallel.deposit_subtree_root), the gathered roots as
    level 0 of the trie above (parallel.deposit_trie_top) = the golden 2^20
    root; a ragged n (2^20 - 12345) against the one-piece device build."""
    import torch

    from prysm_amd import device as D
    from prysm_amd import parallel as P

    g = GOLD["c5"]
    n, dl, depth = g["n"], g["deposit_len"], g["depth"]
    data = torch.empty(n * dl, dtype=torch.uint8, device=gpu)
    D.synth_fill(data, g["seed"])
    for nn in (n, n - 12_345):
        tp = P.trie_plan(nn, world, depth)
        assert tp.height > 0 and tp.nonempty > 1
        roots = torch.zeros(32 * world, dtype=torch.uint8, device=gpu)
        for r in range(world):
            lo, hi = tp.items(r)
            if hi > lo:
                P.deposit_subtree_root(data[lo * dl:hi * dl], hi - lo, dl, tp.height, out=roots[32 * r:32 * r + 32])
        root = P.deposit_trie_top(roots, tp.nonempty, world, depth - tp.height)
        torch.cuda.synchronize()
        if nn == n:
            assert bytes(root.cpu().numpy()).hex() == g["root"]
        else:
            lv = torch.empty(D.deposit_trie_levels_bytes(nn, depth), dtype=torch.uint8, device=gpu)
            want = torch.empty(32, dtype=torch.uint8, device=gpu)
            D.deposit_trie_build(lv, nn, data, nn, dl, depth, depth, want)
            torch.cuda.synchronize()
            assert bytes(root.cpu().numpy()) == bytes(want.cpu().numpy())
