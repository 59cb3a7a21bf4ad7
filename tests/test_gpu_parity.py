"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and the
reference's own vectors.  Bit-exact everywhere (integer/byte work)."""
import os
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    assert _lib.device_count() >= 1, "libprysm_merkle.so sees no gfx950 device"
    _lib.init(0)
    return torch.device("cuda:0")


# ------------------------------------------------------------------ Keccak
def test_hash_kats(gpu, ref_vectors):
    from prysm_amd import hashutil as H

    for kat in ref_vectors["keccak256_kats"]:
        assert H.Hash(bytes.fromhex(kat["in"])).hex() == kat["out"], kat["ref"]


@pytest.mark.parametrize("msg_len", [1, 8, 31, 32, 36, 52, 63, 64, 65, 135, 136, 137, 144, 200, 256, 271, 272,
                                     280, 1000])
def test_hash_batch_fixed(gpu, msg_len):
    from oracle import oracle as O
    from prysm_amd import hashutil as H

    n = 777
    msgs = O.splitmix_bytes(n * msg_len, SEED + msg_len)
    assert np.array_equal(H.hash_batch(msgs, msg_len), O.keccak256_batch(msgs, msg_len))


def test_dev_hash_batch_280_grid_stride(gpu):
    """280-B deposit messages take the grid-stride k_keccak_rec<35>: more
    records than the grid's threads (cap 4096 x 256), odd count, so threads
    hash 2-3 records and prefetch across record boundaries."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n, ln = 2 * 4096 * 256 + 12_345, 280
    msgs = torch.empty(n * ln, dtype=torch.uint8, device=gpu)
    D.synth_fill(msgs, SEED + 281)
    got = D.hash_batch(msgs, n, ln)
    torch.cuda.synchronize()
    want = O.keccak256_batch(msgs.cpu().numpy(), ln, nthreads=16)
    assert np.array_equal(got.cpu().numpy().reshape(n, 32), want)


def test_hash_batch_var(gpu):
    from oracle import oracle as O
    from prysm_amd import hashutil as H

    rng = np.random.default_rng(3)
    msgs = [bytes(rng.integers(0, 256, int(L), dtype=np.uint8)) for L in rng.integers(0, 700, 500)]
    msgs += [b"", b"\x00", b"abc"]
    got = H.hash_batch_var(msgs)
    want = [bytes(r) for r in O.keccak256_var(msgs)]
    assert got == want


def test_dev_hash_batch_64(gpu):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n = (1 << 16) + 5
    buf = torch.empty(n * 64, dtype=torch.uint8, device=gpu)
    D.synth_fill(buf, SEED + 11)
    out = D.hash_batch(buf, n, 64)
    torch.cuda.synchronize()
    host = buf.cpu().numpy()
    assert np.array_equal(host, O.splitmix_bytes(n * 64, SEED + 11))
    assert np.array_equal(out.cpu().numpy().reshape(n, 32), O.keccak256_batch(host, 64))


# ------------------------------------------------------------------ merkleHash
def test_merkle_reference_vectors(gpu, ref_vectors, res_vectors):
    from prysm_amd import ssz

    for vec in ref_vectors["merkle_hash"] + res_vectors["merkle_lists"]:
        items = [bytes.fromhex(x) for x in vec["items"]]
        assert ssz.merkle_hash(items).hex() == vec["output"], vec.get("ref")


def test_merkle_restatement_fixtures(gpu, res_vectors):
    from oracle import oracle as O
    from prysm_amd import ssz

    for c in res_vectors["merkle_flat"]:
        items = O.splitmix_bytes(c["n"] * c["item_len"], c["seed"])
        assert ssz.merkle_hash_flat(items, c["n"], c["item_len"]).hex() == c["root"], (c["n"], c["item_len"])


def test_merkle_edge_errors(gpu):
    from prysm_amd import ssz

    with pytest.raises(ZeroDivisionError):
        ssz.merkle_hash([b"", b"x"])
    with pytest.raises(ZeroDivisionError):
        ssz.merkle_hash_flat(np.zeros(0, np.uint8), 3, 0)


def test_merkle_ragged_list(gpu):
    from oracle import oracle as O
    from prysm_amd import ssz

    lst = [bytes([i]) * (1 + (i * 7) % 50) for i in range(37)]
    assert ssz.merkle_hash(lst) == O.merkle_hash(lst)


@pytest.mark.parametrize("n", [2048 * 4, 2048 * 4 + 4, 1 << 16, (1 << 16) + 3, (1 << 18) + 4 * 1024 + 1,
                               (1 << 20) - 1, 1 << 20, 3_000_001])
def test_dev_merkle_vs_oracle(gpu, n):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    item_len = 32
    items = torch.empty(n * item_len, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 21)
    root = D.merkle_hash(items, n, item_len)
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()) == O.merkle_hash_gen(n, item_len, SEED + 21, nthreads=16)


@pytest.mark.parametrize("item_len,n", [(8, 1 << 18), (8, 250_001), (1, 100_003), (48, 30_001), (128, 20_000),
                                        (200, 9_999), (3, 77_777)])
def test_dev_merkle_item_sizes(gpu, item_len, n):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    nb = n * item_len
    items = torch.empty(nb + (-nb) % 8, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 22)
    root = D.merkle_hash(items, n, item_len)
    torch.cuda.synchronize()
    host = items.cpu().numpy()[:nb]
    assert bytes(root.cpu().numpy()) == O.merkle_hash_flat(host, n, item_len, nthreads=16)


def test_dev_merkle_unaligned_input(gpu):
    """An input pointer that is not 16-B aligned takes the generic path."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n = 70_001
    buf = torch.empty(n * 32 + 64, dtype=torch.uint8, device=gpu)
    D.synth_fill(buf, SEED + 23)
    items = buf[8:8 + n * 32]
    root = D.merkle_hash(items, n, 32)
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()) == O.merkle_hash_flat(items.cpu().numpy(), n, 32, nthreads=16)


# ------------------------------------------------------------------ sharding
@pytest.mark.parametrize("n,world", [(1 << 16, 2), (1 << 16, 8), ((1 << 16) + 12, 8), (41 * 4 + 3, 4),
                                     (999_999, 3), (5, 8), (4099, 8), (1 << 20, 8)])
def test_subtree_sharding_equals_full(gpu, n, world):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    item_len = 32
    h, ne, begin = D.shard_plan(n, item_len, world)
    items = torch.empty(max(16, n * item_len), dtype=torch.uint8, device=gpu)
    D.synth_fill(items[:n * item_len], SEED + 31)
    full = D.merkle_hash(items, n, item_len)
    want = O.merkle_hash_gen(n, item_len, SEED + 31, nthreads=16)
    if ne > 1:
        roots = torch.zeros(world * 32, dtype=torch.uint8, device=gpu)
        for s in range(ne):
            sh = items[begin[s] * item_len:begin[s + 1] * item_len]
            D.merkle_subtree(sh, begin[s + 1] - begin[s], item_len, h, True, out=roots[32 * s:32 * s + 32])
        got = D.merkle_finish(roots, ne, n)
        torch.cuda.synchronize()
        for s in range(ne):  # every shard root against the oracle's subtree
            assert bytes(roots[32 * s:32 * s + 32].cpu().numpy()) == O.merkle_subtree_gen(
                n, item_len, SEED + 31, s, h, nthreads=16), s
        assert bytes(got.cpu().numpy()) == want
    torch.cuda.synchronize()
    assert bytes(full.cpu().numpy()) == want


@pytest.mark.parametrize("n,world,k", [(1 << 16, 8, 4), ((1 << 16) + 12, 8, 5), (999_999, 3, 8), (4099, 8, 3),
                                       (1 << 20, 8, 8), (1 << 22, 4, 10), (41 * 4 + 3, 4, 1)])
def test_frontier_sharding_equals_full(gpu, n, world, k):
    """Each shard's level k below its root equals the oracle's sub-shard
    roots; the concatenated frontiers finish to the full merkleHash root."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd import parallel as P

    item_len = 32
    h, ne, begin = D.shard_plan(n, item_len, world)
    assert ne > 1 and 0 < k < h
    items = torch.empty(n * item_len, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 33)
    level = torch.zeros(world << (k + 5), dtype=torch.uint8, device=gpu)
    counts = []
    for s in range(ne):
        sn = begin[s + 1] - begin[s]
        nodes = D.merkle_subtree_frontier(items[begin[s] * item_len:begin[s + 1] * item_len], sn, item_len, h, k,
                                          True, out=level[(s << (k + 5)):((s + 1) << (k + 5))])
        counts.append(nodes.numel() // 32)
    count = ((ne - 1) << k) + counts[-1]
    root = D.merkle_finish_nodes(level, count, n)
    torch.cuda.synchronize()
    got = level.cpu().numpy()
    for s in range(ne):
        for j in (0, counts[s] - 1):  # first and last node of every frontier
            want = O.merkle_subtree_gen(n, item_len, SEED + 33, (s << k) + j, h - k, nthreads=16)
            off = ((s << k) + j) * 32
            assert bytes(got[off:off + 32]) == want, (s, j)
    assert bytes(root.cpu().numpy()) == O.merkle_hash_gen(n, item_len, SEED + 33, nthreads=16)


@pytest.mark.parametrize("n,world,k,leaf", [(1 << 20, 8, 8, 5), ((1 << 20) + 12, 8, 5, 5), (999_999, 3, 8, 5),
                                            (41 * 4 + 3, 4, 1, 2), (1 << 22, 4, 10, 5), ((1 << 22) - 5, 4, 3, 4),
                                            (1 << 25, 8, 10, 5)])
def test_split_shard_frontier_equals_one_piece(gpu, n, world, k, leaf):
    """ShardedMerklePipeline's split of a shard: the leaf pass to `leaf`
    levels above the chunks, then mk_dev_ssz_merkle_node_frontier from that
    level to the 2^k frontier, equals the one-piece frontier of every shard
    (ragged last shards, lone nodes under pad_at_one)."""
    import torch

    from prysm_amd import device as D

    item_len = 32
    h, ne, begin = D.shard_plan(n, item_len, world)
    assert ne > 1 and 0 < k < h - leaf
    items = torch.empty(n * item_len, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 35)
    for s in range(ne):
        sn = begin[s + 1] - begin[s]
        it = items[begin[s] * item_len:begin[s + 1] * item_len]
        one = D.merkle_subtree_frontier(it, sn, item_len, h, k, True)
        lvl = D.merkle_subtree_frontier(it, sn, item_len, h, h - leaf, True)
        two = D.merkle_node_frontier(lvl, lvl.numel() // 32, h - leaf, k, True)
        torch.cuda.synchronize()
        assert torch.equal(one, two), (s, one.numel(), two.numel())
    # frontier 0: the node levels all the way to the shard root
    sn = begin[1] - begin[0]
    lvl = D.merkle_subtree_frontier(items[:sn * item_len], sn, item_len, h, h - leaf, True)
    top = D.merkle_node_frontier(lvl, lvl.numel() // 32, h - leaf, 0, True)
    root = D.merkle_subtree(items[:sn * item_len], sn, item_len, h, True)
    torch.cuda.synchronize()
    assert torch.equal(top, root)


@pytest.mark.parametrize("n,item_len,k", [(1 << 20, 32, 12), ((1 << 20) + 3, 32, 12), (3_000_017, 32, 16),
                                          (3_000_017, 32, 21), (100_003, 8, 8), (1000, 32, 21), (5, 32, 4),
                                          (777, 200, 3), (1 << 22, 32, None), ((1 << 22) + 9, 32, None)])
def test_pipeline_roots_equal_merkle_hash(gpu, n, item_len, k):
    """MerklePipeline (leaf side on the current stream, top on a side stream
    overlapping the next tree) over 5 consecutive trees of one shape: every
    root equals merkleHash of its own items (oracle), with the double-buffered
    frontier levels and roots reused across submits."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd.pipeline import MerklePipeline

    pipe = MerklePipeline(n, item_len, gpu, frontier_log2=k)
    trees = []
    for t in range(5):
        items = torch.empty(n * item_len, dtype=torch.uint8, device=gpu)
        D.synth_fill(items, SEED + 4000 + t)
        trees.append(items)
    roots = []
    for t, items in enumerate(trees):
        roots.append(pipe.submit(items))
        if t % 2 == 1 or t == len(trees) - 1:  # a root is valid until the submit after next
            torch.cuda.synchronize()
            roots = [r if isinstance(r, bytes) else bytes(r.cpu().numpy()) for r in roots]
    for t, items in enumerate(trees):
        want = O.merkle_hash_flat(items.cpu().numpy(), n, item_len)
        assert roots[t] == want, (t, pipe.k)


@pytest.mark.parametrize("count", [2, 3, 64, 65, 127, 1000, 2048, 2049, 5001])
def test_finish_nodes_vs_reference_loop(gpu, count):
    """The finisher over one gathered tree level: reference level loop with
    the 128-B odd pad, then the length mix-in (hash.go:225-237)."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    nodes = torch.empty(count * 32, dtype=torch.uint8, device=gpu)
    D.synth_fill(nodes, SEED + 34 + count)
    n_total = 123_456_789 + count
    got = D.merkle_finish_nodes(nodes, count, n_total)
    torch.cuda.synchronize()
    host = nodes.cpu().numpy()
    level = [bytes(host[32 * i:32 * i + 32]) for i in range(count)]
    while len(level) > 1:
        if len(level) % 2:
            level.append(bytes(128))
        level = [O.keccak256(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
    want = O.keccak256(level[0] + n_total.to_bytes(8, "little") + bytes(24))
    assert bytes(got.cpu().numpy()) == want


# ------------------------------------------------------------------ TreeHash host mirror
def test_tree_hash_reference_vectors(gpu, ref_vectors):
    from prysm_amd import ssz
    from tests.ssz_types import to_ssz_type, to_value

    assert len(ref_vectors["tree_hash"]) == 60
    for vec in ref_vectors["tree_hash"]:
        t = to_ssz_type(vec["type"])
        v = to_value(vec["type"], vec["value"])
        if vec["error"]:
            with pytest.raises(ssz.HashError) as ei:
                ssz.tree_hash(v, t)
            assert str(ei.value) == vec["error"], vec["ref"]
        else:
            assert ssz.tree_hash(v, t).hex() == vec["output"], vec["ref"]


def test_tree_hash_registry_matches_oracle(gpu):
    """A synthetic validator registry (pb.Validator field order, StatusFlags
    widened to uint64 — SURVEY.md §8d) through TreeHash vs the oracle."""
    from oracle import ssz_ref as S
    from prysm_amd import ssz
    from tests.ssz_types import validator_registry

    t_ref, t_ssz, vals = validator_registry(300, SEED + 51)
    assert ssz.tree_hash(vals, t_ssz) == S.tree_hash(t_ref, vals)


# ------------------------------------------------------------------ hashutil.MerkleRoot
@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 8, 13, 100, 8192])
def test_merkle_root(gpu, n):
    from oracle import oracle as O
    from prysm_amd import hashutil as H

    vals = [struct.pack("<Q", i) * (1 + i % 3) for i in range(n)]
    want = O.merkle_root(vals)
    mutated = list(vals)
    assert H.MerkleRoot(mutated) == want
    assert mutated == [O.keccak256(v) for v in vals]  # merkleRoot.go:16-19 side effect


@pytest.mark.parametrize("n,vlen", [(1, 32), (6, 64), (1000, 32), (1000, 64), (4097, 280), ((1 << 19) + 3, 32)])
def test_merkle_root_uniform(gpu, n, vlen):
    """Equal-length values take the fixed-length leaf kernels (64-B, word,
    byte); 2^19 + 3 values run a partial heap band plus k_reduce node passes."""
    from oracle import oracle as O
    from prysm_amd import hashutil as H

    raw = O.splitmix_bytes(n * vlen, SEED + 17 + vlen)
    vals = [bytes(raw[i * vlen:(i + 1) * vlen]) for i in range(n)]
    want = O.merkle_root(vals)
    mutated = list(vals)
    assert H.MerkleRoot(mutated) == want
    if n <= 1000:
        assert mutated == [O.keccak256(v) for v in vals]


def test_merkle_root_reference_vector(gpu, ref_vectors):
    from prysm_amd import hashutil as H

    for vec in ref_vectors["merkle_root"]:
        assert H.MerkleRoot([bytes.fromhex(v) for v in vec["values"]]).hex() == vec["output"]


# ------------------------------------------------------------------ deposit trie
def test_deposit_trie_fixtures(gpu, res_vectors):
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    for c in res_vectors["deposit_tries"]:
        deps = [bytes(O.splitmix_bytes(c["deposit_len"], c["seed"], c["word_stride"] * i)) for i in range(c["n"])]
        assert T.DepositTrie.build(deps).root().hex() == c["root"], c["n"]


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 8, 33, 1000, 4097])
def test_deposit_trie_levels_branches(gpu, n):
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    deps = [bytes(O.splitmix_bytes(280, SEED + 61, 35 * i)) for i in range(n)]
    root, levels = O.deposit_trie_levels(deps)
    t = T.DepositTrie()
    for d in deps:
        t.update_deposit_trie(d)
    assert t.root() == root
    for i in sorted({0, n // 2, max(n - 1, 0)}) if n else []:
        br = t.generate_merkle_branch(i)
        want = [levels[d][(i >> d) ^ 1] if ((i >> d) ^ 1) < len(levels[d]) else bytes(32) for d in range(32)]
        assert br == want
        assert T.verify_merkle_branch(O.keccak256(deps[i]), br, 32, i, root)
        assert not T.verify_merkle_branch(O.keccak256(deps[i] + b"!"), br, 32, i, root)


def test_deposit_trie_reference_shapes(gpu):
    """deposit_trie_test.go:10-65 shapes: 2 x 4-byte deposits, 3 x 3-byte."""
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    for deps in ([bytes([1, 2, 3, 4]), bytes([5, 6, 7, 8])], [bytes(4), bytes(4)],
                 [bytes([1, 2, 3]), bytes([5, 6, 7]), bytes([8, 9, 10])]):
        t = T.DepositTrie()
        for d in deps:
            t.UpdateDepositTrie(d)
        assert t.deposit_count == len(deps)
        assert t.leaf(len(deps) - 1) == O.keccak256(deps[-1])
        idx = len(deps) - 1
        assert T.VerifyMerkleBranch(O.keccak256(deps[-1]), t.GenerateMerkleBranch(idx), 32, idx, t.Root())
        assert t.Root() == O.deposit_trie_levels(deps)[0]


def test_verify_branches_batch(gpu):
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    n = 2000
    deps = [bytes(O.splitmix_bytes(280, SEED + 71, 35 * i)) for i in range(n)]
    t = T.DepositTrie.build(deps)
    idx = list(range(0, n, 7))
    leaves = [O.keccak256(deps[i]) for i in idx]
    branches = [t.generate_merkle_branch(i) for i in idx]
    roots = [t.root()] * len(idx)
    assert all(T.verify_merkle_branches(leaves, branches, 32, idx, roots))
    bad = list(idx)
    bad[3] += 1
    res = T.verify_merkle_branches(leaves, branches, 32, bad, roots)
    assert res[3] is False and sum(res) == len(idx) - 1


# ------------------------------------------------------------------ typed registry (Hashable plugin)
@pytest.mark.parametrize("n", [1, 2, 5, 300, 4099, 16_384, 70_001])
def test_registry_struct_roots_and_list_root(gpu, n):
    from oracle import oracle as O
    from prysm_amd import registry as R

    reg = R.synthetic_registry(n, SEED + 91)
    raw = reg.records.view(np.uint8).reshape(-1)
    spec = [(k, o, l) for k, o, l in R.VALIDATOR_FIELDS]
    want_roots = O.struct_roots(raw, n, 160, spec, nthreads=16)
    assert np.array_equal(R.struct_roots(reg.records), want_roots)
    assert reg.tree_hash_ssz() == O.merkle_hash_flat(want_roots.reshape(-1), n, 32, nthreads=16)


def test_registry_equals_reflective_tree_hash(gpu):
    """The Hashable fast path equals the reference's reflective TreeHash of
    []*ValidatorRecord (oracle restatement and the host mirror)."""
    from oracle import ssz_ref as OS
    from prysm_amd import registry as R
    from prysm_amd import ssz

    reg = R.synthetic_registry(333, SEED + 92)
    dicts = reg.as_dicts()
    t_ref = ("slice", ("ptr", ("struct", "ssz.ValidatorRecord",
                               [("Pubkey", ("bytes",)), ("WithdrawalCredentialsHash32", ("bytes",)),
                                ("RandaoCommitmentHash32", ("bytes",))] +
                               [(f, ("uint", 64)) for f in ("RandaoLayers", "ActivationEpoch", "ExitEpoch",
                                                            "WithdrawalEpoch", "PenalizedEpoch", "StatusFlags")])))
    want = OS.tree_hash(t_ref, dicts)
    assert ssz.tree_hash(reg, R.REGISTRY_HASHABLE) == want
    assert ssz.tree_hash(dicts, ssz.Slice(ssz.Ptr(R.VALIDATOR_SSZ))) == want


def test_state_root(gpu):
    from oracle import oracle as O
    from prysm_amd import registry as R

    n = 10_000
    reg = R.synthetic_registry(n, SEED + 93)
    bal = R.synthetic_balances(n, SEED + 93)
    spec = [(k, o, l) for k, o, l in R.VALIDATOR_FIELDS]
    roots = O.struct_roots(reg.records.view(np.uint8).reshape(-1), n, 160, spec, nthreads=16)
    want = O.keccak256(O.merkle_hash_flat(roots.reshape(-1), n, 32) +
                       O.merkle_hash_flat(bal.view(np.uint8), n, 8))
    assert R.state_root(reg, bal) == want


# Struct layouts that take the fused one-kernel path (dword-granular fields,
# with and without 16-B loads, one- and two-block messages) and the two-kernel
# fallback (2-byte scalar, >160-B message, non-dword bytes field).
_STRUCT_LAYOUTS = {
    "fused_dword_loads": (100, [(1, 4, 36), (2, 40, 8), (1, 48, 20), (2, 68, 4), (2, 72, 8)]),
    "fused_vec16_two_blocks": (208, [(1, 0, 16), (1, 16, 32), (1, 48, 48), (1, 96, 64), (1, 160, 48)]),
    "fused_tail_field": (96, [(2, 0, 8), (1, 8, 4), (1, 16, 80)]),
    "fallback_u16": (52, [(1, 0, 32), (2, 32, 2), (2, 36, 8)]),
    "fallback_long_msg": (192, [(1, 32 * k, 32) for k in range(6)]),
    "fallback_odd_bytes": (48, [(1, 0, 33), (2, 36, 4)]),
}


@pytest.mark.parametrize("layout", sorted(_STRUCT_LAYOUTS))
@pytest.mark.parametrize("n", [1, 257, 3000])
def test_struct_roots_layouts(gpu, layout, n):
    from oracle import oracle as O
    from prysm_amd import registry as R

    rec_len, spec = _STRUCT_LAYOUTS[layout]
    raw = O.splitmix_bytes(n * rec_len, SEED + 97 + rec_len)
    recs = raw.view(np.dtype((np.void, rec_len)))
    want = O.struct_roots(raw, n, rec_len, spec, nthreads=8)
    assert np.array_equal(R.struct_roots(recs, spec), want)


@pytest.mark.parametrize("layout", sorted(_STRUCT_LAYOUTS) + ["validator"])
@pytest.mark.parametrize("n", [1, 257, 70_001])
def test_dev_struct_roots(gpu, layout, n):
    """mk_dev_ssz_struct_roots (device records, caller's stream) vs oracle."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd import registry as R

    rec_len, spec = (160, list(R.VALIDATOR_FIELDS)) if layout == "validator" else _STRUCT_LAYOUTS[layout]
    raw = O.splitmix_bytes(n * rec_len, SEED + 98 + rec_len)
    want = O.struct_roots(raw, n, rec_len, spec, nthreads=8)
    got = D.struct_roots(torch.from_numpy(raw.copy()).to("cuda:0"), n, rec_len, spec)
    torch.cuda.synchronize()
    assert np.array_equal(got.cpu().numpy().reshape(n, 32), want.reshape(n, 32))


@pytest.mark.parametrize("n", [1 << 25, (1 << 25) + 12_345, (1 << 24) + 7 * 4096])
def test_merkle_hash_shard_sized_leaf_pass(gpu, n):
    """The per-rank shard sizes of a multi-GPU tree (2^24..2^25 items): the
    phase-locked leaf pass (k_leaf_lock_sc, 4 spans per workgroup) plus the
    k_reduce spans after the last whole group.  Unsharded and as an 8-shard
    frontier level.  (Round 3's half-span tail of the free-running leaf pass
    could not run beside the locked pass and was removed in round 4.)"""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    seed = SEED + 2025
    items = torch.empty(n * 32, dtype=torch.uint8, device="cuda:0")
    D.synth_fill(items, seed)
    root = D.merkle_hash(items, n, 32)
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()) == O.merkle_hash_gen(n, 32, seed, nthreads=16)
