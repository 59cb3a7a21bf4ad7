"""Pins the CPU oracle against the reference's own vectors (CPU only).

The oracle is the checker for every GPU parity test, so it is pinned first:
Keccak KATs (hashutil/hash_test.go:13-31), the permutation against FIPS
SHA3-256 (hashlib), every ssz/hash_test.go vector, the merkleHash table and
the example structs; the deposit-trie batch build against a literal
dict-based restatement of UpdateDepositTrie (deposit_trie.go:29-40).
"""
import hashlib
import json
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O
from oracle import ssz_ref as S


def test_keccak_kats(ref_vectors):
    for kat in ref_vectors["keccak256_kats"]:
        assert O.keccak256(bytes.fromhex(kat["in"])).hex() == kat["out"], kat["ref"]
        assert O.py_keccak256(bytes.fromhex(kat["in"])).hex() == kat["out"], kat["ref"]


@pytest.mark.parametrize("n", [0, 1, 7, 64, 135, 136, 137, 200, 271, 272, 273, 1000])
def test_permutation_vs_fips_sha3(n):
    msg = os.urandom(n)
    assert O.sha3_256(msg) == hashlib.sha3_256(msg).digest()
    assert O.py_keccak256(msg, pad=0x06) == hashlib.sha3_256(msg).digest()
    assert O.py_keccak256(msg) == O.keccak256(msg)


def test_unrolled_permutation_equals_loop_form():
    """The CPU baseline's permutation (keccak_fast.c, the x/crypto shape)
    is the same function as the restatement's loop form: random states,
    every sponge through it (KATs, FIPS SHA3-256) and a merkleHash."""
    rng = np.random.default_rng(5)
    for _ in range(256):
        s = rng.integers(0, 2**63, 25, dtype=np.uint64) * np.uint64(3)
        assert np.array_equal(O.keccak_f(s), O.keccak_f(s, unrolled=True))
    items = O.splitmix_bytes(1000 * 32, 11)
    want = O.merkle_hash_flat(items, 1000, 32)
    kats = [(bytes.fromhex(k["in"]), k["out"]) for k in
            json.load(open(os.path.join(os.path.dirname(__file__), "golden",
                                        "reference_vectors.json")))["keccak256_kats"]]
    with O.fast_permutation():
        for n in (0, 1, 135, 136, 137, 500):
            msg = bytes(rng.integers(0, 256, n, dtype=np.uint8))
            assert O.sha3_256(msg) == hashlib.sha3_256(msg).digest()
        for m, out in kats:
            assert O.keccak256(m).hex() == out
        assert O.merkle_hash_flat(items, 1000, 32) == want
    assert O.lib().or_set_fast_permutation(0) == 0  # restored on exit


def _pyval(t, v):
    """Convert JSON fixture values into what ssz_ref expects."""
    k = t[0]
    if k in ("slice", "array"):
        return [_pyval(t[1], e) for e in v]
    if k == "struct":
        return {name: _pyval(ft, v[name]) for name, ft in t[2]} if v is not None else None
    if k == "ptr":
        return None if v is None else _pyval(t[1], v)
    return v


def _pytype(t):
    k = t[0]
    if k == "hashable":
        # hash_test.go:25-32: 28 zero bytes followed by the 4-byte value
        return ("hashable", t[1], lambda v: (bytes(28) + bytes(v))[:32])
    if k in ("slice", "ptr"):
        return (k, _pytype(t[1]))
    if k == "array":
        return (k, _pytype(t[1]), t[2])
    if k == "struct":
        return (k, t[1], [(n, _pytype(ft)) for n, ft in t[2]])
    return tuple(t)


def test_tree_hash_vectors(ref_vectors):
    assert len(ref_vectors["tree_hash"]) == 60
    for vec in ref_vectors["tree_hash"]:
        t = _pytype(vec["type"])
        if vec["error"]:
            with pytest.raises(S.HashError) as ei:
                S.tree_hash(t, _pyval(vec["type"], vec["value"]))
            assert str(ei.value) == vec["error"], vec["ref"]
        else:
            got = S.tree_hash(t, _pyval(vec["type"], vec["value"]))
            assert got.hex() == vec["output"], vec["ref"]


def test_merkle_hash_vectors(ref_vectors, res_vectors):
    for vec in ref_vectors["merkle_hash"] + res_vectors["merkle_lists"]:
        items = [bytes.fromhex(x) for x in vec["items"]]
        assert O.merkle_hash(items).hex() == vec["output"]


def test_merkle_root_vector(ref_vectors):
    for vec in ref_vectors["merkle_root"]:
        assert O.merkle_root([bytes.fromhex(v) for v in vec["values"]]).hex() == vec["output"]


def test_flat_equals_list_semantics():
    rng = np.random.default_rng(1)
    for item_len in (1, 3, 8, 32, 48, 128, 200):
        for n in (0, 1, 2, 4, 5, 9, 17, 40):
            items = rng.integers(0, 256, n * item_len, dtype=np.uint8)
            lst = [bytes(items[i * item_len:(i + 1) * item_len]) for i in range(n)]
            assert O.merkle_hash_flat(items, n, item_len) == O.merkle_hash(lst)


def _py_merkle_hash(lst):
    """Literal list restatement of hash.go:194-239 with the pure-Python digest."""
    lenc = struct.pack("<Q", len(lst)) + bytes(24)
    empty = bytes(128)
    if not lst:
        chunks = [empty]
    elif len(lst[0]) < 128:
        p = 128 // len(lst[0])
        chunks = [b"".join(lst[i:i + p]) for i in range(0, len(lst), p)]
    else:
        chunks = list(lst)
    while len(chunks) > 1:
        if len(chunks) % 2:
            chunks.append(empty)
        chunks = [O.py_keccak256(chunks[i] + chunks[i + 1]) for i in range(0, len(chunks), 2)]
    return O.py_keccak256(chunks[0] + lenc)


def test_c_oracle_equals_pure_python_restatement():
    rng = np.random.default_rng(7)
    for item_len, n in ((32, 9), (32, 13), (8, 40), (3, 50), (200, 5), (1, 300)):
        lst = [bytes(rng.integers(0, 256, item_len, dtype=np.uint8)) for _ in range(n)]
        assert O.merkle_hash(lst) == _py_merkle_hash(lst)


_DictTrie = O.DictTrie


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 8, 13])
def test_deposit_trie_batch_equals_incremental(n):
    deps = [os.urandom(1 + (i * 37) % 300) for i in range(n)]
    t = _DictTrie()
    for d in deps:
        t.update(d)
    root, levels = O.deposit_trie_levels(deps)
    assert root == t.root()
    for i in range(n):
        br = [levels[d][(i >> d) ^ 1] if ((i >> d) ^ 1) < len(levels[d]) else bytes(32) for d in range(32)]
        assert br == t.branch(i)
        assert O.verify_merkle_branch(O.keccak256(deps[i]), br, 32, i, root)
        assert not O.verify_merkle_branch(O.keccak256(deps[i] + b"x"), br, 32, i, root)


@pytest.mark.parametrize("n", [0, 1, 2, 3, 7, 100, 1025])
def test_incremental_c_restatement_equals_dict_and_batch(n):
    """or_deposit_trie_incremental (the reference's per-deposit algorithm in C,
    the C5 CPU baseline) against the dict restatement and the batch build."""
    deps = [bytes([i % 251]) * (1 + (i * 37) % 300) for i in range(n)]
    t = _DictTrie()
    for d in deps:
        t.update(d)
    assert O.deposit_trie_incremental_root(deps) == t.root() == O.deposit_trie_levels(deps)[0]


@pytest.mark.parametrize("n", [0, 1, 2, 3, 6, 33])
def test_deposit_contract_equals_trieutil(n):
    """The reference keeps config 5's tree twice: trieutil.DepositTrie
    (deposit_trie.go:29-63) and the Vyper deposit contract
    (depositContract.v.py:36-71).  The contract restatement's roots, branches
    and per-deposit events against the dict restatement and the batch build
    over the contract's own deposit-data layout (8-B big-endian amount and
    timestamp, then the 264-B DepositInput of C5)."""
    rng = np.random.default_rng(11 + n)
    c, t = O.DepositContract(), _DictTrie()
    datas = []
    for i in range(n):
        amount = 32 * 10**9 - int(rng.integers(0, 1000))
        ts = 1_540_000_000 + i
        ev = c.deposit(amount, ts, bytes(rng.integers(0, 256, 264, dtype=np.uint8)))
        assert ev[0] == t.root()  # previous_deposit_root: the root before this deposit
        assert ev[2] == (i + (1 << 32)).to_bytes(8, "big")
        assert ev[1][:8] == amount.to_bytes(8, "big") and ev[1][8:16] == ts.to_bytes(8, "big")
        assert len(ev[1]) == 280
        t.update(ev[1])
        datas.append(ev[1])
        assert c.get_deposit_root() == t.root()
    root, levels = O.deposit_trie_levels(datas)
    assert c.get_deposit_root() == root == (t.root() if n else bytes(32))
    for i in range(n):
        assert c.get_branch(i) == t.branch(i)
        assert O.verify_merkle_branch(O.keccak256(datas[i]), c.get_branch(i), 32, i, root)


def test_restatement_fixtures_reproduce(res_vectors):
    for c in res_vectors["merkle_flat"][::17]:
        items = O.splitmix_bytes(c["n"] * c["item_len"], c["seed"])
        assert O.merkle_hash_flat(items, c["n"], c["item_len"]).hex() == c["root"]
    sm = res_vectors["splitmix"]
    assert [O.lib().or_splitmix64_word(sm["seed"], k) for k in range(8)] == sm["words"]


def test_generator_and_subtree_oracles_agree():
    seed = 0x5EED000000000004
    for n, item_len in ((4 * 64, 32), (4 * 64 + 12, 32), (1000, 8), (333, 32)):
        items = O.splitmix_bytes(n * item_len, seed)
        full = O.merkle_hash_flat(items, n, item_len)
        assert O.merkle_hash_gen(n, item_len, seed) == full
    # shard roots folded with the reference loop give the same root
    n, item_len, H = 4 * 40 + 3, 32, 3  # 41 chunks, shards of 8 chunks -> 6 shards
    roots = [O.merkle_subtree_gen(n, item_len, seed, s, H) for s in range(6)]
    chunks = roots
    while len(chunks) > 1:
        if len(chunks) % 2:
            chunks = chunks + [bytes(128)]
        chunks = [O.keccak256(chunks[i] + chunks[i + 1]) for i in range(0, len(chunks), 2)]
    final = O.keccak256(chunks[0] + struct.pack("<Q", n) + bytes(24))
    assert final == O.merkle_hash_gen(n, item_len, seed)


def test_tree_hash_bytes_list_oracle_routes():
    """The composed oracle for TreeHash of a byte-string list (hashedEncoding
    digests + merkleHash) equals the reflective restatement, and chunked
    digest generation (make_full_size.py c4tree) equals one pass."""
    import numpy as np

    from oracle import oracle as O
    from oracle import ssz_ref as OS

    rng = np.random.default_rng(3)
    for n, L in ((0, 32), (1, 32), (4, 32), (5, 32), (8, 32), (9, 32), (130, 32), (17, 48), (40, 0), (6, 140)):
        vals = [bytes(rng.integers(0, 256, L, dtype=np.uint8)) for _ in range(n)]
        flat = np.frombuffer(b"".join(vals), dtype=np.uint8) if n * L else np.zeros(0, np.uint8)
        assert O.tree_hash_bytes_list(flat, n, L) == OS.tree_hash(("slice", ("bytes",)), vals), (n, L)
    items = O.splitmix_bytes(5000 * 32, 11)
    one = O.elem_digests(items, 5000, 32)
    parts = np.concatenate([O.elem_digests(O.splitmix_bytes(1000 * 32, 11, word0=lo * 4), 1000, 32)
                            for lo in range(0, 5000, 1000)])
    assert np.array_equal(one, parts)
    assert np.array_equal(O.elem_digests(items, 5000, 32, chunk=777), one)


@pytest.mark.parametrize("count", [1, 2, 3, 5, 8, 13, 64, 1001])
def test_merkle_nodes_oracle(count):
    """or_merkle_nodes (a level of 32-B nodes to the root, the device
    finisher's semantics) against the literal loop of hash.go:225-237 with
    the pure-Python digest, and, from a flat tree's level-1 nodes, against
    the whole flat tree's root."""
    rng = np.random.default_rng(100 + count)
    nodes = rng.integers(0, 256, 32 * count, dtype=np.uint8)
    n_total = int(rng.integers(1, 1 << 40))
    chunks = [bytes(nodes[32 * i:32 * i + 32]) for i in range(count)]
    while len(chunks) > 1:
        if len(chunks) % 2:
            chunks.append(bytes(128))
        chunks = [O.keccak256(chunks[i] + chunks[i + 1]) for i in range(0, len(chunks), 2)]
    want = O.py_keccak256(chunks[0] + struct.pack("<Q", n_total) + bytes(24))
    assert O.merkle_nodes(nodes, count, n_total) == want
    assert O.merkle_nodes(nodes, count, n_total, nthreads=4) == want
    # level-1 nodes of a flat 32-B tree (2 x 128-B chunks per window; the last
    # window of an odd chunk count padded with 0^128) -> the flat root
    n = 8 * count - 3 if count > 1 else 5
    items = O.splitmix_bytes(32 * n, 0x5EED000000000004)
    raw = bytes(items)
    ch = [raw[i:i + 128] for i in range(0, len(raw), 128)]
    if len(ch) % 2:
        ch.append(bytes(128))
    lv1 = np.frombuffer(b"".join(O.keccak256(ch[i] + ch[i + 1]) for i in range(0, len(ch), 2)), dtype=np.uint8)
    assert O.merkle_nodes(lv1, len(ch) // 2, n) == O.merkle_hash_flat(items, n, 32)
