"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes front-end of the C restatement in ``oracle/*.c`` plus a tiny
pure-Python Keccak used to cross-check the C code on small inputs.  Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module; the product package ``prysm_amd`` never does.

Reference algorithms restated (file:line under the reference root):
  * ``keccak256``      shared/hashutil/hash.go:11-25 (legacy Keccak-256,
    golang.org/x/crypto/sha3 @ b8fe1690c613, pad 0x01 .. 0x80, rate 136)
  * ``merkle_hash``    shared/ssz/hash.go:194-239
  * ``deposit_trie``   shared/trieutil/deposit_trie.go:29-81
  * ``merkle_root``    shared/hashutil/merkleRoot.go:12-30
  * ``DepositContract`` contracts/deposit-contract/depositContract.v.py:24-71
    (the same trie kept by the ETH1 contract: the second implementation of
    config 5's tree in the reference, with the deposit-data layout and the
    per-log previous_deposit_root that powchain checks)
Parity pins: hashutil/hash_test.go:13-31 KATs, ssz/hash_test.go:35-178
vectors, ssz/example_and_test.go:105,144 (see tests/golden/).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
DEPOSIT_TREE_DEPTH = 32  # shared/params/config.go:109

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.c_void_p
        L.or_keccak256.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.or_keccak_f1600.argtypes = [u8p]
        L.or_keccak_f1600_unrolled.argtypes = [u8p]
        L.or_set_fast_permutation.argtypes = [ctypes.c_int]
        L.or_set_fast_permutation.restype = ctypes.c_int
        L.or_sha3_256.argtypes = [u8p, ctypes.c_uint64, u8p]
        L.or_keccak256_batch.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_int]
        L.or_keccak256_var.argtypes = [u8p, u8p, ctypes.c_uint64, u8p]
        L.or_splitmix64_word.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.or_splitmix64_word.restype = ctypes.c_uint64
        L.or_fill_splitmix.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.or_merkle_hash.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_int]
        L.or_merkle_hash_var.argtypes = [u8p, u8p, ctypes.c_uint64, u8p]
        L.or_merkle_hash_gen.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, u8p, ctypes.c_int]
        L.or_merkle_nodes.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint64, u8p, ctypes.c_int]
        L.or_merkle_subtree_gen.argtypes = [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                            ctypes.c_uint64, ctypes.c_uint32, u8p, ctypes.c_int]
        L.or_deposit_trie_build.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, u8p]
        L.or_deposit_trie_incremental.argtypes = [u8p, u8p, ctypes.c_uint64, ctypes.c_uint32, u8p]
        L.or_verify_merkle_branch.argtypes = [u8p, u8p, ctypes.c_uint32, ctypes.c_uint64,
                                              ctypes.c_uint32, u8p]
        L.or_merkle_root.argtypes = [u8p, u8p, ctypes.c_uint64, u8p]
        L.or_struct_roots.argtypes = [u8p, ctypes.c_uint64, ctypes.c_uint32, u8p, u8p, u8p, ctypes.c_uint32,
                                      u8p, ctypes.c_int]
        for name in ("or_merkle_hash", "or_merkle_hash_var", "or_merkle_hash_gen", "or_merkle_nodes",
                     "or_merkle_subtree_gen", "or_deposit_trie_build", "or_deposit_trie_incremental",
                     "or_verify_merkle_branch",
                     "or_merkle_root"):
            getattr(L, name).restype = ctypes.c_int
        _lib = L
    return _lib


def keccak_f(state: np.ndarray, unrolled: bool = False) -> np.ndarray:
    """One Keccak-f[1600] of a (25,) uint64 state (a copy): the loop form or
    the unrolled x/crypto-shaped form (keccak_fast.c)."""
    a = np.ascontiguousarray(state, dtype=np.uint64).copy()
    (lib().or_keccak_f1600_unrolled if unrolled else lib().or_keccak_f1600)(a.ctypes.data)
    return a


class fast_permutation:
    """``with fast_permutation():`` every oracle sponge in this process runs
    the unrolled permutation (the CPU baseline's); restored on exit."""

    def __enter__(self):
        self._was = lib().or_set_fast_permutation(1)
        return self

    def __exit__(self, *exc):
        lib().or_set_fast_permutation(self._was)
        return False


def _buf(b: bytes):
    return ctypes.create_string_buffer(bytes(b), max(1, len(b)))


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _flat(msgs):
    msgs = [bytes(m) for m in msgs]
    offs = np.zeros(len(msgs) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(m) for m in msgs]) if msgs else []
    data = np.frombuffer(b"".join(msgs) + b"\0", dtype=np.uint8).copy()
    return data, offs


# --------------------------------------------------------------- digests
def keccak256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_keccak256(_buf(data), len(data), out)
    return out.raw


def sha3_256(data: bytes) -> bytes:
    out = ctypes.create_string_buffer(32)
    lib().or_sha3_256(_buf(data), len(data), out)
    return out.raw


def keccak256_batch(arr: np.ndarray, msg_len: int, nthreads: int = 1) -> np.ndarray:
    """arr: uint8 array of n*msg_len bytes -> (n, 32) uint8."""
    arr = np.ascontiguousarray(arr, dtype=np.uint8)
    n = arr.size // msg_len if msg_len else 0
    out = np.empty((n, 32), dtype=np.uint8)
    lib().or_keccak256_batch(_ptr(arr), n, msg_len, _ptr(out), nthreads)
    return out


def keccak256_var(msgs) -> np.ndarray:
    data, offs = _flat(msgs)
    out = np.empty((len(offs) - 1, 32), dtype=np.uint8)
    lib().or_keccak256_var(_ptr(data), _ptr(offs), len(offs) - 1, _ptr(out))
    return out


# --------------------------------------------------------------- synthetic input
def splitmix_bytes(nbytes: int, seed: int, word0: int = 0) -> np.ndarray:
    out = np.empty(max(1, nbytes), dtype=np.uint8)
    lib().or_fill_splitmix(_ptr(out), nbytes, seed, word0)
    return out[:nbytes]


# --------------------------------------------------------------- merkleHash
def merkle_hash_flat(items: np.ndarray, n: int, item_len: int, nthreads: int = 1) -> bytes:
    items = np.ascontiguousarray(items, dtype=np.uint8)
    out = ctypes.create_string_buffer(32)
    rc = lib().or_merkle_hash(_ptr(items) if items.size else None, n, item_len, out, nthreads)
    if rc != 0:
        raise ZeroDivisionError("integer divide by zero") if rc == -1 else RuntimeError(rc)
    return out.raw


def merkle_hash(lst) -> bytes:
    """Exact list semantics of ssz.merkleHash([][]byte) (hash.go:194-239)."""
    data, offs = _flat(lst)
    out = ctypes.create_string_buffer(32)
    rc = lib().or_merkle_hash_var(_ptr(data), _ptr(offs), len(lst), out)
    if rc == -1:
        raise ZeroDivisionError("integer divide by zero")
    return out.raw


def elem_digests(elems: np.ndarray, n: int, elem_len: int, nthreads: int = 1, chunk: int = 1 << 22) -> np.ndarray:
    """hashedEncoding of n byte strings of elem_len bytes (hash.go:100-107):
    Keccak(le32(elem_len) || element) -> (n, 32), in chunks of messages."""
    elems = np.ascontiguousarray(elems, dtype=np.uint8).reshape(-1)
    out = np.empty((n, 32), dtype=np.uint8)
    pre = np.frombuffer(int(elem_len).to_bytes(4, "little"), dtype=np.uint8)
    for lo in range(0, n, chunk):
        hi = min(n, lo + chunk)
        msgs = np.empty((hi - lo, 4 + elem_len), dtype=np.uint8)
        msgs[:, :4] = pre
        if elem_len:
            msgs[:, 4:] = elems[lo * elem_len:hi * elem_len].reshape(hi - lo, elem_len)
        out[lo:hi] = keccak256_batch(msgs.reshape(-1), 4 + elem_len, nthreads)
    return out


def tree_hash_bytes_list(elems: np.ndarray, n: int, elem_len: int, nthreads: int = 1) -> bytes:
    """ssz.TreeHash of a slice of n byte strings of elem_len bytes
    (makeSliceHasher, hash.go:118-139): merkleHash over their hashedEncoding
    digests.  Composition of the pinned Keccak and merkleHash restatements."""
    return merkle_hash_flat(elem_digests(elems, n, elem_len, nthreads).reshape(-1), n, 32, nthreads)


def merkle_hash_gen(n: int, item_len: int, seed: int, nthreads: int = 1) -> bytes:
    out = ctypes.create_string_buffer(32)
    rc = lib().or_merkle_hash_gen(n, item_len, seed, out, nthreads)
    if rc != 0:
        raise RuntimeError(rc)
    return out.raw


def merkle_nodes(nodes: np.ndarray, count: int, n_total: int, nthreads: int = 1) -> bytes:
    """merkleHash continued from a level of `count` 32-B nodes, then the
    length mix-in of n_total items (or_merkle_nodes)."""
    nodes = np.ascontiguousarray(nodes, dtype=np.uint8).reshape(-1)
    assert nodes.size >= 32 * count
    out = ctypes.create_string_buffer(32)
    rc = lib().or_merkle_nodes(_ptr(nodes), count, n_total, out, nthreads)
    if rc != 0:
        raise RuntimeError(rc)
    return out.raw


def merkle_subtree_gen(n: int, item_len: int, seed: int, shard: int, height: int,
                       nthreads: int = 1) -> bytes:
    out = ctypes.create_string_buffer(32)
    rc = lib().or_merkle_subtree_gen(n, item_len, seed, shard, height, out, nthreads)
    if rc != 0:
        raise RuntimeError(rc)
    return out.raw


# --------------------------------------------------------------- deposit trie
def deposit_trie_levels(deposits, depth: int = DEPOSIT_TREE_DEPTH):
    """Returns (root, levels) where levels[d] is a list of 32-B nodes."""
    n = len(deposits)
    data, offs = _flat(deposits)
    counts = []
    c = n
    for _ in range(depth + 1):
        counts.append(c)
        c = (c + 1) // 2
    total = sum(counts) if n else 0
    lv = np.zeros(max(1, total * 32), dtype=np.uint8)
    root = ctypes.create_string_buffer(32)
    lib().or_deposit_trie_build(_ptr(data), _ptr(offs), n, depth, _ptr(lv) if n else None, root)
    levels, pos = [], 0
    if n:
        for c in counts:
            levels.append([bytes(lv[(pos + i) * 32:(pos + i + 1) * 32]) for i in range(c)])
            pos += c
    return root.raw, levels


def deposit_trie_incremental_root(deposits, depth: int = DEPOSIT_TREE_DEPTH) -> bytes:
    """Root after n calls of the reference's UpdateDepositTrie (C restatement,
    1 + depth hashes per deposit)."""
    data, offs = _flat(deposits)
    root = ctypes.create_string_buffer(32)
    lib().or_deposit_trie_incremental(_ptr(data), _ptr(offs), len(deposits), depth, root)
    return root.raw


class DictTrie:
    """Literal restatement of shared/trieutil/deposit_trie.go:13-63: the
    incremental trie over a map whose missing keys read as 0^32."""

    def __init__(self, depth: int = DEPOSIT_TREE_DEPTH):
        self.depth, self.count, self.m = depth, 0, {}

    def update(self, data: bytes) -> None:  # UpdateDepositTrie (:29-40)
        idx = self.count + (1 << self.depth)
        self.m[idx] = keccak256(data)
        for _ in range(self.depth):
            idx //= 2
            self.m[idx] = keccak256(self.m.get(idx * 2, bytes(32)) + self.m.get(idx * 2 + 1, bytes(32)))
        self.count += 1

    def branch(self, index: int):  # GenerateMerkleBranch (:43-58)
        idx = index + (1 << self.depth)
        out = []
        for _ in range(self.depth):
            out.append(self.m.get(idx - 1 if idx % 2 else idx + 1, bytes(32)))
            idx //= 2
        return out

    def root(self) -> bytes:  # Root (:61-63)
        return self.m.get(1, bytes(32))


class DepositContract:
    """Restatement of the Vyper deposit contract's tree
    (contracts/deposit-contract/depositContract.v.py): deposit_data =
    to_bytes(amount) || to_bytes(timestamp) || deposit_input (:26-27, :43;
    to_bytes = the low 8 bytes of the uint256, big-endian), leaf at heap index
    count + 2^32 (:44, :49), every ancestor rehashed from its two children
    with missing map keys reading as 0^32 (:50-52), root = node 1 (:31-32),
    branch = the sibling at each level (:65-71).  deposit() returns the
    Deposit event (:46): (previous_deposit_root, deposit_data, index bytes)."""

    def __init__(self, depth: int = DEPOSIT_TREE_DEPTH):
        self.depth, self.count, self.tree = depth, 0, {}

    @staticmethod
    def to_bytes(value: int) -> bytes:
        return (value % (1 << 256)).to_bytes(32, "big")[24:]

    def get_deposit_root(self) -> bytes:
        return self.tree.get(1, bytes(32))

    def deposit(self, amount_gwei: int, timestamp: int, deposit_input: bytes):
        data = self.to_bytes(amount_gwei) + self.to_bytes(timestamp) + bytes(deposit_input)
        index = self.count + (1 << self.depth)
        event = (self.get_deposit_root(), data, self.to_bytes(index))
        self.tree[index] = keccak256(data)
        for _ in range(self.depth):
            index //= 2
            self.tree[index] = keccak256(self.tree.get(2 * index, bytes(32)) + self.tree.get(2 * index + 1, bytes(32)))
        self.count += 1
        return event

    def get_branch(self, leaf: int):
        index = leaf + (1 << self.depth)
        out = []
        for _ in range(self.depth):
            out.append(self.tree.get(index ^ 1, bytes(32)))
            index //= 2
        return out


def verify_merkle_branch(leaf: bytes, branch, depth: int, index: int, root: bytes,
                         tree_depth: int = DEPOSIT_TREE_DEPTH) -> bool:
    br = b"".join(bytes(b) for b in branch)
    return bool(lib().or_verify_merkle_branch(_buf(leaf), _buf(br), depth, index, tree_depth, _buf(root)))


def merkle_root(values) -> bytes:
    data, offs = _flat(values)
    out = ctypes.create_string_buffer(32)
    if lib().or_merkle_root(_ptr(data), _ptr(offs), len(values), out) != 0:
        raise IndexError("index out of range")
    return out.raw


# --------------------------------------------------------------- flat structs
def struct_roots(records: np.ndarray, n: int, rec_len: int, fields, nthreads: int = 1) -> np.ndarray:
    """fields: [(kind, offset, len)] with kind 1 = bytes (hashed), 2 = raw."""
    rec = np.ascontiguousarray(records, dtype=np.uint8).reshape(-1)
    kind = np.array([f[0] for f in fields], dtype=np.uint32)
    off = np.array([f[1] for f in fields], dtype=np.uint32)
    ln = np.array([f[2] for f in fields], dtype=np.uint32)
    out = np.empty((n, 32), dtype=np.uint8)
    lib().or_struct_roots(_ptr(rec), n, rec_len, _ptr(kind), _ptr(off), _ptr(ln), len(fields), _ptr(out), nthreads)
    return out


# --------------------------------------------------------------- pure Python (small inputs)
_RC = [0x0000000000000001, 0x0000000000008082, 0x800000000000808A, 0x8000000080008000,
       0x000000000000808B, 0x0000000080000001, 0x8000000080008081, 0x8000000000008009,
       0x000000000000008A, 0x0000000000000088, 0x0000000080008009, 0x000000008000000A,
       0x000000008000808B, 0x800000000000008B, 0x8000000000008089, 0x8000000000008003,
       0x8000000000008002, 0x8000000000000080, 0x000000000000800A, 0x800000008000000A,
       0x8000000080008081, 0x8000000000008080, 0x0000000080000001, 0x8000000080008008]
_RHO = [0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14]
_M = (1 << 64) - 1


def _rot(v, n):
    return ((v << n) | (v >> (64 - n))) & _M if n else v


def py_keccak_f(A):
    for rc in _RC:
        C = [A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20] for x in range(5)]
        D = [C[(x + 4) % 5] ^ _rot(C[(x + 1) % 5], 1) for x in range(5)]
        A = [A[i] ^ D[i % 5] for i in range(25)]
        B = [0] * 25
        for x in range(5):
            for y in range(5):
                B[y + 5 * ((2 * x + 3 * y) % 5)] = _rot(A[x + 5 * y], _RHO[x + 5 * y])
        A = [B[x + 5 * y] ^ ((~B[(x + 1) % 5 + 5 * y]) & B[(x + 2) % 5 + 5 * y]) for y in range(5)
             for x in range(5)]
        A[0] ^= rc
    return A


def py_keccak256(data: bytes, pad: int = 0x01) -> bytes:
    rate = 136
    msg = bytearray(data)
    msg.append(pad)
    while len(msg) % rate:
        msg.append(0)
    msg[-1] ^= 0x80
    A = [0] * 25
    for off in range(0, len(msg), rate):
        for i in range(rate // 8):
            A[i] ^= int.from_bytes(msg[off + 8 * i: off + 8 * i + 8], "little")
        A = py_keccak_f(A)
    return b"".join(A[i].to_bytes(8, "little") for i in range(4))
