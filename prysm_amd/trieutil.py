"""Host mirror of ``shared/trieutil`` (deposit sparse Merkle trie) over the
HIP engine.

Reference: shared/trieutil/deposit_trie.go:13-81, depth 32 from
shared/params/config.go:109.  ``DepositTrie`` keeps the reference's
incremental API (UpdateDepositTrie / GenerateMerkleBranch / Root) but never
hashes one deposit at a time: updates are queued and the trie is rebuilt by
one batched GPU build (leaf Keccak batch + one launch per level) the next
time it is read.  The batch build equals n incremental updates because every
internal node's last recomputation happens when its rightmost leaf is
inserted, at which point its subtree is final; tests check
this against a literal dict restatement.  Empty nodes are 0^32 (Go map
miss), the root of an empty trie is 0^32.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .hashutil import _flatten, _ptr

DEPOSIT_CONTRACT_TREE_DEPTH = 32  # shared/params/config.go:109
ZERO = bytes(32)


def build_levels(deposits: Sequence[bytes], depth: int = DEPOSIT_CONTRACT_TREE_DEPTH):
    """Batch build: returns (root, levels) with levels[d] an (c_d, 32) uint8
    array of the nodes at height d (d = 0: Hash(deposit))."""
    n = len(deposits)
    root = ctypes.create_string_buffer(32)
    if n == 0:
        _lib.check(_lib.load().mk_deposit_trie_build(None, None, 0, depth, None, root), "mk_deposit_trie_build")
        return root.raw, []
    data, offs = _flatten(deposits)
    nbytes = _lib.load().mk_deposit_trie_levels_bytes(n, depth)
    lv = np.empty(nbytes, dtype=np.uint8)
    _lib.check(_lib.load().mk_deposit_trie_build(_ptr(data), _ptr(offs), n, depth, _ptr(lv), root),
               "mk_deposit_trie_build")
    levels, pos, c = [], 0, n
    for _ in range(depth + 1):
        levels.append(lv[pos * 32:(pos + c) * 32].reshape(c, 32))
        pos += c
        c = (c + 1) // 2
    return root.raw, levels


class DepositTrie:
    """trieutil.DepositTrie (deposit_trie.go:13-16)."""

    def __init__(self, depth: int = DEPOSIT_CONTRACT_TREE_DEPTH):
        self.depth = depth
        self.deposit_count = 0
        self._deposits: List[bytes] = []
        self._levels: Optional[list] = None
        self._root = ZERO

    # NewDepositTrie (deposit_trie.go:20-26)
    @classmethod
    def new(cls) -> "DepositTrie":
        return cls()

    @classmethod
    def build(cls, deposits: Sequence[bytes], depth: int = DEPOSIT_CONTRACT_TREE_DEPTH) -> "DepositTrie":
        """Batch constructor: equals NewDepositTrie + UpdateDepositTrie for each."""
        t = cls(depth)
        t._deposits = [bytes(d) for d in deposits]
        t.deposit_count = len(t._deposits)
        return t

    def update_deposit_trie(self, deposit_data: bytes) -> None:
        """UpdateDepositTrie (deposit_trie.go:29-40): deferred to one batch."""
        self._deposits.append(bytes(deposit_data))
        self.deposit_count += 1
        self._levels = None

    UpdateDepositTrie = update_deposit_trie

    def _sync(self):
        if self._levels is None:
            self._root, self._levels = build_levels(self._deposits, self.depth)

    def generate_merkle_branch(self, index: int) -> List[bytes]:
        """GenerateMerkleBranch (deposit_trie.go:43-58): the sibling at each of
        the `depth` levels; missing nodes read as 0^32."""
        self._sync()
        out = []
        for d in range(self.depth):
            sib = (index >> d) ^ 1
            lvl = self._levels[d] if d < len(self._levels) else None
            out.append(bytes(lvl[sib]) if lvl is not None and sib < len(lvl) else ZERO)
        return out

    GenerateMerkleBranch = generate_merkle_branch

    def root(self) -> bytes:
        """Root (deposit_trie.go:61-63): node 1, 0^32 when empty."""
        self._sync()
        return self._root

    Root = root

    def leaf(self, index: int) -> bytes:
        self._sync()
        return bytes(self._levels[0][index]) if self._levels and index < len(self._levels[0]) else ZERO


def verify_merkle_branches(leaves: Sequence[bytes], branches: Sequence[Sequence[bytes]], depth: int,
                           indices: Sequence[int], roots: Sequence[bytes],
                           tree_depth: int = DEPOSIT_CONTRACT_TREE_DEPTH) -> List[bool]:
    """Batched VerifyMerkleBranch: one GPU thread folds one branch."""
    n = len(leaves)
    if n == 0:
        return []
    lv = np.frombuffer(b"".join(bytes(x) for x in leaves), dtype=np.uint8)
    rt = np.frombuffer(b"".join(bytes(x) for x in roots), dtype=np.uint8)
    br = np.frombuffer(b"".join(bytes(b[i]) for b in branches for i in range(depth)) or b"\0", dtype=np.uint8)
    idx = np.asarray(indices, dtype=np.uint64)
    ok = np.zeros(n, dtype=np.uint8)
    _lib.check(_lib.load().mk_verify_merkle_branches(_ptr(lv), _ptr(br), _ptr(idx), n, depth, tree_depth,
                                                     _ptr(rt), _ptr(ok)), "mk_verify_merkle_branches")
    return [bool(x) for x in ok]


def verify_merkle_branch(leaf: bytes, branch: Sequence[bytes], depth: int, index: int, root: bytes,
                         tree_depth: int = DEPOSIT_CONTRACT_TREE_DEPTH) -> bool:
    """VerifyMerkleBranch (deposit_trie.go:68-81)."""
    return verify_merkle_branches([leaf], [branch], depth, [index], [root], tree_depth)[0]


VerifyMerkleBranch = verify_merkle_branch
