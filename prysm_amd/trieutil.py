"""Host mirror of ``shared/trieutil`` (deposit sparse Merkle trie) over the
HIP engine.

Reference: shared/trieutil/deposit_trie.go:13-81, depth 32 from
shared/params/config.go:109.  ``DepositTrie`` keeps the reference's
incremental API (UpdateDepositTrie / GenerateMerkleBranch / Root) over a
device-resident trie handle (``mk_deposit_trie_*``): every level stays in
HBM, and the deposits queued by UpdateDepositTrie are appended at the next
read by one library call that hashes the new leaves and recomputes only the
right edge of each level (<= k/2^d + 2 nodes at level d for k new
deposits).  The live caller, powchain's ``saveInTrie``
(beacon-chain/powchain/service.go:379-386), reads Root() before every
update, so each log costs one leaf hash plus ``depth`` node hashes — the
reference's own O(depth) per deposit — instead of a rebuild.  A batch of
updates followed by one read is the batch build (leaf batch + one launch per
wide level).  Empty nodes are 0^32 (Go map miss); the root of an empty trie
is 0^32.
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
        _lib.invoke("mk_deposit_trie_build", None, None, 0, depth, None, root)
        return root.raw, []
    data, offs = _flatten(deposits)
    nbytes = _lib.load().mk_deposit_trie_levels_bytes(n, depth)
    lv = np.empty(nbytes, dtype=np.uint8)
    _lib.invoke("mk_deposit_trie_build", _ptr(data), _ptr(offs), n, depth, _ptr(lv), root)
    levels, pos, c = [], 0, n
    for _ in range(depth + 1):
        levels.append(lv[pos * 32:(pos + c) * 32].reshape(c, 32))
        pos += c
        c = (c + 1) // 2
    return root.raw, levels


class DepositTrie:
    """trieutil.DepositTrie (deposit_trie.go:13-16) over a device trie handle."""

    def __init__(self, depth: int = DEPOSIT_CONTRACT_TREE_DEPTH, capacity: int = 0, device: int = -1):
        self.depth = depth
        self.deposit_count = 0
        self._queue: List[bytes] = []
        self._handle: Optional[ctypes.c_void_p] = None
        self._capacity = capacity
        self._device = device

    def __del__(self):
        h = getattr(self, "_handle", None)
        if h is not None and _lib is not None:
            try:
                _lib.load().mk_deposit_trie_free(h)
            except Exception:
                pass

    # NewDepositTrie (deposit_trie.go:20-26)
    @classmethod
    def new(cls) -> "DepositTrie":
        return cls()

    @classmethod
    def build(cls, deposits: Sequence[bytes], depth: int = DEPOSIT_CONTRACT_TREE_DEPTH) -> "DepositTrie":
        """Batch constructor: equals NewDepositTrie + UpdateDepositTrie for each."""
        t = cls(depth, capacity=len(deposits))
        for d in deposits:
            t.update_deposit_trie(d)
        return t

    def update_deposit_trie(self, deposit_data: bytes) -> None:
        """UpdateDepositTrie (deposit_trie.go:29-40): queued, appended on the next read."""
        self._queue.append(bytes(deposit_data))
        self.deposit_count += 1

    UpdateDepositTrie = update_deposit_trie

    def _flush(self):
        if not self._queue:
            return
        if self._handle is None:
            h = ctypes.c_void_p()
            _lib.invoke("mk_deposit_trie_new", self.depth, max(self._capacity, len(self._queue)), ctypes.byref(h),
                        device=self._device)
            self._handle = h
        data, offs = _flatten(self._queue)
        _lib.invoke("mk_deposit_trie_append", self._handle, _ptr(data), _ptr(offs), len(self._queue),
                    device=self._device)
        self._queue = []

    def save_logs(self, deposits: Sequence[bytes], log_roots: Sequence[bytes]) -> List[bool]:
        """powchain's ProcessDepositLog -> saveInTrie loop over a batch of logs
        (beacon-chain/powchain/service.go:248-258, 379-386) in one device call:
        in log order, deposit j is appended iff Root() before it equals
        log_roots[j], else the log is skipped.  Returns the per-log accept
        flags; the roots are computed on the device in parallel."""
        if len(deposits) != len(log_roots):
            raise ValueError("one merkle root per log")
        self._flush()
        k = len(deposits)
        if k == 0:
            return []
        if self._handle is None:
            h = ctypes.c_void_p()
            _lib.invoke("mk_deposit_trie_new", self.depth, max(self._capacity, k), ctypes.byref(h),
                        device=self._device)
            self._handle = h
        data, offs = _flatten([bytes(d) for d in deposits])
        roots = b"".join(bytes(r) for r in log_roots)
        if len(roots) != 32 * k:
            raise ValueError("log roots are 32 bytes")
        acc = ctypes.create_string_buffer(k)
        _lib.invoke("mk_deposit_trie_save_logs", self._handle, _ptr(data), _ptr(offs), k, roots, acc,
                    device=self._device)
        flags = [b == 1 for b in acc.raw]
        self.deposit_count += sum(flags)
        return flags

    SaveLogs = save_logs

    def generate_merkle_branch(self, index: int) -> List[bytes]:
        """GenerateMerkleBranch (deposit_trie.go:43-58): the sibling at each of
        the `depth` levels; missing nodes read as 0^32."""
        self._flush()
        if self._handle is None:
            return [ZERO] * self.depth
        out = ctypes.create_string_buffer(32 * self.depth)
        _lib.invoke("mk_deposit_trie_branch", self._handle, index, out, device=self._device)
        raw = out.raw
        return [raw[32 * d:32 * d + 32] for d in range(self.depth)]

    GenerateMerkleBranch = generate_merkle_branch

    def root(self) -> bytes:
        """Root (deposit_trie.go:61-63): node 1, 0^32 when empty."""
        self._flush()
        if self._handle is None:
            return ZERO
        out = ctypes.create_string_buffer(32)
        _lib.invoke("mk_deposit_trie_root", self._handle, out, device=self._device)
        return out.raw

    Root = root

    def leaf(self, index: int) -> bytes:
        """Hash(deposit index) (the leaf the trie stores), 0^32 past the end."""
        self._flush()
        if self._handle is None or index >= self.deposit_count:
            return ZERO
        out = ctypes.create_string_buffer(32)
        _lib.invoke("mk_deposit_trie_leaves", self._handle, index, 1, out, device=self._device)
        return out.raw


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
    _lib.invoke("mk_verify_merkle_branches", _ptr(lv), _ptr(br), _ptr(idx), n, depth, tree_depth, _ptr(rt), _ptr(ok))
    return [bool(x) for x in ok]


def verify_merkle_branch(leaf: bytes, branch: Sequence[bytes], depth: int, index: int, root: bytes,
                         tree_depth: int = DEPOSIT_CONTRACT_TREE_DEPTH) -> bool:
    """VerifyMerkleBranch (deposit_trie.go:68-81)."""
    return verify_merkle_branches([leaf], [branch], depth, [index], [root], tree_depth)[0]


VerifyMerkleBranch = verify_merkle_branch
