"""merkleHash of a stream of trees with each tree's top overlapped with the
next tree's leaves (one GPU, no collective).

A tree's narrow top levels are latency-bound (one permutation latency per
level); run on the stream that hashes the leaves they leave the
chip mostly idle.  ``MerklePipeline.submit`` therefore splits one
``merkleHash`` (shared/ssz/hash.go:194-239) at the level ``frontier_log2``
levels below the root: the leaf side (everything up to that level) runs on
the caller's current stream, the top (the remaining levels and the length
mix-in, hash.go:225-237) on a side stream, where it overlaps the leaf side of
the next submitted tree.  The split is the single-shard case of the subtree
sharding in parallel.py (same planner, same frontier finisher), so each root
is bit-identical to ``device.merkle_hash`` of the same items.

Frontier levels and roots rotate over ``slots`` buffer sets (three by
default): a submit waits for the top of the tree submitted ``slots`` calls
earlier before it overwrites that tree's buffers, and the root returned by a
submit stays valid for the next ``slots - 1`` submits.  The root is produced on ``side``; call ``torch.cuda.synchronize()`` or
make the consuming stream wait on ``side`` before reading it.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import device as D
from .parallel import SlotRing, frontier_count


class MerklePipeline:
    def __init__(self, n: int, item_len: int, device, frontier_log2: Optional[int] = None, leaf_levels: int = 5,
                 slots: int = 3, wait_every: int = 1):
        """Split ``frontier_log2`` levels below the root; by default at the
        leaf pass's output level, ``leaf_levels`` above the chunks (21 below
        the root of a 2^28-item tree of 32-B items).  ``slots`` buffer sets,
        ``wait_every``: parallel.SlotRing.  Three sets: a 2^25-item stream
        runs 1.288 -> 1.254 ms per tree against two (a tree's top waits for
        the next leaf pass's tail); 2^28 is the same either way
        (tools/ring_ab.py, profiles/r02r/ring_ab.jsonl)."""
        self.n, self.item_len = n, item_len
        self.device = torch.device(device)
        height, _, _ = D.shard_plan(n, item_len, 1)
        self.height = height
        if frontier_log2 is None:
            frontier_log2 = height - leaf_levels
        k = min(frontier_log2, height - 2)  # the planner's throughput passes fold at least 2 levels
        # a frontier level of one node is already the tree root's input: no top to split off
        self.k = k if k > 0 and frontier_count(n, item_len, height, k) > 1 else 0
        self.ws = D.subtree_workspace(n, item_len, self.device) if self.k else D.merkle_workspace(n, item_len,
                                                                                                   self.device)
        self._ring = SlotRing(slots, wait_every)
        self.outs = [torch.empty(32, dtype=torch.uint8, device=self.device) for _ in range(slots)]
        if self.k:
            self.count = frontier_count(n, item_len, height, self.k)
            self.bufs = [torch.empty(32 << self.k, dtype=torch.uint8, device=self.device) for _ in range(slots)]
            self.fin_ws = D.finish_workspace(self.count, self.device)
            # high priority: a default-priority side stream can land on the
            # current stream's hardware queue and serialise behind the next
            # leaf pass (rocprofv3: same Queue_Id); a priority stream gets
            # its own queue
            self.side = torch.cuda.Stream(device=self.device, priority=-1)
        else:
            self.side = torch.cuda.current_stream(self.device)

    def submit(self, items: torch.Tensor) -> torch.Tensor:
        """Enqueue merkleHash(items) (n items of item_len bytes); returns the
        (32,) uint8 root tensor, produced on ``self.side``."""
        cur = torch.cuda.current_stream(self.device)
        if not self.k:
            slot = self._ring.acquire(None)
            self._ring.release(None)
            return D.merkle_hash(items, self.n, self.item_len, out=self.outs[slot], ws=self.ws)
        slot = self._ring.acquire(cur)  # the top `slots` trees back no longer reads this set
        level = D.merkle_subtree_frontier(items, self.n, self.item_len, self.height, self.k, False,
                                          out=self.bufs[slot], ws=self.ws)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            root = D.merkle_finish_nodes(level, self.count, self.n, out=self.outs[slot], ws=self.fin_ws)
            ev = torch.cuda.Event()
            ev.record(self.side)
        self._ring.release(ev)
        return root


class TriePipeline:
    """Batch builds of a stream of deposit tries (one trie per ``submit``,
    trieutil.DepositTrie semantics, deposit_trie.go:29-63) with each trie's
    narrow top off the main stream.

    Per trie, on the caller's current stream: the leaf hashes
    (Hash(deposit), one launch) and the wide levels, down to the first level
    of at most 2^17 nodes (one launch per level, every lane busy).  On a
    high-priority side stream, overlapping the next trie's leaves: the
    latency-bound top (k_trie_top3 launches) plus the zero-sibling levels
    up to ``depth`` and the root.  Level arrays and roots rotate over
    ``slots`` sets (two by default: 2/3/4 sets and a wait every 2-3 submits
    measured the same, profiles/r02r/ring_ab.jsonl): a submit waits for the
    top of the trie ``slots`` submits back; a returned root stays valid for
    the next ``slots - 1`` submits."""

    TOP_MAX = 1 << 17  # capi.cpp kTrieTopMax: levels at or below this width run k_trie_top3

    def __init__(self, n: int, deposit_len: int, depth: int, device, split: Optional[int] = None,
                 slots: int = 2, wait_every: int = 1):
        """``split``: the first level built on the side stream (default: the
        first level of at most TOP_MAX nodes); ``slots``, ``wait_every``:
        parallel.SlotRing."""
        self.n, self.dl, self.depth = n, deposit_len, depth
        self.device = torch.device(device)
        if split is None:
            split = 0
            while split < depth and -(-n // (1 << split)) > self.TOP_MAX:
                split += 1
        self.split = split
        nbytes = D.deposit_trie_levels_bytes(n, depth)
        self._ring = SlotRing(slots, wait_every)
        self.levels = [torch.empty(nbytes, dtype=torch.uint8, device=self.device) for _ in range(slots)]
        self.roots = [torch.empty(32, dtype=torch.uint8, device=self.device) for _ in range(slots)]
        self.side = torch.cuda.Stream(device=self.device, priority=-1)  # its own hardware queue

    def submit(self, deposits: torch.Tensor) -> torch.Tensor:
        """Enqueue the trie of n fixed-length deposits held in ``deposits``;
        returns its (32,) root tensor, produced on ``self.side``."""
        if deposits.numel() < self.n * self.dl:
            raise ValueError("deposit buffer shorter than n * deposit_len")
        cur = torch.cuda.current_stream(self.device)
        slot = self._ring.acquire(cur)
        lv, root = self.levels[slot], self.roots[slot]
        D.deposit_trie_build(lv, self.n, deposits, self.n, self.dl, self.split, self.depth)
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            D.deposit_trie_levels(lv, self.n, self.n, self.split, self.depth, self.depth, root)
            ev = torch.cuda.Event()
            ev.record(self.side)
        self._ring.release(ev)
        return root
