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
    narrow top off the critical path.

    ``front="split"`` (the default): per trie, on the caller's current
    stream, the leaf hashes and the wide levels down to the first level of at
    most 2^17 nodes; on the side stream, overlapping the next trie's leaves,
    the latency-bound top (k_trie_top3 launches), the zero-sibling levels up
    to ``depth`` and the root.  ``slots`` sets (two by default: 2/3/4 sets
    and a wait every 2-3 submits measured the same, profiles/r02r/
    ring_ab.jsonl); a submit waits for the top of the trie ``slots`` submits
    back; the returned root is written by the time the side stream has run
    this submit's work, and stays valid for the next ``slots - 1`` submits.

    ``front="pipe"`` (opt-in; the C5 bench's form): trie i's leaves and
    levels 1-2 run in one phase-locked launch that also builds levels 3-7 of
    trie i-1 in its lock-step slots (mk_dev_deposit_trie_build_pipe); trie
    i-1's remaining top (levels 8 .. depth and the root) then runs on a
    high-priority side stream beside trie i+1's front.  **A trie's root is
    therefore written one submit later**: the tensor ``submit`` returns is
    produced once the next ``submit`` or ``flush()`` has been called (then
    synchronise, or wait on ``side``).  Level arrays and roots rotate over
    four sets; a returned root stays valid for the next two submits after it
    is produced.  Takes what mk_deposit_trie_pipe_ok accepts on the current
    stream (280-B deposits, 16-B aligned, n a multiple of 4096 within the
    stream's CUs); ValueError otherwise.  Submits may come from different
    streams: each front waits for the previous one, whose levels it reads.

    ``front="auto"``: "pipe" where the shape allows it, "split" otherwise
    (so the root's timing depends on the shape: only for callers that always
    flush() before reading roots)."""

    TOP_MAX = 1 << 17  # capi.cpp kTrieTopMax: levels at or below this width run k_trie_top3
    PIPE_TOP_FROM = 7  # the last level the pipelined front builds for the previous trie

    def __init__(self, n: int, deposit_len: int, depth: int, device, split: Optional[int] = None,
                 slots: int = 2, wait_every: int = 1, front: str = "split"):
        """``split``: the first level built on the side stream (default: the
        first level of at most TOP_MAX nodes); ``slots``, ``wait_every``:
        parallel.SlotRing (split front); ``front``: "split" (default), "pipe"
        or "auto" (pipe where the shape allows)."""
        if front not in ("auto", "pipe", "split"):
            raise ValueError(f"unknown front {front!r}")
        self.n, self.dl, self.depth = n, deposit_len, depth
        self.device = torch.device(device)
        if split is None:
            split = 0
            while split < depth and -(-n // (1 << split)) > self.TOP_MAX:
                split += 1
        self.split = split
        self.front = front
        self._nbytes = D.deposit_trie_levels_bytes(n, depth)
        self._slots = slots
        self._ring = SlotRing(slots, wait_every)
        # the pipelined form's four sets (allocated unless front == "split")
        # and the split form's `slots` sets (allocated on its first use): the
        # two forms never hand out the same root tensor
        self.levels, self.roots = self._sets(4) if front != "split" else ([], [])
        self._split_sets = None
        self.side = torch.cuda.Stream(device=self.device, priority=-1)  # its own hardware queue
        self._i = 0
        self._pending = None  # pipe: the set of the trie whose levels 3.. are not built yet
        self._done = {}  # pipe: trie index -> event after its top
        self._front_ev = None  # pipe: (stream, event) after the last front

    def _sets(self, k: int):
        return ([torch.empty(self._nbytes, dtype=torch.uint8, device=self.device) for _ in range(k)],
                [torch.empty(32, dtype=torch.uint8, device=self.device) for _ in range(k)])

    def _use_pipe(self, deposits: torch.Tensor) -> bool:
        if self.front == "split":
            return False
        ok = D.deposit_trie_pipe_ok(deposits, self.n, self.dl, self.depth)
        if self.front == "pipe" and not ok:
            raise ValueError("pipelined front: 280-B deposits, n a multiple of 4096 within the CU count")
        return ok

    def submit(self, deposits: torch.Tensor) -> torch.Tensor:
        """Enqueue the trie of n fixed-length deposits held in ``deposits``;
        returns its (32,) root tensor, produced on ``self.side`` (pipe: once
        the next submit or flush() has run)."""
        if deposits.numel() < self.n * self.dl:
            raise ValueError("deposit buffer shorter than n * deposit_len")
        cur = torch.cuda.current_stream(self.device)
        pipe = self._use_pipe(deposits)
        if pipe != getattr(self, "_last_pipe", pipe):  # finish the other form's pending trie first
            self.flush()
        self._last_pipe = pipe
        if not pipe:
            if self._split_sets is None:
                self._split_sets = self._sets(self._slots)
            slot = self._ring.acquire(cur)
            lv, root = self._split_sets[0][slot], self._split_sets[1][slot]
            D.deposit_trie_build(lv, self.n, deposits, self.n, self.dl, self.split, self.depth)
            self.side.wait_stream(cur)
            with torch.cuda.stream(self.side):
                D.deposit_trie_levels(lv, self.n, self.n, self.split, self.depth, self.depth, root)
                ev = torch.cuda.Event()
                ev.record(self.side)
            self._ring.release(ev)
            return root
        nsets = len(self.levels)
        i = self._i
        s = i % nsets
        self._i += 1
        # set s was last used by trie i - nsets, whose top (levels 8.. on the
        # side stream) must be done.  One cross-stream wait every second
        # submit (each costs ~10 us of command-processor time), on the top of
        # trie i - nsets + 1: the side stream runs in order, so it covers the
        # tries of this submit and the next.
        if i % 2 == 0:
            ev = self._done.get(i - nsets + 1)
            if ev is not None:
                cur.wait_event(ev)
        self._done.pop(i - nsets - 1, None)
        prev = self._pending
        if prev is not None and self._front_ev is not None and self._front_ev[0] != cur:
            cur.wait_event(self._front_ev[1])  # the previous front (levels 0-2 read here) ran elsewhere
        D.deposit_trie_build_pipe(self.levels[s], None if prev is None else self.levels[prev], self.n, deposits,
                                  self.n, self.dl, self.depth)
        if prev is not None:
            self._top(i - 1, prev, self.PIPE_TOP_FROM, cur)
        ev = torch.cuda.Event()
        ev.record(cur)
        self._front_ev = (cur, ev)
        self._pending = s
        return self.roots[s]

    def _top(self, trie: int, s: int, d_from: int, cur) -> None:
        self.side.wait_stream(cur)
        with torch.cuda.stream(self.side):
            if d_from == self.PIPE_TOP_FROM:  # beside the next front: one wave per SIMD at most
                D.deposit_trie_pipe_top(self.levels[s], self.n, self.n, self.depth, self.roots[s])
            else:
                D.deposit_trie_levels(self.levels[s], self.n, self.n, d_from, self.depth, self.depth, self.roots[s])
            ev = torch.cuda.Event()
            ev.record(self.side)
        self._done[trie] = ev

    def flush(self) -> None:
        """Finish the last pipelined trie (its levels 3 .. depth and root on
        the side stream); a no-op when nothing is pending."""
        if self._pending is not None:
            cur = torch.cuda.current_stream(self.device)
            if self._front_ev is not None and self._front_ev[0] != cur:
                cur.wait_event(self._front_ev[1])
            self._top(self._i - 1, self._pending, 2, cur)
            self._pending = None
