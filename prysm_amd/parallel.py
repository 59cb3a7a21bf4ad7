"""Multi-GPU merkleHash by subtree sharding.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Each rank Merkleizes its own power-of-two-aligned run of 2^height chunks to a
32-byte subtree root with no data-path communication; the only exchange is
one all-gather of 32 B per rank; rank 0 then runs the reference's level loop
over the gathered roots and the length mix-in (hash.go:225-237).

Frontier mode (``frontier_log2 = k > 0``): each rank stops k levels below
its shard root and contributes its 2^k nodes of that level (8 KB at k = 8);
the gathered blocks, in shard order, are that level of the whole tree, and
rank 0's finisher runs the k + log2(world) top levels.  The k narrowest,
latency-bound levels of every shard (one permutation latency each) leave the
ranks' critical path for a finisher that overlaps rank 0's next step.

The compute steps are injectable so the orchestration and the collective can
be exercised on CPU with the gloo backend (tests/test_distributed.py); the
defaults are the HIP entry points of prysm_amd.device.
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from datetime import timedelta
from typing import Callable, Optional

import torch
import torch.distributed as dist


def dist_timeout() -> timedelta:
    """Collective / rendezvous timeout of the bench's process group: 120 s
    unless PRYSM_DIST_TIMEOUT (seconds) says otherwise.  torch's default (10
    minutes) would let a hung first cross-device RCCL init or all-gather burn
    a whole driver run silently."""
    return timedelta(seconds=float(os.environ.get("PRYSM_DIST_TIMEOUT", "120")))


def init_process_group(backend: str, device=None, timeout: Optional[timedelta] = None) -> None:
    """One process per GPU.  With backend "nccl" (RCCL over xGMI) the
    process group's internal stream is created at high priority: the frontier
    all-gather then gets its own hardware queue instead of queueing behind
    the next leaf pass that the main stream has already issued (the same rule
    as every side stream here).  Every rendezvous and
    collective gives up after `timeout` (dist_timeout() by default) instead
    of waiting forever for a rank that never comes."""
    timeout = timeout or dist_timeout()
    if backend == "nccl":
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", device_id=device, pg_options=opts, timeout=timeout)
    else:
        dist.init_process_group(backend, timeout=timeout)


class SlotRing:
    """Buffer-set rotation of a stream of trees (the pipelines here and in
    pipeline.py).  Submit i uses set ``i % slots`` on the main stream and
    records its side-stream work; set i % slots may be overwritten only once
    the side work of submit i - slots is done.  Instead of one cross-stream
    wait per submit (~10 µs of command-processor time each in the C5 trace),
    the main stream waits every ``wait_every`` submits, on the side work of
    submit i - (slots - wait_every + 1): the side stream runs in order, so
    that covers every submit up to the next wait."""

    def __init__(self, slots: int = 2, wait_every: int = 1):
        if not 1 <= wait_every < slots:
            raise ValueError("need 1 <= wait_every < slots")
        self.slots, self.every = slots, wait_every
        self.dist = slots - wait_every + 1
        self._ev = {}
        self._i = 0

    def acquire(self, cur=None) -> int:
        """The set of the next submit; `cur` (the main stream; None on the
        CPU) waits here when the schedule asks for it."""
        i = self._i
        if cur is not None and i % self.every == 0:
            ev = self._ev.get(i - self.dist)
            if ev is not None:
                cur.wait_event(ev)
        return i % self.slots

    def release(self, ev=None) -> None:
        """Records the side work of the current submit (an event, or None)."""
        self._ev[self._i] = ev
        self._ev.pop(self._i - self.slots, None)  # no later wait names it
        self._i += 1


class PhaseTimer:
    """Per-step phases of one rank's sharded merkleHash step, for the N-GPU
    bench record: marks recorded on the stream that runs each
    phase (torch.cuda.Event = hipEvents on the GPU; the host clock on the
    CPU), read once the timed steps are synchronised.

      leaf    leaf0 -> leaf1     the rank's leaf pass (one-stream step: the
                                 leaf pass and the node passes to the frontier,
                                 one library call)
      nodes   nodes0 -> nodes1   the node passes to the frontier (pipelined
                                 step, side stream; 0 in the one-stream step)
      gather  -> gather1         the frontier all-gather, from the end of the
                                 phase before it
      finish  gather1 -> finish1 rank 0's finisher (0 on the other ranks)

    In the one-stream step the phases run back to back and sum to the step;
    in the pipelined step nodes + gather + finish run on a side stream beside
    the next leaf pass, so the step is the leaf pass plus whatever of the
    side work does not hide."""

    PHASES = ("leaf", "nodes", "gather", "finish")

    def __init__(self, cuda: bool):
        self.cuda = cuda
        self.steps = []
        self._cur = None

    def start_step(self) -> None:
        self._cur = {}
        self.steps.append(self._cur)

    def stop(self) -> None:
        """No marks until the next start_step (steps outside the timed region)."""
        self._cur = None

    def mark(self, name: str, stream=None) -> None:
        if self._cur is None:
            return
        if self.cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
            self._cur[name] = ev
        else:
            import time

            self._cur[name] = time.perf_counter()

    def _ms(self, a, b) -> float:
        if self.cuda:
            return a.elapsed_time(b)
        return (b - a) * 1e3

    def phases_ms(self) -> dict:
        """Average ms per phase over the recorded steps (call after the
        streams that ran them are synchronised)."""
        tot = dict.fromkeys(self.PHASES, 0.0)
        for m in self.steps:
            if "leaf0" in m and "leaf1" in m:
                tot["leaf"] += self._ms(m["leaf0"], m["leaf1"])
            if "nodes0" in m and "nodes1" in m:
                tot["nodes"] += self._ms(m["nodes0"], m["nodes1"])
            prev = m.get("nodes1", m.get("leaf1"))
            if prev is not None and "gather1" in m:
                tot["gather"] += self._ms(prev, m["gather1"])
            if "gather1" in m and "finish1" in m:
                tot["finish"] += self._ms(m["gather1"], m["finish1"])
        n = max(len(self.steps), 1)
        return {k: v / n for k, v in tot.items()}

    def record(self, world: int, device=None, group=None) -> dict:
        """This rank's phases plus every rank's (all-gathered; a collective:
        every rank calls it), for the bench JSON: {"phases_ms": {...,
        "sum": ...}, "per_rank_phases_ms": [[leaf, nodes, gather, finish],
        ...]}."""
        mine = self.phases_ms()
        vec = torch.tensor([mine[k] for k in self.PHASES], dtype=torch.float64,
                           device=device if device is not None else "cpu")
        if world > 1:
            allv = torch.empty(world * len(self.PHASES), dtype=torch.float64, device=vec.device)
            dist.all_gather_into_tensor(allv, vec, group=group)
            rows = allv.view(world, len(self.PHASES)).tolist()
        else:
            rows = [vec.tolist()]
        out = {k: round(v, 4) for k, v in mine.items()}
        out["sum"] = round(sum(mine.values()), 4)
        return {"phases_ms": out, "per_rank_phases_ms": [[round(x, 4) for x in r] for r in rows]}


@dataclass
class ShardPlan:
    height: int
    nonempty: int
    begin: list  # item_begin[world+1]

    def items(self, rank: int):
        return self.begin[rank], self.begin[rank + 1]


def plan(n: int, item_len: int, world: int, plan_fn: Optional[Callable] = None) -> ShardPlan:
    if plan_fn is None:
        from .device import shard_plan as plan_fn
    h, ne, begin = plan_fn(n, item_len, world)
    return ShardPlan(h, ne, begin)


def sharded_merkle_hash(local_items: torch.Tensor, n_total: int, item_len: int, sp: ShardPlan,
                        rank: int, world: int, group=None,
                        subtree_fn: Optional[Callable] = None,
                        full_fn: Optional[Callable] = None,
                        finish_fn: Optional[Callable] = None,
                        gather_buf: Optional[torch.Tensor] = None,
                        finish_stream=None, frontier_log2: int = 0,
                        frontier_fn: Optional[Callable] = None,
                        finish_nodes_fn: Optional[Callable] = None,
                        timer: Optional[PhaseTimer] = None) -> Optional[torch.Tensor]:
    """Returns the 32-byte merkleHash root on rank 0 (None elsewhere).

    ``local_items`` holds this rank's items [begin[rank], begin[rank+1]).
    When the tree is too small to shard (sp.nonempty == 1) rank 0 hashes
    everything and the others contribute nothing.

    ``finish_stream`` (a torch.cuda.Stream, rank 0): run the finisher there so
    it overlaps the caller's next Merkleization instead of delaying it; the
    returned root is then produced on that stream (synchronize before use).
    The next call's all-gather waits for it before reusing ``gather_buf``.

    ``frontier_log2`` (0 < k < sp.height): gather each shard's 2^k-node level
    instead of its root (``frontier_fn(items, sn, il, h, k, pad)`` returns a
    32<<k-byte buffer holding the shard's nodes first;
    ``finish_nodes_fn(level, count, n_total)`` finishes); gather_buf then
    holds world << k nodes.  ``timer``: PhaseTimer marks of the step's
    phases (leaf, gather, finish)."""
    if subtree_fn is None or full_fn is None or finish_fn is None:
        from . import device as D
        subtree_fn = subtree_fn or D.merkle_subtree
        full_fn = full_fn or D.merkle_hash
        finish_fn = finish_fn or D.merkle_finish
    lo, hi = sp.items(rank)
    dev = local_items.device
    if sp.nonempty <= 1:
        if rank == 0:
            return full_fn(local_items, n_total, item_len)
        return None
    k = frontier_log2 if 0 < frontier_log2 < sp.height else 0
    cur = torch.cuda.current_stream(dev) if local_items.is_cuda else None
    if timer is not None:
        timer.mark("leaf0", cur)
    if k:
        if frontier_fn is None or finish_nodes_fn is None:
            from . import device as D
            frontier_fn = frontier_fn or D.merkle_subtree_frontier
            finish_nodes_fn = finish_nodes_fn or D.merkle_finish_nodes
        block = 32 << k
        if hi > lo:
            root = frontier_fn(local_items, hi - lo, item_len, sp.height, k, True)
            if root.numel() != block:  # send a full block; only the counted nodes are read
                full = torch.zeros(block, dtype=torch.uint8, device=dev)
                full[:root.numel()] = root
                root = full
        else:
            root = torch.zeros(block, dtype=torch.uint8, device=dev)
    elif hi > lo:
        root = subtree_fn(local_items, hi - lo, item_len, sp.height, True)
    else:
        root = torch.zeros(32, dtype=torch.uint8, device=dev)
    if timer is not None:
        timer.mark("leaf1", cur)
    if gather_buf is None:
        gather_buf = torch.empty(world * root.numel(), dtype=torch.uint8, device=dev)
    if finish_stream is not None:  # the previous finish still reads gather_buf
        torch.cuda.current_stream(dev).wait_stream(finish_stream)
    if root.is_cuda and dist.get_backend(group) == "gloo":
        # rehearsal of the N-rank path on one GPU (bench.py --backend gloo):
        # gloo gathers host tensors
        host = torch.empty(gather_buf.numel(), dtype=torch.uint8)
        dist.all_gather_into_tensor(host, root.cpu(), group=group)
        gather_buf.copy_(host)
    else:
        dist.all_gather_into_tensor(gather_buf, root, group=group)
    if timer is not None:
        timer.mark("gather1", cur)
    if rank == 0:
        if k:
            last = sp.nonempty - 1
            count = (last << k) + frontier_count(sp.begin[last + 1] - sp.begin[last], item_len, sp.height, k)
            fin = lambda: finish_nodes_fn(gather_buf, count, n_total)  # noqa: E731
        else:
            fin = lambda: finish_fn(gather_buf, sp.nonempty, n_total)  # noqa: E731
        if finish_stream is not None:
            finish_stream.wait_stream(torch.cuda.current_stream(dev))
            # the finisher reads gather_buf on finish_stream after this call
            # returns: keep the caching allocator from handing its block to the
            # next allocation on the current stream meanwhile
            gather_buf.record_stream(finish_stream)
            with torch.cuda.stream(finish_stream):
                r = fin()
                if timer is not None:
                    timer.mark("finish1", finish_stream)
                return r
        r = fin()
        if timer is not None:
            timer.mark("finish1", cur)
        return r
    return None


def frontier_count(shard_n: int, item_len: int, height: int, k: int) -> int:
    """Nodes of a shard `k` levels below its root (>= 1: with pad_at_one the
    odd rule keeps a lone node alive) — same rule as the C planner."""
    cb = (128 // item_len) * item_len if item_len < 128 else item_len
    chunks = -(-shard_n * item_len // cb)
    return max(1, -(-chunks // (1 << (height - k))))


class ShardedMerklePipeline:
    """The sharded merkleHash of a stream of trees (one tree per ``submit``),
    with everything above each rank's leaf pass moved off the rank's main
    stream.

    Per tree, on the caller's current stream: the leaf pass of this rank's
    shard (``frontier_fn`` to the level ``leaf_levels`` above the chunks, the
    levels one k_reduce leaf pass folds).  On a side stream, overlapping the
    next tree's leaf pass: the shard's node passes from that level to its
    frontier ``gather_log2`` levels below the shard root
    (``node_frontier_fn``), the all-gather of the frontiers (RCCL on the side
    stream) and, on rank 0, the finisher (``finish_nodes_fn``).  The split
    levels are the ones ``sharded_merkle_hash`` computes in one piece, so the
    root is the same.  Buffers rotate over ``slots`` sets: a submit waits for
    the side-stream work of the tree submitted ``slots`` calls earlier; a
    returned root (rank 0; None elsewhere) stays valid for the next
    ``slots - 1`` submits.  Three sets, not two: side work dispatched while a
    leaf pass fills every CU only gets workgroup slots in that pass's tail,
    so with two sets the next leaf pass often waited for it (one-GPU probe of
    the 8-GPU rank step, 2^25 items: 0.09-0.11 ms over the leaf pass with
    two sets, 0.05 with three; tools/rank_step_probe.py,
    profiles/r02k/rank_step_slots.jsonl).  Every rank must
    submit the same sequence of trees (one collective per tree).

    ``ok`` is False when the shard is too small to split (fewer than
    ``leaf_levels + gather_log2 + 1`` levels): use ``sharded_merkle_hash``.
    The compute steps are injectable as in ``sharded_merkle_hash``."""

    def __init__(self, n_total: int, item_len: int, sp: ShardPlan, rank: int, world: int, device,
                 gather_log2: int = 10, leaf_levels: int = 5, group=None,
                 frontier_fn: Optional[Callable] = None, node_frontier_fn: Optional[Callable] = None,
                 finish_nodes_fn: Optional[Callable] = None, workspace=None, slots: int = 3,
                 wait_every: int = 1, timer: Optional[PhaseTimer] = None):
        self.n_total, self.item_len, self.sp = n_total, item_len, sp
        self.timer = timer
        self.rank, self.world, self.group = rank, world, group
        self.device = torch.device(device)
        h = sp.height
        lo, hi = sp.items(rank)
        self.sn = hi - lo
        self.k = gather_log2
        self.k_leaf = h - leaf_levels  # the leaf pass's output level, counted down from the shard root
        # the planner's leaf pass folds at least 2 levels (window + pair)
        self.ok = sp.nonempty > 1 and leaf_levels >= 2 and 0 < self.k < self.k_leaf
        if not self.ok:
            return
        self.leaf_count = frontier_count(self.sn, item_len, h, self.k_leaf) if self.sn else 0
        last = sp.nonempty - 1
        self.count = (last << self.k) + frontier_count(sp.begin[last + 1] - sp.begin[last], item_len, h, self.k)
        if frontier_fn is None or node_frontier_fn is None or finish_nodes_fn is None:
            from . import _lib
            from . import device as D
            if workspace is None and self.sn:
                workspace = D.subtree_workspace(self.sn, item_len, device)
            nws = torch.empty(max(256, _lib.load().mk_ssz_merkle_node_frontier_workspace_bytes(
                max(self.leaf_count, 1), self.k_leaf, self.k)), dtype=torch.uint8, device=device)
            fws = D.finish_workspace(self.count, device) if rank == 0 else None
            frontier_fn = frontier_fn or (lambda it, sn, il, hh, kk, pad, out: D.merkle_subtree_frontier(
                it, sn, il, hh, kk, pad, out=out, ws=workspace))
            node_frontier_fn = node_frontier_fn or (lambda nodes, cnt, hh, kk, pad, out: D.merkle_node_frontier(
                nodes, cnt, hh, kk, pad, out=out, ws=nws))
            finish_nodes_fn = finish_nodes_fn or (lambda g, c, nt, out: D.merkle_finish_nodes(g, c, nt, out=out,
                                                                                               ws=fws))
        self.frontier_fn, self.node_frontier_fn, self.finish_nodes_fn = frontier_fn, node_frontier_fn, finish_nodes_fn
        block = 32 << self.k
        dev = self.device
        self.slots = max(2, int(slots))
        S = self.slots
        self._ring = SlotRing(S, wait_every)
        self.levels = [torch.empty(32 << self.k_leaf, dtype=torch.uint8, device=dev) for _ in range(S)]
        self.blocks = [torch.zeros(block, dtype=torch.uint8, device=dev) for _ in range(S)]
        self.gathered = [torch.empty(world * block, dtype=torch.uint8, device=dev) for _ in range(S)]
        self.outs = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(S)]
        self.cuda = dev.type == "cuda"
        # high priority = its own hardware queue (see MerklePipeline)
        self.side = torch.cuda.Stream(device=dev, priority=-1) if self.cuda else None

    def submit(self, local_items: torch.Tensor) -> Optional[torch.Tensor]:
        cur = torch.cuda.current_stream(self.device) if self.cuda else None
        slot = self._ring.acquire(cur)  # side work of `slots` trees back is done
        level = None
        t = self.timer
        if t is not None:
            t.mark("leaf0", cur)
        if self.sn:
            level = self.frontier_fn(local_items, self.sn, self.item_len, self.sp.height, self.k_leaf, True,
                                     self.levels[slot])
        if t is not None:
            t.mark("leaf1", cur)
        if self.cuda:
            self.side.wait_stream(cur)
            with torch.cuda.stream(self.side):
                root = self._top(level, slot)
                ev = torch.cuda.Event()
                ev.record(self.side)
            self._ring.release(ev)
            return root
        root = self._top(level, slot)
        self._ring.release(None)
        return root

    def _top(self, level, slot):
        blk = self.blocks[slot]
        t, side = self.timer, (self.side if self.cuda else None)
        if t is not None:
            t.mark("nodes0", side)
        if level is not None:
            fr = self.node_frontier_fn(level, self.leaf_count, self.k_leaf, self.k, True, blk)
            if fr.data_ptr() != blk.data_ptr():  # an injected step may return its own buffer
                blk[:fr.numel()].copy_(fr)
        if t is not None:
            t.mark("nodes1", side)
        # (an empty shard sends its zero block; only the counted nodes are read)
        g = self.gathered[slot]
        if blk.is_cuda and dist.get_backend(self.group) == "gloo":  # one-GPU rehearsal: gloo gathers host tensors
            host = torch.empty(g.numel(), dtype=torch.uint8)
            dist.all_gather_into_tensor(host, blk.cpu(), group=self.group)
            g.copy_(host)
        else:
            dist.all_gather_into_tensor(g, blk, group=self.group)
        if t is not None:
            t.mark("gather1", side)
        if self.rank == 0:
            r = self.finish_nodes_fn(g, self.count, self.n_total, self.outs[slot])
            if t is not None:
                t.mark("finish1", side)
            return r
        return None


# ---------------------------------------------------------------- deposit trie
@dataclass
class TrieShardPlan:
    """Subtree split of an n-deposit, depth-`depth` trie over `world` ranks
    (SURVEY.md §8e, C5): rank r holds deposits [r·2^height, (r+1)·2^height)
    and builds its height-`height` subtree; nonempty ranks contribute a
    root (an empty shard's node is absent, i.e. 0^32 — the Go map miss of
    deposit_trie.go:35-37).  height == 0 means: too small to shard, rank 0
    builds the whole trie."""
    n: int
    depth: int
    height: int
    nonempty: int

    def items(self, rank: int):
        if self.height == 0:
            return (0, self.n) if rank == 0 else (self.n, self.n)
        lo = min(self.n, rank << self.height)
        return lo, min(self.n, lo + (1 << self.height))


def trie_plan(n: int, world: int, depth: int = 32) -> TrieShardPlan:
    if world < 1 or n < 0 or n > (1 << depth):
        raise ValueError("bad trie shard plan arguments")
    h = 0
    while (1 << h) * world < n:
        h += 1
    ne = -(-n // (1 << h)) if n else 0
    if h == 0 or ne <= 1 or h >= depth:
        return TrieShardPlan(n, depth, 0, 1 if n else 0)
    return TrieShardPlan(n, depth, h, ne)


def deposit_subtree_root(data: torch.Tensor, count: int, deposit_len: int, height: int,
                         out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Root of one shard: the batch build (deposit_trie.go:29-40) of its
    `count` fixed-length deposits as a depth-`height` trie (the shard's
    subtree of the global trie: same leaf hashes, same 0^32 for absent
    nodes), on the device."""
    from . import device as D

    lv = torch.empty(D.deposit_trie_levels_bytes(count, height), dtype=torch.uint8, device=data.device)
    out = out if out is not None else torch.empty(32, dtype=torch.uint8, device=data.device)
    D.deposit_trie_build(lv, count, data, count, deposit_len, height, height, out)
    return out


def deposit_trie_top(roots: torch.Tensor, nonempty: int, world: int, levels_above: int,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The trie above the shards: the `nonempty` gathered shard roots are
    level 0 of a depth-`levels_above` trie (absent right children 0^32, then
    the zero-sibling levels up to the full depth), on the device."""
    from . import device as D

    lv = torch.zeros(D.deposit_trie_levels_bytes(world, levels_above), dtype=torch.uint8, device=roots.device)
    lv[:32 * nonempty] = roots[:32 * nonempty]
    out = out if out is not None else torch.empty(32, dtype=torch.uint8, device=roots.device)
    D.deposit_trie_levels(lv, world, nonempty, 0, levels_above, levels_above, out)
    return out


def sharded_deposit_trie_root(local_data: torch.Tensor, deposit_len: int, tp: TrieShardPlan, rank: int,
                              world: int, group=None, subtree_fn: Optional[Callable] = None,
                              top_fn: Optional[Callable] = None,
                              full_fn: Optional[Callable] = None) -> Optional[torch.Tensor]:
    """Root of the deposit trie of tp.n fixed-length deposits sharded by
    subtree over the ranks ("Deposit trie (C5): same split
    with a 32-B zero pad, plus the zero-sibling levels on GPU 0"): every
    rank builds its subtree with no communication, one all-gather of 32 B
    per rank, rank 0 builds the levels above.  Returns the root on rank 0,
    None elsewhere.  The compute steps are injectable (CPU tests, gloo)."""
    subtree_fn = subtree_fn or deposit_subtree_root
    top_fn = top_fn or deposit_trie_top
    lo, hi = tp.items(rank)
    dev = local_data.device
    if tp.height == 0:  # too small to shard: rank 0 builds it all
        if rank != 0:
            return None
        if full_fn is None:
            def full_fn(d, cnt, ln, depth):
                if cnt == 0:
                    return torch.zeros(32, dtype=torch.uint8, device=d.device)
                return deposit_subtree_root(d, cnt, ln, depth)
        return full_fn(local_data, tp.n, deposit_len, tp.depth)
    if hi > lo:
        root = subtree_fn(local_data, hi - lo, deposit_len, tp.height)
    else:
        root = torch.zeros(32, dtype=torch.uint8, device=dev)
    if root.is_cuda and dist.get_backend(group) == "gloo":
        host = torch.empty(32 * world, dtype=torch.uint8)
        dist.all_gather_into_tensor(host, root.cpu(), group=group)
        gathered = host.to(dev)
    else:
        gathered = torch.empty(32 * world, dtype=root.dtype, device=dev)
        dist.all_gather_into_tensor(gathered, root, group=group)
    if rank == 0:
        return top_fn(gathered, tp.nonempty, world, tp.depth - tp.height)
    return None
