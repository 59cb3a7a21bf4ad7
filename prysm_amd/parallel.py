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

from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist


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
                        finish_nodes_fn: Optional[Callable] = None) -> Optional[torch.Tensor]:
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
    holds world << k nodes."""
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
    if rank == 0:
        if k:
            last = sp.nonempty - 1
            count = (last << k) + frontier_count(sp.begin[last + 1] - sp.begin[last], item_len, sp.height, k)
            fin = lambda: finish_nodes_fn(gather_buf, count, n_total)  # noqa: E731
        else:
            fin = lambda: finish_fn(gather_buf, sp.nonempty, n_total)  # noqa: E731
        if finish_stream is not None:
            finish_stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(finish_stream):
                return fin()
        return fin()
    return None


def frontier_count(shard_n: int, item_len: int, height: int, k: int) -> int:
    """Nodes of a shard `k` levels below its root (>= 1: with pad_at_one the
    odd rule keeps a lone node alive) — same rule as the C planner."""
    cb = (128 // item_len) * item_len if item_len < 128 else item_len
    chunks = -(-shard_n * item_len // cb)
    return max(1, -(-chunks // (1 << (height - k))))
