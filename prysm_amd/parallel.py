"""Multi-GPU merkleHash by subtree sharding.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
Each rank Merkleizes its own power-of-two-aligned run of 2^height chunks to a
32-byte subtree root with no data-path communication; the only exchange is
one all-gather of 32 B per rank; rank 0 then runs the reference's level loop
over the gathered roots and the length mix-in (hash.go:225-237).

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
                        finish_stream=None) -> Optional[torch.Tensor]:
    """Returns the 32-byte merkleHash root on rank 0 (None elsewhere).

    ``local_items`` holds this rank's items [begin[rank], begin[rank+1]).
    When the tree is too small to shard (sp.nonempty == 1) rank 0 hashes
    everything and the others contribute nothing.

    ``finish_stream`` (a torch.cuda.Stream, rank 0): run the finisher there so
    it overlaps the caller's next Merkleization instead of delaying it; the
    returned root is then produced on that stream (synchronize before use).
    The next call's all-gather waits for it before reusing ``gather_buf``."""
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
    if hi > lo:
        root = subtree_fn(local_items, hi - lo, item_len, sp.height, True)
    else:
        root = torch.zeros(32, dtype=torch.uint8, device=dev)
    if gather_buf is None:
        gather_buf = torch.empty(world * 32, dtype=torch.uint8, device=dev)
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
        if finish_stream is not None:
            finish_stream.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(finish_stream):
                return finish_fn(gather_buf, sp.nonempty, n_total)
        return finish_fn(gather_buf, sp.nonempty, n_total)
    return None
