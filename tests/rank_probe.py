"""Rank body for tests/test_launcher.py (CPU, gloo): bench.launch_ranks runs
this as N ranks; each rank Merkleizes its subtree shard with the oracle as
the injected compute (test infrastructure) through parallel.sharded_merkle_hash
(frontier mode), and rank 0 prints {"world": N, "root": ...}."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oracle import oracle as O  # noqa: E402
from prysm_amd import parallel as P  # noqa: E402
from tests.test_distributed import _plan_cpu  # noqa: E402


def main():
    n, seed, k = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    if world > 1:
        dist.init_process_group("gloo")
    sp = P.plan(n, 32, world, plan_fn=_plan_cpu)
    lo, hi = sp.items(rank)
    local = torch.from_numpy(O.splitmix_bytes(n * 32, seed)[lo * 32:hi * 32].copy())
    if world == 1:
        root = O.merkle_hash_flat(local.numpy(), n, 32)
    else:
        def frontier_fn(items, sn, il, h, kk, pad):
            cnt = P.frontier_count(sn, il, h, kk)
            return torch.frombuffer(bytearray(b"".join(
                O.merkle_subtree_gen(n, il, seed, (rank << kk) + j, h - kk) for j in range(cnt))), dtype=torch.uint8)

        def finish_nodes(g, count, nt):
            level = [bytes(g[32 * i:32 * i + 32].numpy()) for i in range(count)]
            while len(level) > 1:
                if len(level) % 2:
                    level.append(bytes(128))
                level = [O.keccak256(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
            return torch.frombuffer(bytearray(O.keccak256(level[0] + nt.to_bytes(8, "little") + bytes(24))),
                                    dtype=torch.uint8)

        r = P.sharded_merkle_hash(local, n, 32, sp, rank, world, subtree_fn=lambda *a: None,
                                  full_fn=lambda *a: None, finish_fn=lambda *a: None, frontier_log2=k,
                                  frontier_fn=frontier_fn, finish_nodes_fn=finish_nodes)
        root = bytes(r.numpy()) if r is not None else None
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"world": world, "root": root.hex()}), flush=True)


if __name__ == "__main__":
    main()
