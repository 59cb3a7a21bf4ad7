"""One rank's pipelined C4 step at N GPUs, emulated on one GPU without the
collective: does the side-stream work (node passes to the 1024-node
frontier, and rank 0's finisher over N x 1024 nodes) hide under the next
leaf pass, or does the double-buffer wait stall the main stream?

Per step, as parallel.ShardedMerklePipeline does it: main stream = the
shard's leaf pass (frontier at the leaf pass's output level); side stream
(high priority) = node passes to the 2^10-node frontier, an N-fold copy of
that block standing in for the all-gather, the finisher.  A submit waits for
the side work of the step two back.  Prints ms/step pipelined, ms of the leaf
pass alone (same launches, no side work), and their difference.

  PRYSM_MERKLE_LIB=<lib> python tools/rank_step_probe.py [--log2n 25] [--world 8]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=25)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--slots", type=int, default=2, help="buffer sets (a submit waits for the side work this many back)")
    a = ap.parse_args()
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd import parallel as P

    dev = torch.device("cuda:0")
    n, il, k = 1 << a.log2n, 32, 10
    h = (n * il // 128 - 1).bit_length()  # the shard's chunk height
    k_leaf = h - 5
    items = torch.empty(n * il, dtype=torch.uint8, device=dev)
    D.synth_fill(items, 0x5EED000000000004)
    ws = D.subtree_workspace(n, il, dev)
    leaf_count = P.frontier_count(n, il, h, k_leaf)
    nws = torch.empty(max(256, _lib.load().mk_ssz_merkle_node_frontier_workspace_bytes(leaf_count, k_leaf, k)),
                      dtype=torch.uint8, device=dev)
    count = a.world << k
    fws = D.finish_workspace(count, dev)
    S = a.slots
    levels = [torch.empty(32 << k_leaf, dtype=torch.uint8, device=dev) for _ in range(S)]
    blocks = [torch.empty(32 << k, dtype=torch.uint8, device=dev) for _ in range(S)]
    gathered = [torch.empty(count * 32, dtype=torch.uint8, device=dev) for _ in range(S)]
    outs = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(S)]
    side = torch.cuda.Stream(device=dev, priority=-1)
    cur = torch.cuda.current_stream(dev)
    done = [None] * S

    def step(i, with_side=True):
        s = i % S
        if done[s] is not None:
            cur.wait_event(done[s])
        lv = D.merkle_subtree_frontier(items, n, il, h, k_leaf, True, out=levels[s], ws=ws)
        if not with_side:
            return
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            D.merkle_node_frontier(lv, leaf_count, k_leaf, k, True, out=blocks[s], ws=nws)
            gathered[s].view(a.world, -1).copy_(blocks[s].view(1, -1).expand(a.world, -1))
            D.merkle_finish_nodes(gathered[s], count, n * a.world, out=outs[s], ws=fws)
            ev = torch.cuda.Event()
            ev.record(side)
        done[s] = ev

    res = {"lib": os.path.basename(os.environ.get("PRYSM_MERKLE_LIB") or "main"), "log2n": a.log2n,
           "world": a.world, "slots": S}
    for mode in ("leaf_only", "pipelined", "leaf_only", "pipelined"):
        done[:] = [None] * S
        for i in range(a.warmup):
            step(i, mode == "pipelined")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i, mode == "pipelined")
        torch.cuda.synchronize()
        res.setdefault(mode + "_ms", []).append((time.perf_counter() - t0) / a.steps * 1e3)
    res = {k2: (min(v) if isinstance(v, list) else v) for k2, v in res.items()}
    res["side_cost_ms"] = res["pipelined_ms"] - res["leaf_only_ms"]
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
