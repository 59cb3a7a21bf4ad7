"""Per-rank critical path of the sharded C4 run, on one GPU: one shard of
the 8-GPU split (2^25 x 32-B items, height 23) reduced to its 32-B root vs to
its frontier level k below the root, plus the rank-0 finisher over the
gathered level (8 ranks x 2^k nodes).  Median of interleaved rounds, hipEvents
on torch's stream (the library launches there).

  python tools/frontier_ab.py [--log2n 25] [--world 8] [--ks 0,6,8,10]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=25, help="items per shard")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ks", default="0,6,8,10")
    ap.add_argument("--rounds", type=int, default=15)
    a = ap.parse_args()
    import torch

    from prysm_amd import device as D

    dev = torch.device("cuda:0")
    sn, il = 1 << a.log2n, 32
    n_total = sn * a.world
    h, ne, begin = D.shard_plan(n_total, il, a.world)
    assert ne == a.world and begin[1] == sn, (h, ne, begin[:2])
    items = torch.empty(sn * il, dtype=torch.uint8, device=dev)
    D.synth_fill(items, 0x5EED000000000004)
    ws = D.subtree_workspace(sn, il, dev)
    ks = [int(x) for x in a.ks.split(",")]
    outs = {k: torch.empty(32 << k, dtype=torch.uint8, device=dev) for k in ks}
    level = {k: torch.empty(a.world << (k + 5), dtype=torch.uint8, device=dev) for k in ks}
    fws = {k: D.finish_workspace(a.world << k, dev) for k in ks}
    fin = torch.empty(32, dtype=torch.uint8, device=dev)
    t_shard = {k: [] for k in ks}
    t_fin = {k: [] for k in ks}

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    for r in range(a.rounds + 2):
        for k in ks:
            if k == 0:
                ts = timed(lambda: D.merkle_subtree(items, sn, il, h, True, out=outs[0], ws=ws))
                level[0][:32 * a.world] = outs[0].repeat(a.world)
                tf = timed(lambda: D.merkle_finish(level[0], a.world, n_total, out=fin))
            else:
                ts = timed(lambda: D.merkle_subtree_frontier(items, sn, il, h, k, True, out=outs[k], ws=ws))
                level[k][:] = outs[k].repeat(a.world)
                tf = timed(lambda: D.merkle_finish_nodes(level[k], a.world << k, n_total, out=fin, ws=fws[k]))
            if r >= 2:
                t_shard[k].append(ts)
                t_fin[k].append(tf)
    for k in ks:
        print(json.dumps({"k": k, "shard_items_log2": a.log2n, "height": h, "world": a.world,
                          "shard_ms": statistics.median(t_shard[k]), "finish_ms": statistics.median(t_fin[k])}))


if __name__ == "__main__":
    main()
