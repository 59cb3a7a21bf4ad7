"""A/B of the pipelines' buffer-set schedules (parallel.SlotRing: `slots`
sets, a main-stream wait every `wait_every` submits) in one process,
interleaved rounds: the C5 stream of 2^20-deposit tries (TriePipeline) and
the one-GPU merkleHash stream (MerklePipeline) at 2^28 and 2^25 items.
Every configuration's last root must equal the first configuration's.

  python tools/ring_ab.py [--rounds 3] [--steps 30]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = [(2, 1), (3, 1), (4, 2), (4, 3)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--only", default="trie,m28,m25")
    a = ap.parse_args()
    import torch

    from prysm_amd import device as D
    from prysm_amd.pipeline import MerklePipeline, TriePipeline

    dev = torch.device("cuda:0")
    work = {}
    if "trie" in a.only:
        n = 1 << 20
        data = torch.empty(n * 280, dtype=torch.uint8, device=dev)
        D.synth_fill(data, 0x5EED000000000005)
        work["trie"] = (data, lambda S, W, nn=n: TriePipeline(nn, 280, 32, dev, slots=S, wait_every=W))
    for tag, lg in (("m28", 28), ("m25", 25)):
        if tag in a.only:
            n = 1 << lg
            items = torch.empty(n * 32, dtype=torch.uint8, device=dev)
            D.synth_fill(items, 0x5EED000000000004)
            work[tag] = (items, (lambda nn: lambda S, W: MerklePipeline(nn, 32, dev, slots=S, wait_every=W))(n))
    res = {}
    roots = {}
    for r in range(a.rounds):
        for tag, (inp, mk) in work.items():
            for S, W in CONFIGS:
                p = mk(S, W)
                for _ in range(a.warmup):
                    p.submit(inp)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.steps):
                    out = p.submit(inp)
                torch.cuda.synchronize()
                res.setdefault((tag, S, W), []).append((time.perf_counter() - t0) / a.steps * 1e3)
                roots.setdefault(tag, set()).add(bytes(out.cpu().numpy()))
                del p
    for tag in work:
        assert len(roots[tag]) == 1, tag
    for (tag, S, W), v in res.items():
        print(json.dumps({"work": tag, "slots": S, "wait_every": W, "median_ms": statistics.median(v),
                          "all_ms": [round(x, 4) for x in v]}), flush=True)


if __name__ == "__main__":
    main()
