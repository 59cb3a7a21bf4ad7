"""A/B of the N=1 pipelined headline step (MerklePipeline) with its side
stream at default vs high priority, plus the one-stream merkleHash, in ONE
process with interleaved rounds on the same 2^log2n x 32-B items.  The
rocprofv3 trace of bench.py showed the default-priority side stream on the
current stream's hardware queue (node passes serialised behind the leaf
pass); a high-priority stream gets its own queue.

  python tools/pipe_prio_ab.py [--log2n 28] [--rounds 5] [--steps 10]
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=28)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd.pipeline import MerklePipeline

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    _lib.init(0)
    n, il = 1 << a.log2n, 32
    items = torch.empty(n * il, dtype=torch.uint8, device=dev)
    D.synth_fill(items, 0x5EED000000000004)
    pipe = MerklePipeline(n, il, dev)
    sides = {"pipe_lo": torch.cuda.Stream(device=dev), "pipe_hi": torch.cuda.Stream(device=dev, priority=-1)}
    ws = D.merkle_workspace(n, il, dev)
    one_out = torch.empty(32, dtype=torch.uint8, device=dev)
    kinds = ["one", "pipe_lo", "pipe_hi"]
    times = {k: [] for k in kinds}
    roots = {}
    for r in range(a.rounds + 1):
        for k in kinds:
            torch.cuda.synchronize()
            if k != "one":
                pipe.side = sides[k]
                pipe._done = [None, None]
            step = (lambda: D.merkle_hash(items, n, il, out=one_out, ws=ws)) if k == "one" else \
                (lambda: pipe.submit(items))
            step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                out = step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps * 1e3
            roots[k] = bytes(out.cpu().numpy()).hex()
            if r:
                times[k].append(dt)
    assert len(set(roots.values())) == 1, roots
    for k in kinds:
        print(json.dumps({"variant": k, "log2n": a.log2n, "median_ms": statistics.median(times[k]),
                          "min_ms": min(times[k]), "leaves_per_s": n / statistics.median(times[k]) * 1e3}))
    print(json.dumps({"root": roots["one"]}))


if __name__ == "__main__":
    main()
