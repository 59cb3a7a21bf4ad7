"""One-process A/B of the C3 step's stream schedule (1M-validator State):
  beside: the balances tree on a side stream started with the struct kernel
          (the round-2 bench schedule)
  after:  registry.DeviceStateHasher -- the struct kernel alone, then the
          balances tree beside the registry tree
Interleaved rounds, same inputs; both roots checked against the host path.

  python tools/c3_schedule_ab.py [--rounds 9] [--steps 20]
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
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch

    from prysm_amd import device as D
    from prysm_amd import registry as R

    dev = torch.device("cuda:0")
    n, seed = 1_000_000, 0x5EED000000000003
    reg, bal = R.synthetic_registry(n, seed), R.synthetic_balances(n, seed)
    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(dev)
    dbal = torch.from_numpy(bal.view(np.uint8).copy()).to(dev)
    want = R.state_root(reg, bal)
    after = R.DeviceStateHasher(n, dev)
    # the round-2 schedule, same buffers' shapes
    b = R.DeviceStateHasher(n, dev)

    def beside():
        cur = torch.cuda.current_stream(dev)
        b.side.wait_stream(cur)
        with torch.cuda.stream(b.side):
            D.merkle_hash(dbal, n, 8, out=b.pair[32:], ws=b.bal_ws)
        D.struct_roots(rec, n, 160, R.VALIDATOR_FIELDS, out=b.roots, ws=b.msg_ws)
        D.merkle_hash(b.roots, n, 32, out=b.pair[:32], ws=b.reg_ws)
        cur.wait_stream(b.side)
        D.hash_batch(b.pair, 1, 64, out=b.out)
        return b.out

    fns = {"beside": beside, "after": lambda: after.submit(rec, dbal)}
    for name, fn in fns.items():
        r = fn()
        torch.cuda.synchronize()
        assert bytes(r.cpu().numpy()) == want, name
    times = {k: [] for k in fns}
    for rnd in range(a.rounds + 1):
        for name, fn in fns.items():
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                fn()
            torch.cuda.synchronize()
            if rnd:
                times[name].append((time.perf_counter() - t0) / a.steps * 1e3)
    for name in fns:
        print(json.dumps({"schedule": name, "median_ms": statistics.median(times[name]), "min_ms": min(times[name]),
                          "rounds": a.rounds}))


if __name__ == "__main__":
    main()
