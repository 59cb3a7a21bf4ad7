"""A/B of how the C3 step (TreeHash of a 1M-validator State) places its two
independent trees on streams, in ONE process, interleaved rounds.  The rocprofv3
trace of the bench step showed the balances tree (side stream) and the
registry's struct kernel (current stream) on the same hardware queue, i.e.
serialised.  Variants:

  serial      everything on the current stream
  side_first  balances on a side stream launched first (bench.py today)
  side_after  struct kernel first, balances on the side stream after it
  hi_first    side_first with a high-priority side stream
  hi_after    side_after with a high-priority side stream
  hi_split    struct roots on the current stream; then the balances tree on a
              high-priority side stream beside the registry merkleHash (the
              latency-bound top leaves CUs idle that the balances can use)

  python tools/c3_streams.py [--rounds 5] [--steps 20]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd import registry as R

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    _lib.init(0)
    L = _lib.load()
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    n = 1_000_000
    reg = R.synthetic_registry(n, 0x5EED000000000003)
    bal = R.synthetic_balances(n, 0x5EED000000000003)
    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(dev)
    dbal = torch.from_numpy(bal.view(np.uint8).copy()).to(dev)
    spec = R._fields(R.VALIDATOR_FIELDS)
    nf = len(R.VALIDATOR_FIELDS)
    ws = torch.empty(L.mk_ssz_struct_list_workspace_bytes(n, spec, nf) + 4096, dtype=torch.uint8, device=dev)
    bws = D.merkle_workspace(n, 8, dev)
    roots = torch.empty(64, dtype=torch.uint8, device=dev)
    out = torch.empty(32, dtype=torch.uint8, device=dev)
    lo = torch.cuda.Stream(device=dev)
    hi = torch.cuda.Stream(device=dev, priority=-1)

    def registry(cur):
        _lib.check(L.mk_dev_ssz_struct_list_root(None, P(rec), n, 160, spec, nf, P(roots), P(ws), ws.numel(),
                                                 ctypes.c_void_p(cur.cuda_stream)), "registry")

    sroots = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    sws = torch.empty(n * 144 + 256, dtype=torch.uint8, device=dev)
    mws = D.merkle_workspace(n, 32, dev)

    def split(cur, side):
        D.struct_roots(rec, n, 160, R.VALIDATOR_FIELDS, out=sroots, ws=sws)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            balances()
        D.merkle_hash(sroots, n, 32, out=roots[:32], ws=mws)

    def balances():
        D.merkle_hash(dbal, n, 8, out=roots[32:], ws=bws)

    def final(cur):
        _lib.check(L.mk_dev_hash_batch(None, P(roots), 1, 64, P(out), ctypes.c_void_p(cur.cuda_stream)), "state")

    def make(kind):
        side = hi if kind.startswith("hi") else lo

        def step():
            cur = torch.cuda.current_stream(dev)
            if kind == "serial":
                registry(cur)
                balances()
            elif kind.endswith("_split"):
                split(cur, side)
            elif kind.endswith("first"):
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    balances()
                registry(cur)
            else:
                side.wait_stream(cur)
                registry(cur)
                with torch.cuda.stream(side):
                    balances()
            if kind != "serial":
                cur.wait_stream(side)
            final(cur)
        return step

    kinds = ["serial", "hi_first", "hi_split", "lo_split"]
    steps = {k: make(k) for k in kinds}
    times = {k: [] for k in kinds}
    want = R.state_root(reg, bal)
    for r in range(a.rounds + 1):
        for k in kinds:
            for _ in range(3):
                steps[k]()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                steps[k]()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps * 1e3
            assert bytes(out.cpu().numpy()) == want, k
            if r:
                times[k].append(dt)
    for k in kinds:
        print(json.dumps({"variant": k, "median_ms": statistics.median(times[k]), "min_ms": min(times[k])}))


if __name__ == "__main__":
    main()
