"""Eager launches vs one HIP-graph replay (torch.cuda.graph) for the
latency-bound device-resident calls: per-call wall time, steady state, in
one process.  The graph removes the per-launch host cost (Python + ctypes +
hipLaunchKernel) and lets the device run the launches back to back.

  python tools/graph_probe.py [--iters 200]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters, warm=30):
    import torch

    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    a = ap.parse_args()
    import numpy as np
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd import registry as R

    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    cases = {}

    n = 16_384  # C1 shape, records resident
    reg = R.synthetic_registry(n, 0x5EED000000000001)
    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(dev)
    f = R._fields(R.VALIDATOR_FIELDS)
    sws = torch.empty(_lib.load().mk_ssz_struct_list_workspace_bytes(n, f, len(R.VALIDATOR_FIELDS)) + 256,
                      dtype=torch.uint8, device=dev)
    sout = torch.empty(32, dtype=torch.uint8, device=dev)
    cases["c1_struct_list_root_16k"] = lambda: D.struct_list_root(rec, n, 160, R.VALIDATOR_FIELDS, out=sout, ws=sws)

    ln, depth, cap = 280, 32, 1 << 20
    data = torch.empty(cap * ln, dtype=torch.uint8, device=dev)
    D.synth_fill(data, 0x5EED000000000005)
    lv = torch.empty(D.deposit_trie_levels_bytes(cap, depth), dtype=torch.uint8, device=dev)
    root = torch.empty(32, dtype=torch.uint8, device=dev)
    cases["c5_trie_build_2^20"] = lambda: D.deposit_trie_append(lv, cap, 0, data, cap, ln, depth, root)
    lv2 = torch.empty_like(lv)
    D.deposit_trie_append(lv2, cap, 0, data, cap - 1, ln, depth, root)
    cases["append_1_at_2^20"] = lambda: D.deposit_trie_append(lv2, cap, cap - 1, data[(cap - 1) * ln:], 1, ln,
                                                              depth, root)
    m = 1 << 20
    items = torch.empty(m * 32, dtype=torch.uint8, device=dev)
    D.synth_fill(items, 0x5EED000000000007)
    mws = D.merkle_workspace(m, 32, dev)
    mout = torch.empty(32, dtype=torch.uint8, device=dev)
    cases["merkle_hash_2^20"] = lambda: D.merkle_hash(items, m, 32, out=mout, ws=mws)

    for name, fn in cases.items():
        fn()
        torch.cuda.synchronize()
        want = None
        eager = timeit(fn, a.iters)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        graph = timeit(g.replay, a.iters)
        print(json.dumps({"case": name, "eager_ms": eager, "graph_ms": graph}), flush=True)
        del want


if __name__ == "__main__":
    main()
