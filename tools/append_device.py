"""Device-side latency of one UpdateDepositTrie + Root() (powchain's one log
at a time, powchain/service.go:379-386): mk_dev_deposit_trie_append of ONE
280-B deposit onto a device-resident trie of `--prefill` deposits, the root
written on the device; `--appends` back-to-back calls on one stream, wall
time per call (every root checked against the oracle's batch restatement at
the end: the trie's levels are compared after the run).

  python tools/append_device.py [--prefill 65536] [--appends 400]"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prefill", type=int, default=1 << 16)
    ap.add_argument("--appends", type=int, default=400)
    a = ap.parse_args()
    import torch

    from oracle import oracle as O
    from prysm_amd import _lib
    from prysm_amd import device as D

    L = _lib.load()
    dev = torch.device("cuda:0")
    dl, depth = 280, 32
    total = a.prefill + a.appends + 20
    host = O.splitmix_bytes(total * dl, 0x5EED000000000005)
    data = torch.from_numpy(host.copy()).to(dev)
    lv = torch.zeros(D.deposit_trie_levels_bytes(total, depth), dtype=torch.uint8, device=dev)
    root = torch.zeros(32, dtype=torch.uint8, device=dev)
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    def app(count, k):
        _lib.check(L.mk_dev_deposit_trie_append(None, P(lv), total, count, P(data[count * dl:]), None, k, dl,
                                                 depth, P(root), st()), "append")

    app(0, a.prefill)
    count = a.prefill
    for _ in range(20):  # warm-up
        app(count, 1)
        count += 1
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.appends):
        app(count, 1)
        count += 1
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / a.appends * 1e6
    want = O.deposit_trie_levels([bytes(host[i * dl:(i + 1) * dl]) for i in range(count)])[0]
    ok = bytes(root.cpu().numpy()) == want
    print(json.dumps({"appends": a.appends, "count_at_start": a.prefill, "us_per_append_and_root": round(us, 2),
                      "root_ok": ok}))
    if not ok:
        raise SystemExit("root mismatch")


if __name__ == "__main__":
    main()
