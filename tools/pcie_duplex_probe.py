"""Can a host->device copy and a device->host copy of PAGEABLE host memory
run at the same time (two host threads, two streams)?  If so, a chunked
host-buffer Hash batch can overlap its upload with its download.  Prints the
time of H2D alone, D2H alone, both serially and both from two threads.

  python tools/pcie_duplex_probe.py [--mb 1024]
"""
import argparse
import json
import threading
import time


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=1024)
    a = ap.parse_args()
    import numpy as np
    import torch

    dev = torch.device("cuda:0")
    nb = a.mb << 20
    up_src = np.ones(nb, dtype=np.uint8)
    dn_dst = np.empty(nb // 2, dtype=np.uint8)
    up_dst = torch.empty(nb, dtype=torch.uint8, device=dev)
    dn_src = torch.ones(nb // 2, dtype=torch.uint8, device=dev)
    s1, s2 = torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)
    up_t, dn_t = torch.from_numpy(up_src), torch.from_numpy(dn_dst)

    def up():
        with torch.cuda.stream(s1):
            up_dst.copy_(up_t, non_blocking=True)
        s1.synchronize()

    def dn():
        with torch.cuda.stream(s2):
            dn_t.copy_(dn_src, non_blocking=True)
        s2.synchronize()

    def timed(fn, reps=3):
        fn()
        best = 1e9
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            best = min(best, time.perf_counter() - t0)
        return best * 1e3

    def both_threads():
        t = threading.Thread(target=up)
        t.start()
        dn()
        t.join()

    res = {"h2d_MB": a.mb, "d2h_MB": a.mb // 2, "pageable": True,
           "h2d_ms": timed(up), "d2h_ms": timed(dn), "serial_ms": timed(lambda: (up(), dn())),
           "two_threads_ms": timed(both_threads)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
