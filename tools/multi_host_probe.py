"""Host-buffer merkleHash through mk_ssz_merkle_hash_multi on ONE device with
1/2/4/8 shards (the same device listed k times: one upload thread per
listed device, pinned staging, shard passes overlapped with the next
upload), against mk_ssz_merkle_hash (single call, chunked pageable H2D):
wall ms and effective host->device GB/s.  Feeds DESIGN §6's expected
multi-device end-to-end time.

  python tools/multi_host_probe.py [--log2n 26] [--reps 3]
"""
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
    ap.add_argument("--log2n", type=int, default=26)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np

    from prysm_amd import _lib

    if os.environ.get("PRYSM_MERKLE_VARIANT"):  # A/B: a variant build of the library
        _lib.LIB_PATH = os.path.join(ROOT, "prysm_amd", "lib", "variants",
                                     f"libprysm_merkle_{os.environ['PRYSM_MERKLE_VARIANT']}.so")
    _lib.init(0)
    n, il = 1 << a.log2n, 32
    items = np.random.default_rng(7).integers(0, 256, n * il, dtype=np.uint8)
    out = ctypes.create_string_buffer(32)
    p = items.ctypes.data_as(ctypes.c_void_p)
    gb = n * il / 1e9
    roots = set()

    def single():
        _lib.invoke("mk_ssz_merkle_hash", p, n, il, out)

    def multi(k):
        arr = (ctypes.c_int * k)(*([0] * k))
        return lambda: _lib.invoke("mk_ssz_merkle_hash_multi", p, n, il, k, arr, out)

    for name, fn in [("single_call", single)] + [(f"multi_{k}_shards", multi(k)) for k in (1, 2, 4, 8)]:
        fn()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        ms = (time.perf_counter() - t0) / a.reps * 1e3
        roots.add(out.raw)
        print(json.dumps({"lib": os.environ.get("PRYSM_MERKLE_VARIANT", "main"), "path": name, "n": n, "GB": gb, "ms": ms, "GBps": gb / ms * 1e3}), flush=True)
    assert len(roots) == 1, "paths disagree"


if __name__ == "__main__":
    main()
