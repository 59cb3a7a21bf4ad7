"""End-to-end merkleHash from a HOST buffer (the cgo caller's view): the
library copies the items over PCIe, Merkleizes and returns the root.  Reports
host->device GB/s and the whole-call time next to the device-resident time
(this is never the bench.py value).  Second argument "tree":
the same for TreeHash([][32]byte) (mk_ssz_tree_hash_bytes_list)."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from prysm_amd import device as D
    from prysm_amd import ssz as S

    log2n = int(sys.argv[1]) if len(sys.argv) > 1 else 26
    tree = len(sys.argv) > 2 and sys.argv[2] == "tree"
    host_fn = (lambda b: S.tree_hash_bytes_list(b, n, 32)) if tree else (lambda b: S.merkle_hash_flat(b, n, 32))
    n = 1 << log2n
    host = np.empty(n * 32, dtype=np.uint8)
    dev = torch.device("cuda:0")
    t = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    D.synth_fill(t, 0x5EED000000000004)
    host[:] = t.cpu().numpy()
    pinned = torch.empty(n * 32, dtype=torch.uint8).pin_memory()
    pinned.copy_(torch.from_numpy(host))
    out = {}
    for name, buf in (("pageable", host), ("pinned", pinned.numpy())):
        host_fn(buf)  # warm (pools, clocks)
        t0 = time.perf_counter()
        root = host_fn(buf)
        out[name + "_ms"] = (time.perf_counter() - t0) * 1e3
        out[name + "_root"] = root.hex()
    ws = D.tree_hash_bytes_list_workspace(n, 32, dev) if tree else D.merkle_workspace(n, 32, dev)
    dev_fn = (lambda: D.tree_hash_bytes_list(t, n, 32, ws=ws)) if tree else (lambda: D.merkle_hash(t, n, 32, ws=ws))
    r = dev_fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        r = dev_fn()
    torch.cuda.synchronize()
    out["device_resident_ms"] = (time.perf_counter() - t0) / 5 * 1e3
    out["device_root"] = bytes(r.cpu().numpy()).hex()
    out["bytes"] = n * 32
    out["pinned_h2d_GBps_effective"] = n * 32 / (out["pinned_ms"] - out["device_resident_ms"]) / 1e6
    out["log2n"] = log2n
    out["path"] = "tree_hash_bytes_list" if tree else "merkle_hash"
    print(json.dumps(out))


if __name__ == "__main__":
    main()
