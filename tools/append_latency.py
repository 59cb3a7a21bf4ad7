"""powchain's read-Root-then-Update loop (powchain/service.go:379-386) through
the host trie handle (prysm_amd.trieutil.DepositTrie -> mk_deposit_trie_append
+ mk_deposit_trie_root): wall time per Root() read with k new deposits
queued before it (k = 1 is the live caller's shape), against the oracle's C
restatement of the reference's incremental UpdateDepositTrie loop on the
host CPU (1 thread).  One JSON line per k.

  python tools/append_latency.py [--prefill 65536] [--reads 200]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prefill", type=int, default=1 << 16)
    ap.add_argument("--reads", type=int, default=200)
    a = ap.parse_args()
    import numpy as np

    from oracle import oracle as O
    from prysm_amd import _lib
    from prysm_amd import trieutil as T

    _lib.init(0)
    ln = 280
    total = a.prefill + 256 * a.reads
    raw = O.splitmix_bytes(total * ln, 0x5EED000000000005)
    deps = [bytes(raw[i * ln:(i + 1) * ln]) for i in range(total)]
    # CPU: the reference's per-deposit loop (35 permutations per deposit)
    m = 4096
    t0 = time.perf_counter()
    O.deposit_trie_incremental_root(deps[:m])
    cpu_us = (time.perf_counter() - t0) / m * 1e6
    for k in (1, 4, 16, 64, 256):
        t = T.DepositTrie(32, capacity=total)
        for d in deps[:a.prefill]:
            t.update_deposit_trie(d)
        t.root()
        pos = a.prefill
        reads = max(20, a.reads // k) if k > 1 else a.reads
        for _ in range(5):  # warm-up
            for d in deps[pos:pos + k]:
                t.update_deposit_trie(d)
            pos += k
            t.root()
        t0 = time.perf_counter()
        for _ in range(reads):
            for d in deps[pos:pos + k]:
                t.update_deposit_trie(d)
            pos += k
            t.root()
        us = (time.perf_counter() - t0) / reads * 1e6
        print(json.dumps({"deposits_per_root": k, "us_per_root_read": us, "us_per_deposit": us / k,
                          "cpu_incremental_us_per_deposit": cpu_us, "gpu_over_cpu_per_deposit": cpu_us / (us / k),
                          "count_at_start": a.prefill}), flush=True)
    # the same loop with every log's Root() check (saveInTrie) in one call per
    # batch: mk_deposit_trie_save_logs; the expected roots come from a scratch
    # trie read after every deposit
    for k in (1, 16, 256, 1024):
        ref = T.DepositTrie(32, capacity=total)
        t = T.DepositTrie(32, capacity=total)
        for d in deps[:a.prefill]:
            ref.update_deposit_trie(d)
            t.update_deposit_trie(d)
        batches = max(3, min(20, 4096 // k))
        logs = []
        pos = a.prefill
        for _ in range(batches + 2):
            roots = []
            for d in deps[pos:pos + k]:
                roots.append(ref.root())
                ref.update_deposit_trie(d)
            logs.append((deps[pos:pos + k], roots))
            pos += k
        t.root()
        for dd, rr in logs[:2]:  # warm-up
            assert all(t.save_logs(dd, rr))
        t0 = time.perf_counter()
        for dd, rr in logs[2:]:
            assert all(t.save_logs(dd, rr))
        us = (time.perf_counter() - t0) / batches * 1e6
        print(json.dumps({"save_logs_batch": k, "us_per_batch": us, "us_per_log": us / k,
                          "cpu_incremental_us_per_deposit": cpu_us, "gpu_over_cpu_per_log": cpu_us / (us / k)}),
              flush=True)


if __name__ == "__main__":
    main()
