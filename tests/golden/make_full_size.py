"""Generates tests/golden/full_size_roots.json: the CPU oracle's results for
the BASELINE.json configurations at their full sizes, on the same seeded
synthetic inputs bench.py / tools/bench_configs.py use, so the GPU tests can
check the device path bit-exactly at full size (restatement-derived, like
restatement_vectors.json; the oracle is pinned by reference_vectors.json).

  c2: hashutil.Hash of 2^24 x 64-B SplitMix64 messages -> Keccak-256 of the
      concatenated 2^24 digests (a checksum of checksums)
  c3: TreeHash of State{1,000,000 synthetic validators, balances}
  c4: merkleHash of 2^28 x 32-B SplitMix64 items (the headline tree)
  c5: depth-32 deposit trie root of 2^20 x 280-B SplitMix64 deposits

Run:  python tests/golden/make_full_size.py   (C oracle, all host cores;
about a minute on 8 cores).
"""
from __future__ import annotations

import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from oracle import oracle as O  # noqa: E402

SEED = 0x5EED000000000000  # seed = 0x5EED.. + config id


def main():
    nt = os.cpu_count() or 1
    out = {"_generated_by": "tests/golden/make_full_size.py", "_oracle": "oracle/*.c (CPU restatement)"}
    t0 = time.time()

    n = 1 << 24
    msgs = O.splitmix_bytes(n * 64, SEED + 2)
    dig = O.keccak256_batch(msgs, 64, nthreads=nt)
    out["c2"] = {"n": n, "msg_len": 64, "seed": SEED + 2, "digest_of_digests": O.keccak256(dig.tobytes()).hex()}
    del msgs, dig

    from prysm_amd import registry as R

    n = 1_000_000
    reg = R.synthetic_registry(n, SEED + 3)
    bal = R.synthetic_balances(n, SEED + 3)
    roots = O.struct_roots(reg.records.view(np.uint8).reshape(-1), n, 160, R.VALIDATOR_FIELDS, nthreads=nt)
    reg_root = O.merkle_hash_flat(roots.reshape(-1), n, 32, nthreads=nt)
    bal_root = O.merkle_hash_flat(bal.view(np.uint8), n, 8, nthreads=nt)
    out["c3"] = {"n": n, "seed": SEED + 3, "registry_root": reg_root.hex(), "balances_root": bal_root.hex(),
                 "state_root": O.keccak256(reg_root + bal_root).hex()}

    n = 1 << 28
    out["c4"] = {"n": n, "item_len": 32, "seed": SEED + 4,
                 "root": O.merkle_hash_gen(n, 32, SEED + 4, nthreads=nt).hex()}

    n, dl = 1 << 20, 280
    host = O.splitmix_bytes(n * dl, SEED + 5)
    deps = [host[i * dl:(i + 1) * dl].tobytes() for i in range(n)]
    root, _ = O.deposit_trie_levels(deps)
    out["c5"] = {"n": n, "deposit_len": dl, "seed": SEED + 5, "depth": 32, "root": bytes(root).hex()}

    with open(os.path.join(HERE, "full_size_roots.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote full_size_roots.json in {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
