"""Expected outputs of tests/c_abi/harness.c's inputs, computed with the CPU
oracle (test infrastructure).  Writes tests/golden/c_abi_fixture.json.

  python tests/golden/make_c_abi_fixture.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

SEED_BASE = 0x5EED000000000700


def main():
    merkle, batch = [], []
    for t in range(8):
        n = 100003 + t
        merkle.append(O.merkle_hash_flat(O.splitmix_bytes(n * 32, SEED_BASE + t), n, 32).hex())
        msgs = O.splitmix_bytes(1000 * 64, SEED_BASE + 0x100 + t)
        batch.append(O.keccak256(O.keccak256_batch(msgs, 64).tobytes()).hex())
    deps = [bytes(O.splitmix_bytes(280, SEED_BASE + 0x200, 35 * i)) for i in range(300)]
    tr = O.DictTrie()
    for d in deps:
        tr.update(d)
    branch = O.keccak256(b"".join(tr.branch(7))).hex()
    buf = O.splitmix_bytes(160 + 8000, SEED_BASE + 0x300)
    many = [O.merkle_hash_flat(buf[:160], 5, 32).hex(), O.merkle_hash_flat(buf[160:], 1000, 8).hex(),
            O.merkle_hash_flat(buf[:0], 0, 32).hex()]
    out = {"merkle": merkle, "batch": batch, "trie_root": tr.root().hex(), "branch": branch, "many": many,
           "note": "expected outputs of tests/c_abi/harness.c (CPU oracle); inputs are SplitMix64 streams"}
    with open(os.path.join(ROOT, "tests", "golden", "c_abi_fixture.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
