"""Expected outputs of tests/c_abi/harness.c's inputs, computed with the CPU
oracle (test infrastructure).  Writes tests/golden/c_abi_fixture.json.

  python tests/golden/make_c_abi_fixture.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

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
    # `harness cgo`: the reference's own vectors where they exist (copied from
    # reference_vectors.json, each checked against the oracle here), the oracle
    # for the shapes no reference vector covers
    with open(os.path.join(ROOT, "tests", "golden", "reference_vectors.json")) as f:
        ref = json.load(f)
    mh = {v["ref"]: v["output"] for v in ref["merkle_hash"]}
    th = {v["ref"]: v["output"] for v in ref["tree_hash"]}
    cgo = {
        "m0": mh["shared/ssz/hash_test.go:152"],
        "m1": th["shared/ssz/hash_test.go:81"],  # TreeHash([]uint16{1}) = merkleHash([le16(1)])
        "m2": mh["shared/ssz/hash_test.go:153"],
        "m5": O.merkle_hash_flat(O.splitmix_bytes(5 * 32, SEED_BASE + 0x400), 5, 32).hex(),
        "m10x16": mh["shared/ssz/hash_test.go:154-165"],
        "m10x32": mh["shared/ssz/hash_test.go:166-177"],
        "t0": th["shared/ssz/hash_test.go:80"],  # TreeHash of an empty slice = merkleHash([])
        "tz4": O.tree_hash_bytes_list(np.zeros(0, dtype=np.uint8), 4, 0).hex(),
        "t1x6": O.tree_hash_bytes_list(np.arange(1, 7, dtype=np.uint8), 1, 6).hex(),
    }
    assert cgo["m0"] == O.merkle_hash([]).hex() and cgo["m1"] == O.merkle_hash([b"\x01\x00"]).hex()
    assert cgo["m2"] == O.merkle_hash([b"\x01\x02", b"\x03\x04"]).hex() and cgo["t0"] == cgo["m0"]
    assert cgo["m10x16"] == O.merkle_hash([bytes([i]) * 16 for i in range(1, 11)]).hex()
    assert cgo["m10x32"] == O.merkle_hash([bytes([i]) * 32 for i in range(1, 11)]).hex()
    out = {"merkle": merkle, "batch": batch, "trie_root": tr.root().hex(), "branch": branch, "many": many,
           "cgo": cgo,
           "note": "expected outputs of tests/c_abi/harness.c (CPU oracle); inputs are SplitMix64 streams"}
    with open(os.path.join(ROOT, "tests", "golden", "c_abi_fixture.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
