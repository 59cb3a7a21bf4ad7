"""Generates tests/golden/full_size_roots.json: the CPU oracle's results for
the BASELINE.json configurations at their full sizes, on the same seeded
synthetic inputs bench.py / tools/bench_configs.py use, so the GPU tests can
check the device path bit-exactly at full size (restatement-derived, like
restatement_vectors.json; the oracle is pinned by reference_vectors.json).

  c1: TreeHash([]*ValidatorRecord) of 16,384 synthetic validators (C struct
      roots + merkleHash, cross-checked against the reflective ssz_ref walk)
  c2: hashutil.Hash of 2^24 x 64-B SplitMix64 messages -> Keccak-256 of the
      concatenated 2^24 digests and merkleHash of the digests as 32-B items
      (checksums of checksums)
  c3: TreeHash of State{1,000,000 synthetic validators, balances}
  c4: merkleHash of 2^28 x 32-B SplitMix64 items (the headline tree)
  c4tree: TreeHash([][32]byte) of 2^28 SplitMix64 elements (the C4 secondary:
      every element hashed as Keccak(le32(32) || element), then merkleHash)
  c5: depth-32 deposit trie root of 2^20 x 280-B SplitMix64 deposits
  c3_state: TreeHash of the synthetic pb.BeaconState of prysm_amd/state.py
      with 1,000,000 validators (oracle/ssz_ref.py's reflective restatement,
      the registry root from the C oracle's struct roots + merkleHash)

Run:  python tests/golden/make_full_size.py [c1,c2,c3,c3_state,c4,c4tree,c5]
(C oracle, all host cores; about a minute on 8 cores; named configs are
recomputed and merged into the existing file).
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


def c3_state(nt):
    from oracle import ssz_ref as OS
    from prysm_amd import registry as R
    from prysm_amd import state as ST
    from tests.ssz_types import to_ref_type

    n, seed = 1_000_000, SEED + 3
    st = ST.synthetic_state(n, seed)
    roots = O.struct_roots(st.registry.records.view(np.uint8).reshape(-1), n, 160, R.VALIDATOR_FIELDS, nthreads=nt)
    reg_root = O.merkle_hash_flat(roots.reshape(-1), n, 32, nthreads=nt)
    small = ST.synthetic_state(0, seed)  # everything but the 1M-entry lists, as a reflective value
    small.balances = st.balances
    small.attestations, small.scalars = st.attestations, st.scalars
    for f in ("randao_mixes", "seeds", "crosslink_epochs", "crosslink_roots", "latest_block_roots",
              "batched_block_roots", "penalized_balances", "index_roots", "eth1_data", "eth1_votes",
              "eth1_vote_counts", "fork"):
        setattr(small, f, getattr(st, f))
    val = small.as_value()
    val["ValidatorRegistry"] = "precomputed"
    t = to_ref_type(ST.STATE_SSZ)
    fields = [(name, ("hashable", "ValidatorRegistry", lambda _v: reg_root) if name == "ValidatorRegistry" else ft)
              for name, ft in t[2]]
    root = OS.tree_hash(("struct", t[1], fields), val)
    return {"n": n, "seed": seed, "registry_root": reg_root.hex(), "state_root": root.hex(),
            "shape": "prysm_amd/state.py synthetic_state defaults (8192-entry arrays, 1024 crosslinks, "
                     "128 attestations, 16 batched roots, 4 eth1 votes)"}


def main(only=None):
    nt = os.cpu_count() or 1
    path = os.path.join(HERE, "full_size_roots.json")
    out = {"_generated_by": "tests/golden/make_full_size.py", "_oracle": "oracle/*.c (CPU restatement)"}
    if only and os.path.exists(path):
        with open(path) as f:
            out = json.load(f)
    want = lambda c: not only or c in only  # noqa: E731
    t0 = time.time()

    if want("c1"):
        # BASELINE config 1: ssz.TreeHash([]*ValidatorRecord) of 16,384
        # synthetic validators (bench_configs.py c1's seeded registry).  Two
        # independent oracle paths must agree: the C struct roots + merkleHash
        # and the reflective type walk of ssz/hash.go:118-159 (ssz_ref.py).
        from oracle import ssz_ref as OS
        from prysm_amd import registry as R

        n = 16_384
        reg = R.synthetic_registry(n, SEED + 1)
        roots = O.struct_roots(reg.records.view(np.uint8).reshape(-1), n, 160, R.VALIDATOR_FIELDS, nthreads=nt)
        root = O.merkle_hash_flat(roots.reshape(-1), n, 32, nthreads=nt)
        t_ref = ("slice", ("ptr", ("struct", "ssz.ValidatorRecord",
                                   [("Pubkey", ("bytes",)), ("WithdrawalCredentialsHash32", ("bytes",)),
                                    ("RandaoCommitmentHash32", ("bytes",))] +
                                   [(f, ("uint", 64)) for f in ("RandaoLayers", "ActivationEpoch", "ExitEpoch",
                                                                "WithdrawalEpoch", "PenalizedEpoch", "StatusFlags")])))
        refl = OS.tree_hash(t_ref, reg.as_dicts())
        assert refl == root, "c1: reflective restatement and C struct path disagree"
        out["c1"] = {"n": n, "seed": SEED + 1, "root": root.hex(),
                     "generator": "registry.synthetic_registry(16384, seed) (SplitMix64 stream)",
                     "checked": "C oracle struct roots + merkleHash == reflective ssz_ref.tree_hash"}

    if want("c2"):
        n = 1 << 24
        msgs = O.splitmix_bytes(n * 64, SEED + 2)
        dig = O.keccak256_batch(msgs, 64, nthreads=nt)
        # two checksums of the 2^24 digests: Keccak of their concatenation, and
        # merkleHash of them as 32-B items (what bench.py checks on the device)
        out["c2"] = {"n": n, "msg_len": 64, "seed": SEED + 2, "digest_of_digests": O.keccak256(dig.tobytes()).hex(),
                     "merkle_of_digests": O.merkle_hash_flat(dig.reshape(-1), n, 32, nthreads=nt).hex()}
        del msgs, dig

    if want("c3"):
        from prysm_amd import registry as R

        n = 1_000_000
        reg = R.synthetic_registry(n, SEED + 3)
        bal = R.synthetic_balances(n, SEED + 3)
        roots = O.struct_roots(reg.records.view(np.uint8).reshape(-1), n, 160, R.VALIDATOR_FIELDS, nthreads=nt)
        reg_root = O.merkle_hash_flat(roots.reshape(-1), n, 32, nthreads=nt)
        bal_root = O.merkle_hash_flat(bal.view(np.uint8), n, 8, nthreads=nt)
        out["c3"] = {"n": n, "seed": SEED + 3, "registry_root": reg_root.hex(), "balances_root": bal_root.hex(),
                     "state_root": O.keccak256(reg_root + bal_root).hex(),
                     "generator": "registry.synthetic_registry / synthetic_balances (SplitMix64 stream)"}

    if want("c3_state"):
        out["c3_state"] = c3_state(nt)

    if want("c4"):
        n = 1 << 28
        out["c4"] = {"n": n, "item_len": 32, "seed": SEED + 4,
                     "root": O.merkle_hash_gen(n, 32, SEED + 4, nthreads=nt).hex()}

    if want("c4tree"):
        # SURVEY 8(d)'s C4 secondary: TreeHash([][32]byte) of 2^28 elements =
        # merkleHash over Keccak(le32(32) || element_i) (hash.go:100-107,118-139);
        # elements generated chunk by chunk from the SplitMix64 stream
        n, L, seed = 1 << 28, 32, SEED + 0x40
        dig = np.empty((n, 32), dtype=np.uint8)
        step = 1 << 24
        for lo in range(0, n, step):
            chunk = O.splitmix_bytes(step * L, seed, word0=lo * L // 8)
            dig[lo:lo + step] = O.elem_digests(chunk, step, L, nthreads=nt)
        out["c4tree"] = {"n": n, "elem_len": L, "seed": seed,
                         "root": O.merkle_hash_flat(dig.reshape(-1), n, 32, nthreads=nt).hex(),
                         "what": "ssz.TreeHash([][32]byte): merkleHash over Keccak(le32(32) || element)"}
        del dig

    if want("c5"):
        n, dl = 1 << 20, 280
        host = O.splitmix_bytes(n * dl, SEED + 5)
        deps = [host[i * dl:(i + 1) * dl].tobytes() for i in range(n)]
        root, _ = O.deposit_trie_levels(deps)
        out["c5"] = {"n": n, "deposit_len": dl, "seed": SEED + 5, "depth": 32, "root": bytes(root).hex()}

    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")
    print(f"wrote full_size_roots.json in {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main(sys.argv[1].split(",") if len(sys.argv) > 1 else None)
