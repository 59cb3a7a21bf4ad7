"""TreeHash of a whole synthetic pb.BeaconState (SURVEY.md §8f row 4,
prysm_amd/state.py: 7 library calls from host arrays, the Go caller's form)
at 1,000,000 validators: wall time per state root, with the share of the
registry's host-buffer call (records cross PCIe) beside it.  One JSON line.

  python tools/bench_state.py [--n 1000000] [--steps 5] [--warmup 2]
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
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    a = ap.parse_args()
    from prysm_amd import _lib
    from prysm_amd import state as ST

    _lib.init(0)
    st = ST.synthetic_state(a.n, 0x5EED000000000000 + 77)
    for _ in range(a.warmup):
        root = st.tree_hash_ssz()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        assert st.tree_hash_ssz() == root
    sec = (time.perf_counter() - t0) / a.steps
    t0 = time.perf_counter()
    for _ in range(a.steps):
        st.registry.tree_hash_ssz()
    reg = (time.perf_counter() - t0) / a.steps
    rec_mb = st.registry.records.nbytes / 1e6
    print(json.dumps({"metric": "BeaconState TreeHash (host arrays)", "n_validators": a.n, "ms_per_state": sec * 1e3,
                      "registry_call_ms": reg * 1e3, "registry_records_MB": rec_mb,
                      "registry_h2d_GBps_effective": rec_mb / 1e3 / reg, "root": root.hex(),
                      "steps": a.steps, "warmup": a.warmup}))


if __name__ == "__main__":
    main()
