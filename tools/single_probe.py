"""The latency forms of the side configs, alone, for a kernel trace: C5 one
whole trie (mk_dev_deposit_trie_append on an empty trie), C3 one state
(registry.DeviceStateHasher "level1"), C1 device-resident (struct_list_root).
Each is run --steps times back to back after --warmup, wall-clock timed, root
checked against tests/golden/full_size_roots.json.  Under rocprofv3
--kernel-trace, `python tools/trace_tail.py TRACE K` shows the last step.

  python tools/single_probe.py c5 c3 c1 [--steps 100 --warmup 20]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="+")
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    a = ap.parse_args()
    import torch

    import bench_configs as B
    from prysm_amd import device as D
    from prysm_amd import registry as R

    dev = torch.device("cuda:0")
    _lib, L, st, P = B._lib_handles()
    for c in a.configs:
        g = B.golden(c)
        if c == "c5":
            n, dl, depth = g["n"], g["deposit_len"], g["depth"]
            data = torch.empty(n * dl, dtype=torch.uint8, device=dev)
            D.synth_fill(data, g["seed"])
            lv = torch.empty(L.mk_deposit_trie_levels_bytes(n, depth), dtype=torch.uint8, device=dev)
            out = torch.empty(32, dtype=torch.uint8, device=dev)
            fn = lambda: _lib.check(L.mk_dev_deposit_trie_append(None, P(lv), n, 0, P(data), None, n, dl, depth,  # noqa
                                                                  P(out), st()), "c5")
            want = g["root"]
        elif c == "c3":
            n = g["n"]
            rec = R.synthetic_registry_device(n, g["seed"], dev)
            dbal = R.synthetic_balances_device(n, g["seed"], dev)
            h = R.DeviceStateHasher(n, dev, schedule=os.environ.get("PRYSM_C3_SCHED", "fused"))
            out = h.out
            fn = lambda: h.submit(rec, dbal)  # noqa: E731
            want = g["state_root"]
        elif c == "c1":
            n = g["n"]
            reg = R.synthetic_registry(n, g["seed"])
            drec = torch.from_numpy(reg.records.view("uint8").reshape(-1).copy()).to(dev)
            out = torch.empty(32, dtype=torch.uint8, device=dev)
            ws = torch.empty(L.mk_ssz_struct_list_workspace_bytes(n, R._fields(R.VALIDATOR_FIELDS), 9) + 256,
                             dtype=torch.uint8, device=dev)
            fn = lambda: D.struct_list_root(drec, n, 160, R.VALIDATOR_FIELDS, out=out, ws=ws)  # noqa: E731
            want = g["root"]
        else:
            raise SystemExit(f"unknown config {c}")
        sec = B._timeit(fn, a.steps, a.warmup)
        got = bytes(out.cpu().numpy()).hex()
        print(json.dumps({"config": c, "ms": round(sec * 1e3, 4), "root_ok": got == want}), flush=True)
        if got != want:
            raise SystemExit(f"{c}: root {got} != golden {want}")


if __name__ == "__main__":
    main()
