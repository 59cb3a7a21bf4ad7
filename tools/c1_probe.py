"""C1 device-resident (16,384 ValidatorRecords, TreeHash of the list) by
parts: the shipped list root (struct roots + the list's tree) and the
struct roots alone.  Wall-clock per step over --steps after
--warmup (tools/bench_configs._timeit); roots checked against
tests/golden/full_size_roots.json.

  python tools/c1_probe.py [--steps 200 --warmup 40]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=40)
    a = ap.parse_args()
    import torch

    import bench_configs as B
    from prysm_amd import device as D
    from prysm_amd import registry as R

    dev = torch.device("cuda:0")
    _lib, L, st, P = B._lib_handles()
    g = B.golden("c1")
    n = g["n"]
    reg = R.synthetic_registry(n, g["seed"])
    drec = torch.from_numpy(reg.records.view("uint8").reshape(-1).copy()).to(dev)
    f = R._fields(R.VALIDATOR_FIELDS)
    out = torch.empty(32, dtype=torch.uint8, device=dev)
    ws = torch.empty(L.mk_ssz_struct_list_workspace_bytes(n, f, 9) + 256, dtype=torch.uint8, device=dev)
    roots = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    rws = torch.empty(L.mk_ssz_struct_list_workspace_bytes(n, f, 9) + 256, dtype=torch.uint8, device=dev)
    forms = {
        "list": lambda: D.struct_list_root(drec, n, 160, R.VALIDATOR_FIELDS, out=out, ws=ws),
        "roots": lambda: D.struct_roots(drec, n, 160, R.VALIDATOR_FIELDS, out=roots, ws=rws),
    }
    for name, fn in forms.items():
        out.zero_()
        fn()
        sec = B._timeit(fn, a.steps, a.warmup)
        got = bytes(out.cpu().numpy()).hex()
        ok = name == "roots" or got == g["root"]
        print(json.dumps({"form": name, "ms": round(sec * 1e3, 4), "root_ok": ok}), flush=True)
        if not ok:
            raise SystemExit(f"{name}: root {got} != golden {g['root']}")


if __name__ == "__main__":
    main()
