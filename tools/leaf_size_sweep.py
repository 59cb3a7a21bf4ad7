"""Leaf-pass efficiency against tree size (one process, interleaved rounds):
ns per 256-B window of the k_reduce leaf launch for n = 2^25 x f items, and
the leaf grid's workgroups per resident slot (1280 = 5 per CU x 256 CUs).
The question it answers: why the 2^25-item tree (the per-GPU shard at 8
GPUs) runs its leaf pass ~8 % slower per window than 2^26..2^28.

  python tools/leaf_size_sweep.py [--rounds 7] [--lib main|<variant>]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--fracs", default="0.5,0.75,1,1.125,1.25,1.5,1.75,2,3,4")
    ap.add_argument("--libs", default="main")
    a = ap.parse_args()
    import torch

    from tools.ab_leaf import load

    dev = torch.device("cuda:0")
    libs = {}
    for v in a.libs.split(","):
        p = os.path.join(ROOT, "prysm_amd", "lib", "libprysm_merkle.so") if v == "main" else \
            os.path.join(ROOT, "prysm_amd", "lib", "variants", f"libprysm_merkle_{v}.so")
        libs[v] = load(p)
        assert libs[v].mk_init(0) == 0
    fr = [float(x) for x in a.fracs.split(",")]
    sizes = [int((1 << 25) * f) // 8 * 8 for f in fr]
    nmax = max(sizes)
    items = torch.empty(nmax * 32, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    L0 = next(iter(libs.values()))
    assert L0.mk_dev_synth_fill(None, ctypes.c_void_p(items.data_ptr()), nmax * 32, 0x5EED000000000004, 0, st) == 0
    ws = torch.empty(L0.mk_ssz_merkle_workspace_bytes(nmax, 32) + 4096, dtype=torch.uint8, device=dev)
    out = torch.empty(32, dtype=torch.uint8, device=dev)
    leaf = {(v, n): [] for v in libs for n in sizes}
    for r in range(a.rounds + 1):
        for n in sizes:
            for v, L in libs.items():
                L.mk_prof_enable(1)
                L.mk_prof_read(None, None, None, None, None)
                rc = L.mk_dev_ssz_merkle_hash(None, ctypes.c_void_p(items.data_ptr()), n, 32,
                                              ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                              ws.numel(), st)
                torch.cuda.synchronize()
                assert rc == 0
                ms = ctypes.c_double()
                L.mk_prof_read(None, ctypes.byref(ms), None, None, None)
                L.mk_prof_enable(0)
                if r:
                    leaf[(v, n)].append(ms.value)
    for n in sizes:
        windows = n // 8
        for v in libs:
            med = statistics.median(leaf[(v, n)])
            print(json.dumps({"lib": v, "n": n, "log2n": round(n.bit_length() - 1 + (n / (1 << (n.bit_length() - 1)) - 1), 3),
                              "windows": windows, "wgs": windows // 1024, "rounds_of_1280": windows / 1024 / 1280,
                              "leaf_ms": med, "ns_per_window": med * 1e6 / windows}), flush=True)


if __name__ == "__main__":
    main()
