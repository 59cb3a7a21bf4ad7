"""A/B timing of libprysm_merkle variants in ONE process (cdna guide §5.4
rule 24): interleaved rounds, same device, same data; reports the median
time of a full merkleHash and of its leaf pass per variant, and checks that
every variant returns the same root.

  python tools/ab_leaf.py [--log2n 26] [--rounds 7] base loadall w5 ...
(variants are prysm_amd/lib/variants/libprysm_merkle_<name>.so; "main" is
the in-tree library)."""
import argparse
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def load(path):
    from prysm_amd import _lib

    L = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    for name, (res, args) in _lib._SIGS.items():
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--log2n", type=int, default=26)
    ap.add_argument("--item-len", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--trie", action="store_true", help="A/B the depth-32 deposit trie over 2^log2n x 280-B deposits")
    ap.add_argument("--struct", action="store_true", help="A/B the typed registry root of 1,000,000 validators")
    ap.add_argument("--c2", action="store_true", help="A/B the batched Keccak of 2^log2n x 64-B messages")
    ap.add_argument("--host-struct", type=int, default=0,
                    help="A/B mk_ssz_struct_list_root from host records (this many validators)")
    ap.add_argument("--append", type=int, default=0,
                    help="A/B this many single-deposit appends on a 2^log2n-capacity trie (Root after each)")
    ap.add_argument("variants", nargs="+")
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda:0")
    libs = {}
    for v in a.variants:
        p = os.path.join(ROOT, "prysm_amd", "lib", "libprysm_merkle.so") if v == "main" else \
            os.path.join(ROOT, "prysm_amd", "lib", "variants", f"libprysm_merkle_{v}.so")
        libs[v] = load(p)
        assert libs[v].mk_init(0) == 0
    if a.append:
        return ab_append(a, libs, dev)
    if a.trie:
        return ab_trie(a, libs, dev)
    if a.struct:
        return ab_struct(a, libs, dev)
    if a.c2:
        return ab_c2(a, libs, dev)
    if a.host_struct:
        return ab_host_struct(a, libs)
    n, il = 1 << a.log2n, a.item_len
    items = torch.empty(n * il, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    first = libs[a.variants[0]]
    assert first.mk_dev_synth_fill(None, ctypes.c_void_p(items.data_ptr()), n * il, 0x5EED000000000004, 0, st) == 0
    ws = torch.empty(max(L.mk_ssz_merkle_workspace_bytes(n, il) for L in libs.values()) + 4096, dtype=torch.uint8, device=dev)
    outs = {v: torch.empty(32, dtype=torch.uint8, device=dev) for v in a.variants}
    times = {v: [] for v in a.variants}
    leaf = {v: [] for v in a.variants}
    for r in range(a.rounds + 1):
        for v, L in libs.items():
            L.mk_prof_enable(1)
            L.mk_prof_read(None, None, None, None, None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = L.mk_dev_ssz_merkle_hash(None, ctypes.c_void_p(items.data_ptr()), n, il,
                                          ctypes.c_void_p(outs[v].data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                          ws.numel(), st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (v, rc)
            ms = ctypes.c_double()
            cnt = ctypes.c_uint64()
            perms = ctypes.c_double()
            L.mk_prof_read(None, ctypes.byref(ms), ctypes.byref(cnt), ctypes.byref(perms), None)
            L.mk_prof_enable(0)
            if r:  # round 0 is warmup
                times[v].append(e0.elapsed_time(e1))
                leaf[v].append(ms.value)
    # "nl_*" variants are compute-only probes (MK_NOLOAD): their roots differ
    roots = {v: bytes(o.cpu().numpy()).hex() for v, o in outs.items() if not v.startswith("nl_")}
    assert len(set(roots.values())) <= 1, roots
    for v in a.variants:
        print(json.dumps({"variant": v, "log2n": a.log2n, "median_ms": statistics.median(times[v]),
                          "min_ms": min(times[v]), "leaf_median_ms": statistics.median(leaf[v]),
                          "leaves_per_s": n / (statistics.median(times[v]) / 1e3)}))
    print(json.dumps({"root": next(iter(roots.values()), None)}))


def ab_trie(a, libs, dev):
    import torch

    n, ln, depth = 1 << a.log2n, 280, 32
    data = torch.empty(n * ln, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    first = libs[a.variants[0]]
    assert first.mk_dev_synth_fill(None, ctypes.c_void_p(data.data_ptr()), n * ln, 0x5EED000000000005, 0, st) == 0
    lv = torch.empty(first.mk_deposit_trie_levels_bytes(n, depth), dtype=torch.uint8, device=dev)
    outs = {v: torch.empty(32, dtype=torch.uint8, device=dev) for v in a.variants}
    times = {v: [] for v in a.variants}
    for r in range(a.rounds + 1):
        for v, L in libs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = L.mk_dev_deposit_trie_append(None, ctypes.c_void_p(lv.data_ptr()), n, 0,
                                              ctypes.c_void_p(data.data_ptr()), None, n, ln, depth,
                                              ctypes.c_void_p(outs[v].data_ptr()), st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (v, rc)
            if r:
                times[v].append(e0.elapsed_time(e1))
    roots = {v: bytes(o.cpu().numpy()).hex() for v, o in outs.items()}
    # "nl_*" variants are compute probes (MK_TRIE_PROBE): their roots differ
    assert len({r for v, r in roots.items() if not v.startswith("nl_")}) == 1, roots
    # the C5 bench's form: a stream of tries, each trie's front (leaves + levels
    # wider than 2^17 nodes) on the main stream, its top on a high-priority
    # side stream overlapping the next front (pipeline.TriePipeline, 2 slots)
    split = 0
    while -(-n // (1 << split)) > (1 << 17):
        split += 1
    side = torch.cuda.Stream(priority=-1)
    sst = ctypes.c_void_p(side.cuda_stream)
    lvs = [lv, torch.empty_like(lv)]
    souts = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(2)]
    stream_ms = {v: [] for v in a.variants}
    S = 20
    for r in range(a.rounds + 1):
        for v, L in libs.items():
            torch.cuda.synchronize()
            evs = [None, None]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(S):
                s = i % 2
                if evs[s] is not None:
                    torch.cuda.current_stream().wait_event(evs[s])
                assert L.mk_dev_deposit_trie_build(None, ctypes.c_void_p(lvs[s].data_ptr()), n,
                                                   ctypes.c_void_p(data.data_ptr()), None, n, ln, split, depth,
                                                   None, st) == 0
                side.wait_stream(torch.cuda.current_stream())
                assert L.mk_dev_deposit_trie_levels(None, ctypes.c_void_p(lvs[s].data_ptr()), n, n, split, depth,
                                                    depth, ctypes.c_void_p(souts[s].data_ptr()), sst) == 0
                evs[s] = torch.cuda.Event()
                evs[s].record(side)
            torch.cuda.current_stream().wait_stream(side)
            e1.record()
            torch.cuda.synchronize()
            assert v.startswith("nl_") or bytes(souts[(S - 1) % 2].cpu().numpy()).hex() == roots[v], v
            if r:
                stream_ms[v].append(e0.elapsed_time(e1) / S)
    # the C5 bench's form since round 4: the pipelined front (trie i's locked
    # front also builds levels 3-7 of trie i-1; trie i-1's top on the side
    # stream beside trie i+1's front), pipeline.TriePipeline(front="pipe")
    pipe_ms = {v: [] for v in a.variants}
    P = 100
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    if first.mk_deposit_trie_pipe_ok(vp(data), n, ln, depth, st):
        plv = [torch.empty_like(lv) for _ in range(4)]
        prt = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(4)]
        for r in range(a.rounds + 1):
            for v, L in libs.items():
                torch.cuda.synchronize()
                done = {}
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                prev = None
                for i in range(P):
                    s = i % 4
                    if i % 2 == 0 and (i - 3) in done:
                        torch.cuda.current_stream().wait_event(done[i - 3])
                    assert L.mk_dev_deposit_trie_build_pipe(None, vp(plv[s]), None if prev is None else vp(plv[prev]),
                                                            n, vp(data), n, ln, depth, st) == 0
                    if prev is not None:
                        side.wait_stream(torch.cuda.current_stream())
                        assert L.mk_dev_deposit_trie_pipe_top(None, vp(plv[prev]), n, n, depth, vp(prt[prev]),
                                                              sst) == 0
                        done[i - 1] = torch.cuda.Event()
                        done[i - 1].record(side)
                    prev = s
                side.wait_stream(torch.cuda.current_stream())
                assert L.mk_dev_deposit_trie_levels(None, vp(plv[prev]), n, n, 2, depth, depth, vp(prt[prev]),
                                                    sst) == 0
                torch.cuda.current_stream().wait_stream(side)
                e1.record()
                torch.cuda.synchronize()
                assert v.startswith("nl_") or bytes(prt[prev].cpu().numpy()).hex() == roots[v], v
                if r:
                    pipe_ms[v].append(e0.elapsed_time(e1) / P)
    for v in a.variants:
        print(json.dumps({"variant": v, "trie_log2n": a.log2n, "median_ms": statistics.median(times[v]),
                          "min_ms": min(times[v]), "stream_median_ms": statistics.median(stream_ms[v]),
                          "stream_min_ms": min(stream_ms[v]),
                          "pipe_median_ms": statistics.median(pipe_ms[v]) if pipe_ms[v] else None,
                          "pipe_min_ms": min(pipe_ms[v]) if pipe_ms[v] else None}))
    print(json.dumps({"root": next(iter(roots.values()), None)}))


def ab_append(a, libs, dev):
    """UpdateDepositTrie + Root() latency: each variant owns a trie holding
    2^log2n - append deposits, then appends one deposit at a time."""
    import torch

    cap, ln, depth, k = 1 << a.log2n, 280, 32, a.append
    data = torch.empty(cap * ln, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    first = libs[a.variants[0]]
    assert first.mk_dev_synth_fill(None, ctypes.c_void_p(data.data_ptr()), cap * ln, 0x5EED000000000005, 0, st) == 0
    nb = first.mk_deposit_trie_levels_bytes(cap, depth)
    lvs = {v: torch.empty(nb, dtype=torch.uint8, device=dev) for v in a.variants}
    outs = {v: torch.empty(32, dtype=torch.uint8, device=dev) for v in a.variants}
    base = cap - k
    for v, L in libs.items():
        assert L.mk_dev_deposit_trie_append(None, ctypes.c_void_p(lvs[v].data_ptr()), cap, 0,
                                            ctypes.c_void_p(data.data_ptr()), None, base, ln, depth,
                                            ctypes.c_void_p(outs[v].data_ptr()), st) == 0
    torch.cuda.synchronize()
    times = {v: [] for v in a.variants}
    for i in range(k):
        for v, L in libs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = L.mk_dev_deposit_trie_append(None, ctypes.c_void_p(lvs[v].data_ptr()), cap, base + i,
                                              ctypes.c_void_p(data.data_ptr() + (base + i) * ln), None, 1, ln, depth,
                                              ctypes.c_void_p(outs[v].data_ptr()), st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (v, rc)
            times[v].append(e0.elapsed_time(e1))
    roots = {v: bytes(o.cpu().numpy()).hex() for v, o in outs.items()}
    assert len(set(roots.values())) == 1, roots
    for v in a.variants:
        t = times[v][8:]
        print(json.dumps({"variant": v, "append_cap_log2": a.log2n, "appends": k, "median_us": 1e3 * statistics.median(t),
                          "min_us": 1e3 * min(t)}))
    print(json.dumps({"root": next(iter(roots.values()), None)}))


def ab_struct(a, libs, dev):
    import numpy as np
    import torch

    from prysm_amd import registry as R

    n = 1_000_000
    reg = R.synthetic_registry(n, 0x5EED000000000003)
    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(dev)
    spec = R._fields(R.VALIDATOR_FIELDS)
    nf = len(R.VALIDATOR_FIELDS)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    first = libs[a.variants[0]]
    ws = torch.empty(max(L.mk_ssz_struct_list_workspace_bytes(n, spec, nf) for L in libs.values()) + 4096,
                     dtype=torch.uint8, device=dev)
    outs = {v: torch.empty(32, dtype=torch.uint8, device=dev) for v in a.variants}
    times = {v: [] for v in a.variants}
    for r in range(a.rounds + 1):
        for v, L in libs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = L.mk_dev_ssz_struct_list_root(None, ctypes.c_void_p(rec.data_ptr()), n, 160, spec, nf,
                                               ctypes.c_void_p(outs[v].data_ptr()), ctypes.c_void_p(ws.data_ptr()),
                                               ws.numel(), st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (v, rc)
            if r:
                times[v].append(e0.elapsed_time(e1))
    roots = {v: bytes(o.cpu().numpy()).hex() for v, o in outs.items()}
    assert len(set(roots.values())) == 1, roots
    for v in a.variants:
        print(json.dumps({"variant": v, "struct_n": n, "median_ms": statistics.median(times[v]),
                          "min_ms": min(times[v])}))
    print(json.dumps({"root": next(iter(roots.values()), None)}))



def ab_c2(a, libs, dev):
    import torch

    n = 1 << a.log2n
    msgs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    first = libs[a.variants[0]]
    assert first.mk_dev_synth_fill(None, ctypes.c_void_p(msgs.data_ptr()), n * 64, 0x5EED000000000002, 0, st) == 0
    outs = {v: torch.empty(n * 32, dtype=torch.uint8, device=dev) for v in a.variants}
    times = {v: [] for v in a.variants}
    for r in range(a.rounds + 1):
        for v, L in libs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rc = L.mk_dev_hash_batch(None, ctypes.c_void_p(msgs.data_ptr()), n, 64, ctypes.c_void_p(outs[v].data_ptr()), st)
            e1.record()
            torch.cuda.synchronize()
            assert rc == 0, (v, rc)
            if r:
                times[v].append(e0.elapsed_time(e1))
    ref = next(iter(outs.values()))
    assert all(torch.equal(ref, o) for o in outs.values())
    for v in a.variants:
        print(json.dumps({"variant": v, "c2_log2n": a.log2n, "median_ms": statistics.median(times[v]),
                          "min_ms": min(times[v]), "hashes_per_s": n / (statistics.median(times[v]) / 1e3)}))


def ab_host_struct(a, libs):
    """Host-buffer TreeHash of a synthetic registry (H2D + struct kernel +
    merkleHash + D2H in one library call), wall time per call."""
    import time

    import numpy as np

    from prysm_amd import registry as R

    n = a.host_struct
    reg = R.synthetic_registry(n, 0x5EED000000000001)
    rec = np.ascontiguousarray(reg.records)
    raw = rec.view(np.uint8).reshape(-1)
    f = R._fields(R.VALIDATOR_FIELDS)
    times = {v: [] for v in a.variants}
    roots = {}
    for r in range(a.rounds + 1):
        for v, L in libs.items():
            out = ctypes.create_string_buffer(32)
            t0 = time.perf_counter()
            rc = L.mk_ssz_struct_list_root(None, raw.ctypes.data_as(ctypes.c_void_p), n, rec.dtype.itemsize, f,
                                           len(R.VALIDATOR_FIELDS), out)
            dt = time.perf_counter() - t0
            assert rc == 0, (v, rc)
            roots[v] = out.raw
            if r:
                times[v].append(dt * 1e3)
    assert len(set(roots.values())) == 1, roots
    for v in a.variants:
        print(json.dumps({"variant": v, "host_struct_n": n, "median_ms": statistics.median(times[v]),
                          "min_ms": min(times[v])}))


if __name__ == "__main__":
    main()
