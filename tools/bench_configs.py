"""The other BASELINE.json configs, single GPU: each ``measure_cX`` builds its
device-resident inputs, checks the root against tests/golden/
full_size_roots.json, times >= 100 steps (wall clock bracketed by
torch.cuda.synchronize()) and returns one record.  ``bench.py`` (the
driver's C4 line) runs every one of them after its own timed region and
puts the compact records in ``side_configs``; ``bench.py --config cX`` prints
one config's full line (``run_config``), with its CPU baseline.

  c1: ssz.TreeHash of 16,384 synthetic ValidatorRecords from host buffers
      (typed Hashable path; the device-resident call and the reflective
      mirror timed beside it)
  c2: hashutil.Hash over 2^24 x 64-B messages (one Keccak-f each)
  c3: TreeHash of a synthetic 1,000,000-validator State{registry, balances}
      via the typed Hashable path (struct kernels + merkleHash)
  c4tree: ssz.TreeHash([][32]byte) of 2^28 elements (SURVEY 8(d)'s C4
      secondary: element digests fused into the leaf pass)
  c5: depth-32 deposit trie from 2^20 x 280-B synthetic deposits, as a
      stream of tries (pipelined front) and one trie alone
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK_INT_OPS = 256 * 4 * 32 * 2.4e9
OPS_PER_PERM = 4320
# A hash's final permutation only has to produce the 32-B digest: its last
# round needs theta on the 5 diagonal lanes and chi on 4 (58 ops, not 180).
OPS_SAVED_PER_HASH = 122
SEED = 0x5EED000000000000  # seed = 0x5EED.. + config id
SIDE_ORDER = ("c2", "c3", "c5", "c1")  # the order bench.py runs them in


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def golden(cfg: str):
    with open(os.path.join(ROOT, "tests", "golden", "full_size_roots.json")) as f:
        return json.load(f).get(cfg)


_SCLK = {}  # seconds per step -> the shader clock sampled while that loop ran


def _timeit(fn, steps, warmup):
    import torch

    from bench import ClockSampler

    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    sampler = ClockSampler(torch.cuda.current_device())
    sampler.start()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / steps
    _SCLK[sec] = sampler.stop()
    return sec


def _ops(perms, hashes):
    return perms * OPS_PER_PERM - hashes * OPS_SAVED_PER_HASH


def _lib_handles():
    import torch

    sys.path.insert(0, ROOT)
    from prysm_amd import _lib

    L = _lib.load()
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    return _lib, L, st, P


def measure_c1(dev, steps, warmup):
    """ssz.TreeHash([]*ValidatorRecord) of 16,384 synthetic validators, the
    reference's `go test -bench` shape: host records in, 32-B root out.
    value: the typed Hashable path (one library call: H2D, struct kernel,
    merkleHash, D2H); the same root from records already in HBM and the
    reflective mirror (makeSliceHasher -> makeStructHasher per element,
    batched digests) are reported beside it."""
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd import registry as R
    from prysm_amd import ssz as S

    L = _lib.load()
    g = golden("c1")
    n = g["n"]
    reg = R.synthetic_registry(n, g["seed"])
    typ = S.Slice(S.Ptr(R.VALIDATOR_SSZ))
    vals = reg.as_dicts()
    want = reg.tree_hash_ssz()
    assert S.tree_hash(vals, typ) == want, "c1: reflective and typed roots differ"
    sec = _timeit(reg.tree_hash_ssz, steps, warmup)
    drec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(dev)
    dout = torch.empty(32, dtype=torch.uint8, device=dev)
    dws = torch.empty(L.mk_ssz_struct_list_workspace_bytes(n, R._fields(R.VALIDATOR_FIELDS), 9) + 256,
                      dtype=torch.uint8, device=dev)
    sec_dev = _timeit(lambda: D.struct_list_root(drec, n, 160, R.VALIDATOR_FIELDS, out=dout, ws=dws), steps, warmup)
    dev_root = bytes(dout.cpu().numpy())
    t0 = time.perf_counter()
    for _ in range(3):
        S.tree_hash(vals, typ)
    refl = (time.perf_counter() - t0) / 3
    perms = 5 * n + (n / 4 / 2) * 2 + n / 8 + 1
    hashes = 4 * n + n / 8 + n / 8 + 1  # one final permutation per hash
    ok = want.hex() == g["root"] and dev_root == want
    return {"metric": "ssz.TreeHash of a 16,384-entry []ValidatorRecord (host buffers)", "unit": "validators/s",
            "value": n / sec, "sec": sec, "perms": perms, "hashes": hashes,
            "dominant_kernel": "k_struct_list_fused<3,6> (the whole list in one launch: 4 lanes per record -- the 3 field hashes side by side, the 2-block struct message on a lo/hi lane pair --, 8 windows per workgroup one per wave, 3 levels, then groups of 16 workgroups to the root and the mix-in)",
            "root": want.hex(), "root_matches_golden": ok,
            "config": {"workload": "C1: TreeHash([]*ValidatorRecord), 16,384 synthetic validators, host records",
                       "n": n, "root": want.hex(), "root_matches_golden": ok,
                       "reflective_mirror_ms": refl * 1e3, "device_resident_ms": sec_dev * 1e3,
                       "device_resident_frac": _ops(perms, hashes) / sec_dev / PEAK_INT_OPS,
                       "host_overhead_ms": (sec - sec_dev) * 1e3}}


def measure_c2(dev, steps, warmup):
    """hashutil.Hash over 2^24 x 64-B messages in HBM (mk_dev_hash_batch).
    Checked through a checksum of checksums: merkleHash of the 2^24 digests
    as 32-B items (the library's own tree, 0.6 ms) against the golden."""
    import torch

    from prysm_amd import device as D

    _lib, L, st, P = _lib_handles()
    g = golden("c2")
    n = g["n"]
    msgs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
    D.synth_fill(msgs, g["seed"])
    out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    sec = _timeit(lambda: _lib.check(L.mk_dev_hash_batch(None, P(msgs), n, 64, P(out), st()), "c2"), steps, warmup)
    check = bytes(D.merkle_hash(out, n, 32).cpu().numpy()).hex()
    ok = check == g.get("merkle_of_digests")
    del msgs, out
    return {"metric": "hashutil.Hash throughput, 2^24 x 64-B messages", "unit": "hashes/s",
            "value": n / sec, "sec": sec, "perms": n, "hashes": n,
            "dominant_kernel": "k_keccak64_lock (phase-locked, one 64-B message per lane)",
            "root": check, "root_matches_golden": ok,
            "config": {"workload": "C2: batched Keccak-256 of 2^24 x 64-B messages (1 GiB)", "n": n, "msg_len": 64,
                       "merkle_of_digests": check, "root_matches_golden": ok,
                       "hbm_GBps_algorithmic": n * 96 / sec / 1e9}}


def measure_c3(dev, steps, warmup):
    """TreeHash of State{registry, balances} at 10^6 validators, records and
    balances generated in HBM (registry.synthetic_*_device: the same bytes as
    the host generators the golden was made from).  The step: a stream of
    states through registry.StatePipeline (each state's registry levels 2..10
    in the next state's struct launch, its tops beside that launch; the last
    state's top inside the timed region).  Beside it, one state alone through
    registry.DeviceStateHasher ("fused"; PRYSM_C3_SCHED: another schedule).
    PRYSM_C3_STREAM=0: time the one-state form as the step."""
    import torch

    from prysm_amd import device as D
    from prysm_amd import registry as R

    g = golden("c3")
    n = g["n"]
    rec = R.synthetic_registry_device(n, g["seed"], dev)
    dbal = R.synthetic_balances_device(n, g["seed"], dev)
    hasher = R.DeviceStateHasher(n, dev, schedule=os.environ.get("PRYSM_C3_SCHED", "fused"))
    out = hasher.out
    sec_one = _timeit(lambda: hasher.submit(rec, dbal), steps, warmup)
    one = bytes(out.cpu().numpy()).hex()
    stream = os.environ.get("PRYSM_C3_STREAM", "1") == "1" and D.struct_pipe_ok(rec, n, 160, R.VALIDATOR_FIELDS)
    got = one
    sec = sec_one
    if stream:
        p = R.StatePipeline(n, dev)
        for _ in range(warmup):
            p.submit(rec, dbal)
        p.flush()
        p.wait()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            h = p.submit(rec, dbal)
        p.flush()
        p.wait()
        torch.cuda.synchronize()
        sec = (time.perf_counter() - t0) / steps
        got = bytes(h.cpu().numpy()).hex()
    ok = got == g["state_root"] and one == g["state_root"]
    # perms: 3 field hashes + 2 struct blocks per validator, registry + balances merkle, final
    perms = 5 * n + (n / 4 / 2) * 2 + n / 8 + (n / 16 / 2) * 2 + n / 32 + 1
    hashes = 4 * n + n / 8 + n / 8 + n / 32 + n / 32 + 1
    del rec, dbal
    return {"metric": "TreeHash of a 1M-validator State (registry + balances)", "unit": "validators/s",
            "value": n / sec, "sec": sec, "perms": perms, "hashes": hashes,
            "dominant_kernel": ("k_struct_lock<true> (phase-locked, 5 perms per record + both trees' level-1 windows "
                                "+ the previous state's registry levels 2-10 in one extra slot per wave)" if stream
                                else "k_struct_lock<false> (phase-locked, 5 perms per record + both trees' level-1 "
                                     "windows)"),
            "root": got, "root_matches_golden": ok,
            "config": {"workload": "C3: synthetic State{[]*ValidatorRecord, []uint64}, 1,000,000 validators, "
                                   "device-resident" + (", a stream of states (registry.StatePipeline)" if stream
                                                        else ""),
                       "n": n, "root": got, "root_matches_golden": ok, "stream": stream,
                       "schedule": hasher.schedule, "single_state_ms": sec_one * 1e3,
                       "single_state_frac": _ops(perms, hashes) / sec_one / PEAK_INT_OPS}}


def measure_c5(dev, steps, warmup):
    """The depth-32 deposit trie of 2^20 x 280-B deposits in HBM: a stream of
    tries through pipeline.TriePipeline(front="pipe") (trie i's locked front
    also builds levels 3-7 of trie i-1; its top beside trie i+1's front; the
    last trie's top inside the timed region), and one whole trie alone
    (mk_dev_deposit_trie_append: leaves, levels, top, in order)."""
    import torch

    from prysm_amd import device as D
    from prysm_amd.pipeline import TriePipeline

    _lib, L, st, P = _lib_handles()
    g = golden("c5")
    n, dl, depth = g["n"], g["deposit_len"], g["depth"]
    data = torch.empty(n * dl, dtype=torch.uint8, device=dev)
    D.synth_fill(data, g["seed"])
    lv = torch.empty(L.mk_deposit_trie_levels_bytes(n, depth), dtype=torch.uint8, device=dev)
    root = torch.empty(32, dtype=torch.uint8, device=dev)
    one = lambda: _lib.check(L.mk_dev_deposit_trie_append(None, P(lv), n, 0, P(data), None, n, dl, depth,  # noqa
                                                           P(root), st()), "c5")
    sec_one = _timeit(one, steps, warmup)
    one_root = bytes(root.cpu().numpy())
    front = os.environ.get("PRYSM_C5_FRONT", "pipe")
    if front == "pipe" and not D.deposit_trie_pipe_ok(data, n, dl, depth):
        front = "split"
    pipe = TriePipeline(n, dl, depth, dev, front=front)
    got = pipe.submit(data)
    pipe.flush()
    torch.cuda.synchronize()
    if bytes(got.cpu().numpy()) != one_root:
        raise SystemExit("c5: pipelined root differs from the one-call root")
    for _ in range(warmup):
        pipe.submit(data)
    pipe.flush()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        got = pipe.submit(data)
    pipe.flush()
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / steps
    last = bytes(got.cpu().numpy())
    ok = one_root.hex() == g["root"] and last == one_root
    perms = 3 * n + (n - 1) + (depth - 20)
    hashes = n + (n - 1) + (depth - 20)
    del data, lv
    return {"metric": "deposit trie build, 2^20 x 280-B deposits, depth 32", "unit": "deposits/s",
            "value": n / sec, "sec": sec, "perms": perms, "hashes": hashes,
            "dominant_kernel": ("k_trie_rec_lock<1024,4,true> (phase-locked front: leaves + levels 1-2 of trie i, "
                                "levels 3-7 of trie i-1)" if front == "pipe" else
                                "k_keccak_rec<35> + k_trie_level (split front)"),
            "root": one_root.hex(), "root_matches_golden": ok,
            "config": {"workload": "C5: trieutil deposit trie, 2^20 synthetic 280-B deposits (stream of tries, "
                                   "each trie's top overlapping the next trie's front)", "n": n,
                       "root": one_root.hex(), "root_matches_golden": ok, "front": front,
                       "single_trie_ms": sec_one * 1e3,
                       "single_trie_frac": _ops(perms, hashes) / sec_one / PEAK_INT_OPS,
                       # the reference's own algorithm (UpdateDepositTrie per deposit,
                       # deposit_trie.go:29-40): 3 leaf perms + 32 node perms per deposit
                       "reference_incremental_perms": 35 * n, "batch_perms": perms}}


MEASURE = {"c1": measure_c1, "c2": measure_c2, "c3": measure_c3, "c5": measure_c5}


def side_entry(r):
    """The compact record bench.py puts in ``side_configs``."""
    ops = _ops(r["perms"], r["hashes"])
    e = {"metric": r["metric"], "value": r["value"], "unit": r["unit"], "ms_per_step": r["sec"] * 1e3,
         "frac": ops / r["sec"] / PEAK_INT_OPS, "achieved_Tops": ops / r["sec"] / 1e12,
         "perms_per_step": r["perms"], "dominant_kernel": r["dominant_kernel"], "root": r["root"],
         "root_matches_golden": r["root_matches_golden"]}
    for k in ("single_trie_ms", "single_trie_frac", "single_state_ms", "single_state_frac", "stream",
              "device_resident_ms", "device_resident_frac", "schedule", "front", "reference_incremental_perms",
              "hbm_GBps_algorithmic"):
        if k in r["config"]:
            e[k] = r["config"][k]
    return e


def side_configs(dev, steps: int = 200, warmup: int = 40, only=SIDE_ORDER, cpu: bool = True):
    """Every side config, one after the other, in this process (bench.py);
    a config that fails is recorded with its error, not raised.  ``cpu``:
    also C5's CPU baseline of the reference's incremental algorithm on a
    small sample (the fast permutation), the unit of its ``value``."""
    import torch

    out = {}
    for c in only:
        t0 = time.perf_counter()
        try:
            e = side_entry(MEASURE[c](dev, steps, warmup))
            if c == "c5" and cpu:
                e["cpu_reference_incremental"] = cpu_c5_incremental(1 << 14)
        except Exception as ex:  # noqa: BLE001 -- recorded in the line
            e = {"error": f"{type(ex).__name__}: {ex}"[:500], "root_matches_golden": False}
        torch.cuda.empty_cache()
        e["wall_s"] = round(time.perf_counter() - t0, 2)
        out[c] = e
    return out


def cpu_c5_incremental(m: int):
    """The reference's deposit-trie algorithm (UpdateDepositTrie per deposit,
    deposit_trie.go:29-40: 3 leaf + 32 node permutations each), oracle C
    port with the unrolled permutation, 1 thread, m deposits of the same
    SplitMix64 stream."""
    from oracle import oracle as O

    g = golden("c5")
    host = O.splitmix_bytes(m * g["deposit_len"], g["seed"])
    deps = [bytes(host[i * g["deposit_len"]:(i + 1) * g["deposit_len"]]) for i in range(m)]
    with O.fast_permutation():
        t0 = time.perf_counter()
        O.deposit_trie_incremental_root(deps)
        dt = time.perf_counter() - t0
    return {"value": m / dt, "unit": "deposits/s", "cores": 1, "kind": "port", "cpu_model": _cpu_model(),
            "ns_per_perm": dt / (35 * m) * 1e9,
            "sample": f"oracle or_deposit_trie_incremental (UpdateDepositTrie loop, 35 perms/deposit), "
                      f"2^{m.bit_length() - 1} x 280-B deposits, unrolled permutation, 1 thread, {dt:.2f} s"}


def _line(args, r, cpu=None):
    ops = _ops(r["perms"], r["hashes"])
    out = {"metric": r["metric"], "value": r["value"], "unit": r["unit"], "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": r["sec"] * 1e3, "higher_is_better": True, "scaling": "none",
           "vs_baseline": None, "dtype": "u64 (Keccak lanes as u32 pairs)", "data": "synthetic",
           "config": r["config"],
           "roofline": {"bound": "valu-int", "kernel": r["dominant_kernel"], "achieved": ops / r["sec"] / 1e12,
                        "peak": PEAK_INT_OPS / 1e12, "unit": "Tops/s (int32 VALU, whole step)",
                        "frac": ops / r["sec"] / PEAK_INT_OPS, "perms_per_step": r["perms"],
                        "hashes_per_step": r["hashes"]}}
    sclk = _SCLK.get(r["sec"])
    out["roofline"]["sclk_sampled"] = sclk
    out["roofline"]["frac_at_sampled_clock"] = (ops / r["sec"] / (PEAK_INT_OPS / 2.4e3 * sclk["mean_MHz"])
                                                if sclk and sclk["mean_MHz"] > 0 else None)
    out["roofline"].update(r.get("extra", {}))
    if cpu:
        out["cpu_baseline"] = cpu
    print(json.dumps(out), flush=True)
    return 0 if r["root_matches_golden"] else 1


def _cpu_port(fn, unit, sample, m):
    """Times fn() once with the unrolled permutation (1 thread)."""
    from oracle import oracle as O

    with O.fast_permutation():
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
    return {"value": m / dt, "unit": unit, "cores": 1, "kind": "port", "cpu_model": _cpu_model(),
            "sample": f"{sample}, unrolled permutation, 1 thread, {dt:.2f} s"}


def run_config(args):
    import torch

    sys.path.insert(0, ROOT)
    from prysm_amd import _lib
    from prysm_amd import device as D

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    _lib.init(0)
    cpu_on = not args.no_cpu_baseline

    if args.config in MEASURE:
        r = MEASURE[args.config](dev, args.steps, args.warmup)
        cpu = None
        if cpu_on:
            from oracle import oracle as O
            from prysm_amd import registry as R

            if args.config == "c1":
                reg = R.synthetic_registry(r["config"]["n"], SEED + 1)
                raw = reg.records.view(np.uint8).reshape(-1)
                n = r["config"]["n"]
                cpu = _cpu_port(lambda: O.merkle_hash_flat(O.struct_roots(raw, n, 160, R.VALIDATOR_FIELDS)
                                                           .reshape(-1), n, 32),
                                "validators/s", "oracle struct_roots + merkleHash, the same 16,384 validators", n)
            elif args.config == "c2":
                m = 1 << 21
                host = O.splitmix_bytes(m * 64, SEED + 2)
                cpu = _cpu_port(lambda: O.keccak256_batch(host, 64), "hashes/s",
                                "oracle keccak256_batch, 2^21 x 64-B messages", m)
            elif args.config == "c3":
                m = 1 << 17
                reg = R.synthetic_registry(m, SEED + 3)
                bal = R.synthetic_balances(m, SEED + 3)
                raw = reg.records.view(np.uint8).reshape(-1)

                def c3cpu():
                    rr = O.struct_roots(raw, m, 160, R.VALIDATOR_FIELDS)
                    O.merkle_hash_flat(rr.reshape(-1), m, 32)
                    O.merkle_hash_flat(bal.view(np.uint8), m, 8)
                cpu = _cpu_port(c3cpu, "validators/s", "oracle struct_roots + merkleHash, 2^17 validators + "
                                "balances", m)
            elif args.config == "c5":
                cpu = cpu_c5_incremental(1 << 16)
        return _line(args, r, cpu)

    if args.config == "c4tree":
        # SURVEY 8(d)'s C4 secondary: ssz.TreeHash([][32]byte) of 2^28
        # elements (8 GiB in HBM) = merkleHash over Keccak(le32(32) || e_i):
        # +2^28 permutations on top of C4 (x3.67 the work), element digests
        # fused into the leaf pass; one call per step.
        g = golden("c4tree")
        n, el = g["n"], g["elem_len"]
        items = torch.empty(n * el, dtype=torch.uint8, device=dev)
        D.synth_fill(items, g["seed"])
        out = torch.empty(32, dtype=torch.uint8, device=dev)
        ws = D.tree_hash_bytes_list_workspace(n, el, dev)
        D.tree_hash_bytes_list(items, n, el, out=out, ws=ws)
        torch.cuda.synchronize()
        root = bytes(out.cpu().numpy()).hex()
        if root != g["root"]:
            raise SystemExit(f"c4tree: root {root} != golden {g['root']}")
        D.prof_enable(True)
        D.prof_read()
        sec = _timeit(lambda: D.tree_hash_bytes_list(items, n, el, out=out, ws=ws), args.steps, args.warmup)
        D.prof_enable(False)
        leaf_ms, launches, lperms, lhashes = D.prof_read()
        # whole step: n element perms + the C4-shaped tree (2^25 windows x 2,
        # 2^25 - 1 pair nodes, 1 mix-in); one final permutation per hash
        perms = n + (n // 8) * 2 + (n // 8 - 1) + 1
        hashes = n + n // 8 + (n // 8 - 1) + 1
        nl = max(launches, 1)
        leaf_s = leaf_ms / 1e3 / nl
        leaf_ops = _ops(lperms / nl, lhashes / nl)
        # the locked form needs n % 8 == 0 and n >= 2^23, true at 2^28
        kname = "k_elem_lock"
        kdesc = ("k_elem_lock (phase-locked element windows: 1024-thread workgroups, s_barrier in every Keccak "
                 "round; 8 element digests + the window hash per thread, 10 permutations; coalesced LDS-DMA "
                 "staging)")
        from bench import load_pmc

        traffic, clk, pmc_src = load_pmc(kname)
        cpu = None
        if cpu_on:
            from oracle import oracle as O

            m = 1 << 23
            host = O.splitmix_bytes(m * el, g["seed"])
            cpu = _cpu_port(lambda: O.tree_hash_bytes_list(host, m, el), "leaves/s",
                            "oracle elem digests + merkleHash, 2^23 x 32-B elements (same stream)", m)
        r = {"metric": "tree-hash leaves/sec @2^28 chunks, TreeHash([][32]byte) (element digests + merkleHash)",
             "unit": "leaves/s", "value": n / sec, "sec": sec, "perms": perms, "hashes": hashes,
             "dominant_kernel": kdesc, "root": root, "root_matches_golden": True,
             "config": {"workload": "C4 secondary: ssz.TreeHash of 2^28 x [32]byte elements (8 GiB), one device "
                                    "call, element digests fused into the leaf pass", "n": n, "elem_len": el,
                        "root": root, "root_matches_golden": True},
             "extra": {"traffic": traffic, "traffic_source": pmc_src, "effective_clock_GHz": clk,
                       "leaf_kernel_ms": leaf_s * 1e3, "leaf_kernel_achieved": leaf_ops / leaf_s / 1e12,
                       "leaf_kernel_frac": leaf_ops / leaf_s / PEAK_INT_OPS, "leaf_perms_per_launch": lperms / nl,
                       "leaf_hashes_per_launch": lhashes / nl, "perms_per_leaf": perms / n,
                       "hbm_GBps_algorithmic": n * el / leaf_s / 1e9}}
        return _line(args, r, cpu)
    raise SystemExit(f"unknown config {args.config}")
