"""Single-GPU side benchmarks for the other BASELINE.json configs
(bench.py --config c1|c2|c3|c4tree|c5).  Same JSON shape as the headline line; inputs
resident in HBM before timing; hipEvent-free wall timing bracketed by
torch.cuda.synchronize(); the dominant kernel is timed with the library's
own hipEvents where the library exposes them (merkle passes).

  c1: ssz.TreeHash of 16,384 synthetic ValidatorRecords from host buffers
      (typed Hashable path; the reflective mirror timed beside it)
  c2: hashutil.Hash over 2^24 x 64-B messages (one Keccak-f each)
  c3: TreeHash of a synthetic 1,000,000-validator State{registry, balances}
      via the typed Hashable path (struct kernels + merkleHash)
  c4tree: ssz.TreeHash([][32]byte) of 2^28 elements (SURVEY 8(d)'s C4
      secondary: element digests fused into the leaf pass)
  c5: depth-32 deposit trie from 2^20 x 280-B synthetic deposits
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PEAK_INT_OPS = 256 * 4 * 32 * 2.4e9
OPS_PER_PERM = 4320
# A hash's final permutation only has to produce the 32-B digest: its last
# round needs theta on the 5 diagonal lanes and chi on 4 (58 ops, not 180).
OPS_SAVED_PER_HASH = 122


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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


def _line(metric, value, unit, args, sec, perms, hashes, config, cpu=None, extra=None):
    achieved = (perms * OPS_PER_PERM - hashes * OPS_SAVED_PER_HASH) / sec
    out = {"metric": metric, "value": value, "unit": unit, "n_gpus": 1, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": sec * 1e3, "higher_is_better": True, "scaling": "none",
           "vs_baseline": None, "dtype": "u64 (Keccak lanes as u32 pairs)", "data": "synthetic",
           "config": config,
           "roofline": {"bound": "valu-int", "achieved": achieved / 1e12, "peak": PEAK_INT_OPS / 1e12,
                        "unit": "Tops/s (int32 VALU, whole step)", "frac": achieved / PEAK_INT_OPS,
                        "perms_per_step": perms, "hashes_per_step": hashes}}
    sclk = _SCLK.get(sec)
    out["roofline"]["sclk_sampled"] = sclk
    out["roofline"]["frac_at_sampled_clock"] = (achieved / (PEAK_INT_OPS / 2.4e3 * sclk["mean_MHz"])
                                                if sclk and sclk["mean_MHz"] > 0 else None)
    if extra:
        out["roofline"].update(extra)
    if cpu:
        out["cpu_baseline"] = cpu
    print(json.dumps(out), flush=True)


def run_config(args):
    import torch

    sys.path.insert(0, ROOT)
    from prysm_amd import _lib
    from prysm_amd import device as D

    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    _lib.init(0)
    L = _lib.load()
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)  # noqa: E731
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    seed = 0x5EED000000000000

    if args.config == "c1":
        # ssz.TreeHash([]*ValidatorRecord) of 16,384 synthetic validators, the
        # reference's `go test -bench` shape: host records in, 32-B root out.
        # value: the typed Hashable path (one library call: H2D, struct
        # kernel, merkleHash, D2H); the reflective mirror (makeSliceHasher ->
        # makeStructHasher per element, batched digests) is reported beside it.
        from prysm_amd import registry as R
        from prysm_amd import ssz as S

        n = 16_384
        reg = R.synthetic_registry(n, seed + 1)
        typ = S.Slice(S.Ptr(R.VALIDATOR_SSZ))
        vals = reg.as_dicts()
        want = reg.tree_hash_ssz()
        assert S.tree_hash(vals, typ) == want, "c1: reflective and typed roots differ"
        sec = _timeit(reg.tree_hash_ssz, args.steps, args.warmup)
        # the same root from records already in HBM: what the host-buffer call
        # spends beyond the device work is PCIe (2.6 MB) + launch/sync latency
        drec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(dev)
        dout = torch.empty(32, dtype=torch.uint8, device=dev)
        dws = torch.empty(L.mk_ssz_struct_list_workspace_bytes(n, R._fields(R.VALIDATOR_FIELDS), 9) + 256,
                          dtype=torch.uint8, device=dev)
        D.struct_list_root(drec, n, 160, R.VALIDATOR_FIELDS, out=dout, ws=dws)
        torch.cuda.synchronize()
        assert bytes(dout.cpu().numpy()) == want
        sec_dev = _timeit(lambda: D.struct_list_root(drec, n, 160, R.VALIDATOR_FIELDS, out=dout, ws=dws),
                          args.steps, args.warmup)
        t0 = time.perf_counter()
        for _ in range(3):
            S.tree_hash(vals, typ)
        refl = (time.perf_counter() - t0) / 3
        perms = 5 * n + (n / 4 / 2) * 2 + n / 8 + 1
        hashes = 4 * n + n / 8 + n / 8 + 1  # one final permutation per hash
        cpu = None
        if not args.no_cpu_baseline:
            from oracle import oracle as O

            raw = reg.records.view(np.uint8).reshape(-1)
            t0 = time.perf_counter()
            for _ in range(10):
                rr = O.struct_roots(raw, n, 160, R.VALIDATOR_FIELDS, nthreads=1)
                O.merkle_hash_flat(rr.reshape(-1), n, 32)
            dt = (time.perf_counter() - t0) / 10
            cpu = {"value": n / dt, "unit": "validators/s", "cores": 1, "kind": "port", "cpu_model": _cpu_model(),
                   "sample": f"oracle struct_roots + merkleHash, the same 16,384 validators, 1 thread, {dt * 1e3:.1f} ms"}
        _line("ssz.TreeHash of a 16,384-entry []ValidatorRecord (host buffers)", n / sec, "validators/s", args, sec,
              perms, hashes, {"workload": "C1: TreeHash([]*ValidatorRecord), 16,384 synthetic validators, host records",
                      "n": n, "root": want.hex(), "reflective_mirror_ms": refl * 1e3,
                      "device_resident_ms": sec_dev * 1e3,
                      "host_overhead_ms": (sec - sec_dev) * 1e3}, cpu)
        return

    if args.config == "c2":
        n = 1 << 24
        msgs = torch.empty(n * 64, dtype=torch.uint8, device=dev)
        D.synth_fill(msgs, seed + 2)
        out = torch.empty(n * 32, dtype=torch.uint8, device=dev)
        sec = _timeit(lambda: _lib.check(L.mk_dev_hash_batch(None, P(msgs), n, 64, P(out), st()), "c2"),
                      args.steps, args.warmup)
        cpu = None
        if not args.no_cpu_baseline:
            from oracle import oracle as O

            m = 1 << 21
            host = O.splitmix_bytes(m * 64, seed + 2)
            t0 = time.perf_counter()
            O.keccak256_batch(host, 64, nthreads=1)
            dt = time.perf_counter() - t0
            cpu = {"value": m / dt, "unit": "hashes/s", "cores": 1, "kind": "port", "cpu_model": _cpu_model(),
                   "sample": f"oracle keccak256_batch, 2^21 x 64-B messages, 1 thread, {dt:.1f} s"}
        _line("hashutil.Hash throughput, 2^24 x 64-B messages", n / sec, "hashes/s", args, sec, n, n,
              {"workload": "C2: batched Keccak-256 of 2^24 x 64-B messages (1 GiB)", "n": n, "msg_len": 64},
              cpu, {"hbm_GBps_algorithmic": n * 96 / sec / 1e9})
        return

    if args.config == "c3":
        from prysm_amd import registry as R

        n = 1_000_000
        reg = R.synthetic_registry(n, seed + 3)
        bal = R.synthetic_balances(n, seed + 3)
        rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(dev)
        dbal = torch.from_numpy(bal.view(np.uint8).copy()).to(dev)
        # registry.DeviceStateHasher (schedule "level1"): one launch for the
        # struct roots and both trees' level-1 windows, then the two trees'
        # top levels side by side, the second finisher hashing
        # Keccak(reg_root || bal_root).  PRYSM_C3_SCHED=list|two: the other
        # schedules (A/B only)
        hasher = R.DeviceStateHasher(n, dev, schedule=os.environ.get("PRYSM_C3_SCHED", "level1"))

        def step():
            return hasher.submit(rec, dbal)

        out = hasher.out
        sec = _timeit(step, args.steps, args.warmup)
        got = bytes(out.cpu().numpy())
        assert got == R.state_root(reg, bal), "c3 root mismatch vs host-buffer path"
        # perms: 3 field hashes + 2 struct blocks per validator, registry + balances merkle, final
        perms = 5 * n + (n / 4 / 2) * 2 + n / 8 + (n / 16 / 2) * 2 + n / 32 + 1
        hashes = 4 * n + n / 8 + n / 8 + n / 32 + n / 32 + 1
        cpu = None
        if not args.no_cpu_baseline:
            from oracle import oracle as O

            m = 1 << 17
            raw = reg.records[:m].view(np.uint8).reshape(-1)
            t0 = time.perf_counter()
            rr = O.struct_roots(raw, m, 160, R.VALIDATOR_FIELDS, nthreads=1)
            O.merkle_hash_flat(rr.reshape(-1), m, 32)
            O.merkle_hash_flat(bal[:m].view(np.uint8), m, 8)
            dt = time.perf_counter() - t0
            cpu = {"value": m / dt, "unit": "validators/s", "cores": 1, "kind": "port", "cpu_model": _cpu_model(),
                   "sample": f"oracle struct_roots + merkleHash, 2^17 validators + balances, 1 thread, {dt:.1f} s"}
        _line("TreeHash of a 1M-validator State (registry + balances)", n / sec, "validators/s", args, sec, perms, hashes,
              {"workload": "C3: synthetic State{[]*ValidatorRecord, []uint64}, 1,000,000 validators",
               "n": n, "root": got.hex(), "schedule": hasher.schedule}, cpu)
        return

    if args.config == "c4tree":
        # SURVEY 8(d)'s C4 secondary: ssz.TreeHash([][32]byte) of 2^28
        # elements (8 GiB in HBM) = merkleHash over Keccak(le32(32) || e_i):
        # +2^28 permutations on top of C4 (x3.67 the work), element digests
        # fused into the leaf pass (k_reduce_elem); one call per step.
        import json as _json

        g = _json.load(open(os.path.join(ROOT, "tests", "golden", "full_size_roots.json")))["c4tree"]
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
        leaf_ops = (lperms / nl) * OPS_PER_PERM - (lhashes / nl) * OPS_SAVED_PER_HASH
        # the element pass this build runs (mk_version carries MK_ELEM_LOCK;
        # the locked form needs n % 8 == 0 and n >= 2^23, true at 2^28)
        if "elem_lock=1" in _lib.load().mk_version().decode():
            kname = "k_elem_lock"
            kdesc = ("k_elem_lock (phase-locked element windows: 1024-thread workgroups, s_barrier in every Keccak "
                     "round; 8 element digests + the window hash per thread, 10 permutations; coalesced LDS-DMA "
                     "staging)")
        else:
            kname = "k_reduce_elem"
            kdesc = "k_reduce_elem<FAST> (8 element digests + window + pair level + 3 LDS levels)"
        from bench import load_pmc

        traffic, clk, pmc_src = load_pmc(kname)
        cpu = None
        if not args.no_cpu_baseline:
            from oracle import oracle as O

            m = 1 << 23
            host = O.splitmix_bytes(m * el, g["seed"])
            t0 = time.perf_counter()
            O.tree_hash_bytes_list(host, m, el, nthreads=1)
            dt = time.perf_counter() - t0
            cpu = {"value": m / dt, "unit": "leaves/s", "cores": 1, "kind": "port", "cpu_model": _cpu_model(),
                   "sample": f"oracle elem digests + merkleHash, 2^23 x 32-B elements (same stream), 1 thread, "
                             f"{dt:.1f} s"}
        _line("tree-hash leaves/sec @2^28 chunks, TreeHash([][32]byte) (element digests + merkleHash)", n / sec,
              "leaves/s", args, sec, perms, hashes,
              {"workload": "C4 secondary: ssz.TreeHash of 2^28 x [32]byte elements (8 GiB), one device call, "
                           "element digests fused into the leaf pass", "n": n, "elem_len": el, "root": root,
               "root_matches_golden": True},
              cpu, {"kernel": kdesc, "traffic": traffic, "traffic_source": pmc_src, "effective_clock_GHz": clk,
                    "leaf_kernel_ms": leaf_s * 1e3, "leaf_kernel_achieved": leaf_ops / leaf_s / 1e12,
                    "leaf_kernel_frac": leaf_ops / leaf_s / PEAK_INT_OPS,
                    "leaf_perms_per_launch": lperms / nl, "leaf_hashes_per_launch": lhashes / nl,
                    "perms_per_leaf": perms / n, "hbm_GBps_algorithmic": n * el / leaf_s / 1e9})
        return

    if args.config == "c5":
        n, dl, depth = 1 << 20, 280, 32
        data = torch.empty(n * dl, dtype=torch.uint8, device=dev)
        D.synth_fill(data, seed + 5)
        lv = torch.empty(L.mk_deposit_trie_levels_bytes(n, depth), dtype=torch.uint8, device=dev)
        root = torch.empty(32, dtype=torch.uint8, device=dev)
        one = lambda: _lib.check(L.mk_dev_deposit_trie_append(None, P(lv), n, 0, P(data), None, n, dl, depth,  # noqa
                                                               P(root), st()), "c5")
        sec_one = _timeit(one, args.steps, args.warmup)  # one trie: leaves, levels, top, in order
        one_root = bytes(root.cpu().numpy())
        # a stream of tries (TriePipeline, front "pipe" at this shape): trie
        # i's leaves and levels 1-2 in one phase-locked launch that also builds
        # levels 3-7 of trie i-1; trie i-1's top (levels 8-32, root) on a
        # high-priority side stream beside trie i+1's front.  The last trie's
        # top (flush) runs inside the timed region.  PRYSM_C5_FRONT=split: the
        # round-3 form (A/B).
        from prysm_amd.pipeline import TriePipeline

        pipe = TriePipeline(n, dl, depth, dev, front=os.environ.get("PRYSM_C5_FRONT", "auto"))
        got = pipe.submit(data)
        pipe.flush()
        torch.cuda.synchronize()
        if bytes(got.cpu().numpy()) != one_root:
            raise SystemExit("c5: pipelined root differs from the one-call root")
        front = "pipe" if pipe._last_pipe else "split"
        for _ in range(args.warmup):
            pipe.submit(data)
        pipe.flush()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            got = pipe.submit(data)
        pipe.flush()
        torch.cuda.synchronize()
        sec = (time.perf_counter() - t0) / args.steps
        if bytes(got.cpu().numpy()) != one_root:
            raise SystemExit("c5: last pipelined root differs from the one-call root")
        perms = 3 * n + (n - 1) + (depth - 20)
        hashes = n + (n - 1) + (depth - 20)
        cpu = None
        if not args.no_cpu_baseline:
            from oracle import oracle as O

            # SURVEY 8d / BASELINE.md 3: both CPU algorithms on 2^17 deposits,
            # the reference's incremental UpdateDepositTrie (1 + 32 hashes per
            # deposit) and the batch form (1 + ~1 per deposit)
            m = 1 << 17
            host = O.splitmix_bytes(m * dl, seed + 5)
            deps = [bytes(host[i * dl:(i + 1) * dl]) for i in range(m)]
            t0 = time.perf_counter()
            r_inc = O.deposit_trie_incremental_root(deps)
            dt_inc = time.perf_counter() - t0
            t0 = time.perf_counter()
            r_bat, _ = O.deposit_trie_levels(deps)
            dt = time.perf_counter() - t0
            assert r_inc == r_bat
            cpu = {"value": m / dt_inc, "unit": "deposits/s", "cores": 1, "kind": "port",
                   "cpu_model": _cpu_model(),
                   "sample": f"oracle or_deposit_trie_incremental (the reference's UpdateDepositTrie loop, "
                             f"35 perms/deposit), 2^17 x 280-B deposits, 1 thread, {dt_inc:.1f} s",
                   "batch_form": {"value": m / dt, "unit": "deposits/s", "cores": 1,
                                  "sample": f"oracle or_deposit_trie_build (batch, ~4 perms/deposit), the same "
                                            f"2^17 deposits, 1 thread, {dt:.2f} s"}}
        _line("deposit trie build, 2^20 x 280-B deposits, depth 32", n / sec, "deposits/s", args, sec, perms, hashes,
              {"workload": "C5: trieutil deposit trie, 2^20 synthetic 280-B deposits (stream of tries, "
                           "each trie's top overlapping the next trie's leaves)", "n": n,
               "root": one_root.hex(), "pipelined": True, "front": front,
               "split_level": pipe.split if front == "split" else TriePipeline.PIPE_TOP_FROM,
               "single_trie_ms": sec_one * 1e3}, cpu)
        return


import numpy as np  # noqa: E402
