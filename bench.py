"""Headline benchmark: ssz.merkleHash of 2^28 x 32-B synthetic items (8 GiB,
BASELINE.json configs[3]) on N MI355X, subtree-sharded.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--log2n 28] [--item-len 32]
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
  python bench.py --gpus N --single-process      (one process, N devices: the cgo caller's form)

With --gpus N > 1 and no WORLD_SIZE in the environment, bench.py launches
itself as N ranks (torch.distributed.run as a child process, started before
this process touches the GPU) and exits with the child's status.

One step = one complete Merkleization of the whole tree.  N = 1 (default):
one stream, the persistent phase-locked leaf pass then the node passes and
the length mix-in (device.merkle_hash).  N > 1: every rank reduces its shard
to the level 10 below its shard root (1024 nodes, the "frontier"), one
32-KB-per-rank RCCL all-gather, rank 0 finishes the top levels and the
length mix-in; with --pipeline 1 (the N > 1 default) each rank's node passes
down to its frontier, the all-gather and rank 0's finisher run on a side
stream that overlaps the next step's leaf pass (parallel.ShardedMerklePipeline;
at N = 1, --pipeline 1 splits the tree at the leaf pass's output level,
prysm_amd/pipeline.py: 1.0-1.9 % slower than one stream on one GPU, two boxes).
The pipelined root is checked against the one-stream root before timing, and
every step's work completes inside the timed region.  Inputs are generated on the device before timing and
stay resident in HBM.  Total work is fixed as N grows ("strong" scaling);
value = 2^log2n leaves x K / max-over-ranks wall time.  Rank 0 prints one
JSON line; progress goes to stderr.

N = 1: after the timed region, the CPU baseline (the oracle's C port with the
unrolled permutation, oracle/keccak_fast.c) and every other BASELINE config
(C2, C3, C5, C1: tools/bench_configs.py, device-resident, 200 timed steps
each, roots checked against tests/golden/full_size_roots.json) go into the
same line (`side_configs`).  N > 1: rank 0 also times the whole tree on its
GPU alone after the timed region (`single_gpu_ms`), and the line carries
`parallel_efficiency`, every rank's leaf fraction and the aggregate fraction.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

INT_OPS_PER_PERM = 4320  # 24 rounds x 180 int32 VALU ops
# A hash's final permutation only has to produce the 32-B digest: its last round
# needs theta on the 5 diagonal lanes and chi on 4 (58 ops, not 180).
INT_OPS_SAVED_PER_HASH = 122
# gfx950 integer VALU peak: 256 CU x 4 SIMD x 32 lanes x 2.4 GHz (MI355X_MICROARCH.md:
# SIMD-32, 2-cycle wave64 issue; = FP32 vector peak 157.3 TFLOPS / 2 flops per FMA).
PEAK_INT_OPS = 256 * 4 * 32 * 2.4e9
SEED = 0x5EED000000000000 + 4  # seed = 0x5EED.. + config_id


def log(*a):
    print("[bench]", *a, file=sys.stderr, flush=True)


def cpu_model() -> str:
    """The host CPU's model name (state the CPU model)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def tree_work(n: int, item_len: int):
    """(permutations, hashes) of merkleHash over n items of item_len bytes
    (shared/ssz/hash.go:194-239): every message of m bytes
    costs m // 136 + 1 permutations; the algorithmic op count of the whole
    tree is perms x 4320 - hashes x 122."""
    def p(m):
        return m // 136 + 1

    cb = (128 // item_len) * item_len if item_len < 128 else item_len
    total = n * item_len
    full, rem = divmod(total, cb)
    count = full + (1 if rem else 0)
    if count <= 1:  # a single (or empty: 0^128) chunk is the root's input
        return p((rem or cb if n else 128) + 32), 1
    pairs = count // 2
    if count % 2:  # the last chunk alone, padded with 0^128
        perms = pairs * p(2 * cb) + p((rem or cb) + 128)
    else:
        perms = (pairs - 1) * p(2 * cb) + p(cb + (rem or cb))
    hashes = count = (count + 1) // 2
    while count > 1:  # 64-B node pairs; an odd node + 0^128 is 160 B
        perms += count // 2 + (2 if count % 2 else 0)
        count = (count + 1) // 2
        hashes += count
    return perms + 1, hashes + 1  # the length mix-in K(root || le64(n) || 0^24)


def cpu_baseline(item_len: int, log2n_sample: int, threads: int = 1):
    """The oracle (a C port of hash.go:194-239; 1 thread = the reference's
    single-goroutine shape, more threads split the tree by subtrees) on a
    bounded sample of the same workload, with the unrolled permutation
    (oracle/keccak_fast.c: the 25-locals, rounds-unrolled shape of the
    x/crypto keccakF1600 the reference runs, WORKSPACE:542-546)."""
    from oracle import oracle as O

    n = 1 << log2n_sample
    items = O.splitmix_bytes(n * item_len, SEED)
    perms, _ = tree_work(n, item_len)
    with O.fast_permutation():
        t0 = time.perf_counter()
        O.merkle_hash_flat(items, n, item_len, nthreads=threads)
        dt = time.perf_counter() - t0
    ns = dt / perms * 1e9 * threads
    return {"value": n / dt, "unit": "leaves/s", "cores": threads, "kind": "port", "cpu_model": cpu_model(),
            "ns_per_perm": ns,
            "sample": f"oracle/merkle_ref.c or_merkle_hash, 2^{log2n_sample} x {item_len}-B items "
                      f"(same SplitMix64 stream, {perms} perms), unrolled permutation (oracle/keccak_fast.c), "
                      f"{threads} thread{'s' if threads > 1 else ''}, {dt:.1f} s, {ns:.0f} ns per permutation"
                      f"{' per thread' if threads > 1 else ''}"}


def leaf_kernel():
    """(kernel-name substring, description) of the C4 leaf pass this library
    build runs (mk_version carries the compile-time knobs)."""
    from prysm_amd import _lib

    v = _lib.load().mk_version().decode()
    if "leaf_lock=1" in v:
        return ("k_leaf_lock_sc",
                "k_leaf_lock_sc (phase-locked leaf pass: 1024-thread workgroups, s_barrier in every Keccak round; "
                "4 windows -> 1 node per thread, 3 levels; coalesced LDS-DMA staging)")
    return "k_reduce<true, true, 2>", "k_reduce<LEAF, FAST, 2> (leaf pass: 256-B windows + 4 fused levels)"


def load_pmc(kernel):
    """HBM bytes per leaf-kernel launch and the effective clock under that
    load from the newest committed rocprofv3 PMC summary of this leaf kernel
    (profiles/*_pmc.json, tools/pmc_summary.py), with the file they come
    from.  These are NOT measured by this run (PMC counters need their own
    rocprofv3 pass)."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        if d.get("kernel", "k_reduce<true, true, 2>") != kernel:
            continue
        return (d.get("hbm_bytes_per_leaf_launch"), d.get("effective_clock_GHz"),
                os.path.relpath(path, ROOT) + f" ({d.get('box', 'builder lease')}, not this run)")
    return None, None, None


class ClockSampler:
    """Samples this GPU's current shader clock (sysfs pp_dpm_sclk, the line
    marked '*') every ~2 ms on a host thread while the timed steps run.
    OFF unless PRYSM_BENCH_SCLK=1: each read is a query to the power-
    management firmware, and sampling slowed the measured GPU itself (C2
    1.54 -> 1.82 ms, C4 9.76-9.85 -> 10.06-10.07 ms, alternating runs on one
    box, profiles/r02z2/ab.txt), so the default bench line carries only the
    committed PMC clock.  Host-side only; None where the file is absent."""

    def __init__(self, dev_index: int):
        import threading

        import torch

        self.path = None
        if os.environ.get("PRYSM_BENCH_SCLK") != "1":
            self.samples, self._t = [], None
            return
        try:
            p = torch.cuda.get_device_properties(dev_index)
            bdf = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
            path = f"/sys/bus/pci/devices/{bdf}/pp_dpm_sclk"
            if self._read(path) is not None:
                self.path = path
        except Exception:
            pass
        self.samples = []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True) if self.path else None

    @staticmethod
    def _read(path):
        try:
            with open(path) as f:
                for line in f:
                    if line.rstrip().endswith("*"):
                        return float(line.split(":", 1)[1].strip().split("Mhz")[0].split("MHz")[0])
        except (OSError, ValueError, IndexError):
            return None
        return None

    def _run(self):
        while not self._stop.is_set():
            v = self._read(self.path)
            if v is not None:
                self.samples.append(v)
            self._stop.wait(0.002)

    def start(self):
        if self._t:
            self._t.start()

    def stop(self):
        if self._t:
            self._stop.set()
            self._t.join()
        if not self.samples:
            return None
        xs = sorted(self.samples)
        return {"mean_MHz": sum(xs) / len(xs), "median_MHz": xs[len(xs) // 2], "min_MHz": xs[0],
                "max_MHz": xs[-1], "samples": len(xs), "source": self.path}


def golden_root(log2n: int, item_len: int):
    """The committed oracle root of this exact workload, if there is one
    (tests/golden/full_size_roots.json: 2^28 x 32 B, seed 0x5EED..04)."""
    try:
        with open(os.path.join(ROOT, "tests", "golden", "full_size_roots.json")) as f:
            g = json.load(f)["c4"]
    except (OSError, KeyError, ValueError):
        return None
    return g["root"] if (g["n"], g["item_len"], g["seed"]) == (1 << log2n, item_len, SEED) else None


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(nproc: int, argv, script: str = None) -> int:
    """Runs `script argv` as nproc ranks of one node (torch.distributed.run,
    127.0.0.1 rendezvous) in a child process and returns its exit status.
    Called before this process has touched the GPU (it never execs)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", script or os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this pool
    log(f"launching {nproc} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    # sub-millisecond steps (C1/C3/C5) need ~10-20 ms of work before the
    # clocks settle: C5 0.559 ms/step after 3 warmup steps, 0.478 after 30;
    # the 10-ms C4 step is the same after 3 or 20 (profiles/r02d/warmup.txt)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--log2n", type=int, default=28)
    ap.add_argument("--item-len", type=int, default=32)
    ap.add_argument("--cpu-sample-log2n", type=int, default=27)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-side-configs", action="store_true",
                    help="N = 1: skip the C2/C3/C5/C1 side configs after the C4 line's own measurements")
    ap.add_argument("--side-steps", type=int, default=200)
    ap.add_argument("--side-warmup", type=int, default=40)
    ap.add_argument("--no-single-gpu", action="store_true",
                    help="N > 1: skip rank 0's single-GPU run of the whole tree (parallel_efficiency)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="collective backend (nccl = RCCL over xGMI; gloo only to rehearse N ranks on one GPU)")
    ap.add_argument("--share-device", action="store_true",
                    help="all ranks on cuda:0 (rehearsal of the N-rank path on a one-GPU box, with --backend gloo)")
    ap.add_argument("--frontier", type=int, default=10,
                    help="N>1: each rank gathers its tree level this many levels below its shard root "
                         "(2^k nodes) and rank 0 finishes the top (0 = gather the 32-B shard roots)")
    ap.add_argument("--pipeline", type=int, default=-1, choices=[-1, 0, 1],
                    help="1: everything above the leaf pass (5 levels above the chunks) runs on a side stream "
                         "overlapping the next step's leaf pass: N=1 the node passes and the length mix-in "
                         "(prysm_amd/pipeline.py), N>1 each rank's node passes, the all-gather and rank 0's "
                         "finisher (parallel.ShardedMerklePipeline).  0 = one stream.  -1 (default): 0 at N = 1 "
                         "(the one-stream tree with the persistent locked leaf pass measured 1.0-1.9 %% faster than "
                         "the pipelined form on two boxes, DESIGN.md §6), 1 at N > 1")
    ap.add_argument("--config", default="c4", choices=["c1", "c2", "c3", "c4", "c4tree", "c5"],
                    help="BASELINE.json config: c4 = headline (default); c1/c2/c3/c5 = single-GPU side benches; "
                         "c4tree = the C4 secondary, TreeHash([][32]byte) of 2^28 elements")
    ap.add_argument("--single-process", action="store_true",
                    help="N devices from one process through mk_dev_ssz_merkle_hash_multi (the cgo caller's "
                         "form: one shard per device, RCCL all-gather inside the library)")
    args = ap.parse_args()
    if args.config == "c5" and args.gpus > 1:  # SURVEY §8e's C5 split over N ranks
        if "WORLD_SIZE" not in os.environ:
            return launch_ranks(args.gpus, sys.argv[1:])
    elif args.config != "c4":
        from tools.bench_configs import run_config

        return run_config(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and not args.single_process:
        return launch_ranks(args.gpus, sys.argv[1:])
    if args.single_process:
        return run_single_process(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"ERROR: --gpus {args.gpus} but WORLD_SIZE {world}")
        return 2
    if args.share_device:
        local = 0
    body = run_c5_ranks if args.config == "c5" else run_ranks
    if world == 1:
        return body(args, world, rank, local)
    # N ranks: every failure (a rank that never joins, a collective that
    # times out after parallel.dist_timeout(), a HIP/RCCL error) ends this rank
    # with an error JSON line and a non-zero status instead of a silent hang;
    # a host-side deadline covers whatever the timeouts do not
    watchdog = Deadline(float(os.environ.get("PRYSM_BENCH_DEADLINE", "900")),
                        lambda: error_line(args, world, rank, "deadline exceeded (PRYSM_BENCH_DEADLINE)"))
    try:
        return body(args, world, rank, local)
    except Exception as e:  # noqa: BLE001 -- reported, then the rank fails
        error_line(args, world, rank, f"{type(e).__name__}: {e}")
        return 3
    finally:
        watchdog.cancel()


class Deadline:
    """Host-side last resort for the N-rank run: after `seconds` it prints the
    error line and ends the process with status 124 (os._exit: no exec, and
    no further GPU call from this thread)."""

    def __init__(self, seconds: float, report):
        import threading

        self._t = threading.Timer(seconds, self._fire, args=(report,))
        self._t.daemon = True
        self._t.start()

    @staticmethod
    def _fire(report):
        report()
        os._exit(124)

    def cancel(self):
        self._t.cancel()


def error_line(args, world: int, rank: int, msg: str) -> None:
    """The JSON record of a failed N-rank run (rank 0 on stdout, the other
    ranks on stderr, so the driver still reads one line)."""
    rec = {"metric": "tree-hash leaves/sec @2^28 chunks (ssz.merkleHash, 32-B leaves)", "value": None,
           "unit": "leaves/s", "n_gpus": args.gpus, "world_size": world, "rank": rank,
           "backend": args.backend, "error": msg[:2000]}
    log(f"rank {rank}: ERROR {msg[:2000]}")
    print(json.dumps(rec), file=sys.stdout if rank == 0 else sys.stderr, flush=True)


def run_ranks(args, world: int, rank: int, local: int) -> int:
    """One rank of the headline bench (world == 1: the only one)."""
    import torch
    import torch.distributed as dist

    from prysm_amd import parallel as P

    if world > 1 and args.backend == "gloo":  # no device needed to rendezvous
        P.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 and args.backend == "nccl":
        P.init_process_group("nccl", dev)
    from prysm_amd import device as D

    if world > 1:  # what actually initialised, for the record
        world_pg, backend_pg = dist.get_world_size(), str(dist.get_backend())
        if world_pg != world:
            raise RuntimeError(f"process group has {world_pg} ranks, WORLD_SIZE is {world}")
    else:
        world_pg, backend_pg = 1, None

    n, item_len = 1 << args.log2n, args.item_len
    sp = P.plan(n, item_len, world)
    lo, hi = sp.items(rank)
    local_n = hi - lo
    nbytes = local_n * item_len
    items = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=dev)
    if nbytes:
        assert (lo * item_len) % 8 == 0 and nbytes % 8 == 0
        D.synth_fill(items[:nbytes], SEED, word0=lo * item_len // 8)
    ws = D.subtree_workspace(local_n, item_len, dev) if sp.nonempty > 1 else D.merkle_workspace(n, item_len, dev)
    root_buf = torch.empty(32, dtype=torch.uint8, device=dev)
    # frontier: the narrowest (latency-bound) k levels of every shard move to
    # rank 0's finisher, which overlaps its next step (parallel.py)
    k = args.frontier if sp.nonempty > 1 and 0 < args.frontier < sp.height - 4 else 0
    block = 32 << k
    frontier_buf = torch.empty(block, dtype=torch.uint8, device=dev)
    gather_buf = torch.empty(world * block, dtype=torch.uint8, device=dev)
    finish_out = torch.empty(32, dtype=torch.uint8, device=dev)
    finish_ws = D.finish_workspace(world << k, dev) if k and rank == 0 else None
    # rank 0 finishes the top levels on a side stream, overlapping its next step
    finish_stream = torch.cuda.Stream(device=dev, priority=-1) if world > 1 and rank == 0 else None
    torch.cuda.synchronize()
    log(f"rank {rank}/{world}: {local_n} items ({nbytes / 2**30:.2f} GiB), shard height {sp.height}, "
        f"nonempty {sp.nonempty}, frontier {k}")

    # N > 1: hipEvent marks of the rank step's phases (leaf pass, node passes
    # to the frontier, all-gather, finisher), recorded during the timed steps
    timer = P.PhaseTimer(cuda=True) if world > 1 else None

    def step_one_stream(t=None):
        return P.sharded_merkle_hash(
            items, n, item_len, sp, rank, world,
            subtree_fn=lambda it, sn, il, h, pad: D.merkle_subtree(it, sn, il, h, pad, out=root_buf, ws=ws),
            full_fn=lambda it, nn, il: D.merkle_hash(it, nn, il, out=root_buf, ws=ws),
            finish_fn=lambda g, nr, nt: D.merkle_finish(g, nr, nt, out=finish_out),
            gather_buf=gather_buf, finish_stream=finish_stream, frontier_log2=k,
            frontier_fn=lambda it, sn, il, h, kk, pad: D.merkle_subtree_frontier(it, sn, il, h, kk, pad,
                                                                                 out=frontier_buf, ws=ws),
            finish_nodes_fn=lambda g, c, nt: D.merkle_finish_nodes(g, c, nt, out=finish_out, ws=finish_ws),
            timer=t)

    # --pipeline: everything above the leaf pass of step i runs on a side
    # stream that overlaps step i+1's leaf pass (N = 1: pipeline.py; N > 1:
    # node passes, the all-gather and rank 0's finisher, parallel.py)
    pipe = None
    if args.pipeline < 0:
        args.pipeline = 1 if world > 1 else 0
    if args.pipeline > 0:
        if world == 1:
            from prysm_amd.pipeline import MerklePipeline

            pipe = MerklePipeline(n, item_len, dev)
            k = pipe.k
        else:
            pipe = P.ShardedMerklePipeline(n, item_len, sp, rank, world, dev, gather_log2=k, workspace=ws,
                                           timer=timer)
            pipe = pipe if pipe.ok else None
    if pipe is not None:
        # the pipelined root must equal the one-stream root of the same items
        want = step_one_stream()
        torch.cuda.synchronize()
        want = bytes(want.cpu().numpy()) if want is not None else None
        got = pipe.submit(items)
        torch.cuda.synchronize()
        same = torch.ones(1, dtype=torch.int32, device=dev if args.backend == "nccl" else "cpu")
        if rank == 0 and bytes(got.cpu().numpy()) != want:
            same.zero_()
        if world > 1:  # every rank takes the same path
            dist.all_reduce(same, op=dist.ReduceOp.MIN)
        if not same.item():  # never expected (tests pin the split): a wrong root is a failed run
            log(f"rank {rank}: ERROR pipelined root differs from the one-stream root")
            if world > 1:
                dist.destroy_process_group()
            return 1
        log(f"rank {rank}: pipelined (frontier {k}), the levels above the leaf pass on a side stream")

    def step():
        return pipe.submit(items) if pipe is not None else step_one_stream(timer)

    for i in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    root_hex = None

    status = 0
    D.prof_enable(True)
    D.prof_read()  # reset
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    sampler = ClockSampler(local)
    sampler.start()
    if timer is not None:
        timer.steps.clear()  # warmup steps were not marked (start_step not called)
    t0 = time.perf_counter()
    last_log = t0
    for i in range(args.steps):
        if timer is not None:
            timer.start_step()
        r = step()
        if time.perf_counter() - last_log > 30:
            log(f"step {i + 1}/{args.steps}")
            last_log = time.perf_counter()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    sclk = sampler.stop()
    D.prof_enable(False)
    leaf_ms, leaf_launches, leaf_perms, leaf_hashes = D.prof_read()
    if rank == 0 and r is not None:
        root_hex = bytes(r.cpu().numpy()).hex()
        want = golden_root(args.log2n, item_len)
        if want is not None and root_hex != want:
            log(f"ERROR: root {root_hex} != golden {want}")
            status = 1

    if timer is not None:
        timer.stop()  # no marks after the timed region
    phases = timer.record(world, dev if args.backend == "nccl" else None) if timer is not None else None
    # N = 1: the latency of one complete Merkleization (one stream, not
    # pipelined), hipEvents over >= 20 runs, after the timed region
    single_tree_ms = None
    if world == 1:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        runs = max(20, args.steps)
        step_one_stream()
        e0.record()
        for _ in range(runs):
            step_one_stream()
        e1.record()
        torch.cuda.synchronize()
        single_tree_ms = e0.elapsed_time(e1) / runs

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
    per_rank = per_rank_leaf_frac = None
    nl = max(leaf_launches, 1)
    if world > 1:
        # every rank's step time, leaf-kernel launch average and the ops of
        # its average leaf launch, for the record
        mine = torch.tensor([elapsed / args.steps * 1e3, leaf_ms / nl,
                             leaf_perms / nl * INT_OPS_PER_PERM - leaf_hashes / nl * INT_OPS_SAVED_PER_HASH],
                            dtype=torch.float64, device=t.device)
        allr = torch.empty(world * 3, dtype=torch.float64, device=t.device).view(world, 3)
        dist.all_gather_into_tensor(allr.view(-1), mine)
        rows = allr.tolist()
        per_rank = [[round(r[0], 4), round(r[1], 4)] for r in rows]
        per_rank_leaf_frac = [round(r[2] / (r[1] / 1e3) / PEAK_INT_OPS, 4) if r[1] > 0 else None for r in rows]
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    t_max = t.item()
    # N > 1: the same whole tree on rank 0's GPU alone (one stream, the
    # N = 1 bench's step, same steps/warmup), after the timed region, so the
    # line carries its own strong-scaling efficiency t_1 / (N t_N)
    single_gpu_ms = None
    if world > 1 and rank == 0 and not args.no_single_gpu:
        single_gpu_ms = single_gpu_step_ms(args, dev, n, item_len)

    if rank == 0:
        value = n * args.steps / t_max
        avg_leaf_s = (leaf_ms / 1e3) / max(leaf_launches, 1)
        perms_per_launch = leaf_perms / max(leaf_launches, 1)
        hashes_per_launch = leaf_hashes / max(leaf_launches, 1)
        ops_per_launch = perms_per_launch * INT_OPS_PER_PERM - hashes_per_launch * INT_OPS_SAVED_PER_HASH
        achieved = ops_per_launch / avg_leaf_s if avg_leaf_s > 0 else 0.0
        kname, kdesc = leaf_kernel()
        traffic, clk, pmc_src = load_pmc(kname) if args.log2n == 28 else (None, None, None)
        if traffic is not None and world > 1:  # the committed PMC is of a whole 2^28 leaf launch
            traffic *= local_n / n
            pmc_src += f", scaled by this rank's {local_n}/{n} of the leaves"
        step_s = t_max / args.steps
        tree_perms, tree_hashes = tree_work(n, item_len)
        tree_ops = tree_perms * INT_OPS_PER_PERM - tree_hashes * INT_OPS_SAVED_PER_HASH
        out = {
            "metric": "tree-hash leaves/sec @2^28 chunks (ssz.merkleHash, 32-B leaves)",
            "value": value,
            "unit": "leaves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "u64 (Keccak lanes as u32 pairs)",
            "data": "synthetic (device SplitMix64, seed 0x5EED000000000004)",
            "config": {"workload": f"C4: ssz.merkleHash of 2^{args.log2n} x {item_len}-B items "
                                   f"({n * item_len / 2**30:.0f} GiB), subtree-sharded",
                       "n_items": n, "item_len": item_len, "parallelism": f"subtree{world}",
                       "shard_height": sp.height, "frontier_log2": k, "pipelined": pipe is not None and k > 0,
                       "root": root_hex, "root_matches_golden": None if golden_root(args.log2n, item_len) is None
                       else root_hex == golden_root(args.log2n, item_len),
                       "backend": backend_pg, "world_size": world_pg, "share_device": bool(args.share_device),
                       "per_rank_ms_per_step_and_leaf_ms": per_rank,
                       # one complete Merkleization alone (N = 1: one stream, not pipelined)
                       "single_tree_ms": single_tree_ms,
                       # N > 1: rank 0's phases of the step and every rank's [leaf, nodes, gather,
                       # finish] (parallel.PhaseTimer; pipelined: nodes/gather/finish overlap the
                       # next leaf pass, so their sum exceeds ms_per_step)
                       "phases_ms": phases["phases_ms"] if phases else None,
                       "per_rank_phases_ms": phases["per_rank_phases_ms"] if phases else None,
                       # every rank's leaf-kernel fraction of one GPU's peak (its own launches)
                       "per_rank_leaf_frac": per_rank_leaf_frac,
                       # N > 1: the whole tree on rank 0's GPU alone, same steps, after the timed
                       # region; parallel_efficiency = single_gpu_ms / (N x ms_per_step)
                       "single_gpu_ms": single_gpu_ms,
                       "parallel_efficiency": (single_gpu_ms / (world * step_s * 1e3)
                                               if single_gpu_ms else None)},
            "roofline": {
                "bound": "valu-int",
                "kernel": kdesc,
                "achieved": achieved / 1e12,
                "peak": PEAK_INT_OPS / 1e12,
                "unit": "Tops/s (int32 VALU)",
                "frac": achieved / PEAK_INT_OPS,
                "traffic": traffic,
                # also against the sustained clock the PMC run measured under this load
                "effective_clock_GHz": clk,
                "traffic_source": pmc_src,
                "frac_at_effective_clock": achieved / (PEAK_INT_OPS / 2.4 * clk) if clk else None,
                # this run's own clock (rank 0's GPU) from sysfs, only with PRYSM_BENCH_SCLK=1
                "sclk_sampled": sclk,
                "frac_at_sampled_clock": (achieved / (PEAK_INT_OPS / 2.4e3 * sclk["mean_MHz"])
                                          if sclk and sclk["mean_MHz"] > 0 else None),
                "perms_per_launch": perms_per_launch,
                "hashes_per_launch": hashes_per_launch,
                "avg_launch_ms": avg_leaf_s * 1e3,
                "hbm_GBps_algorithmic": (local_n * item_len) / avg_leaf_s / 1e9 if avg_leaf_s > 0 else None,
                # the whole step: the tree's algorithmic ops (tree_work) / (step time x N GPUs x peak)
                "tree_perms": tree_perms,
                "step_frac_aggregate": tree_ops / (step_s * world * PEAK_INT_OPS),
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline ...")
            out["cpu_baseline"] = cpu_baseline(item_len, args.cpu_sample_log2n)
            # also the restatement on the host's share of cores (16 on the GPU box)
            nt = min(16, len(os.sched_getaffinity(0)))
            out["cpu_baseline_threads"] = cpu_baseline(item_len, args.cpu_sample_log2n, threads=nt)
        if world == 1 and not args.no_side_configs:
            # every other BASELINE config, device-resident, >= 100 steps each,
            # roots against tests/golden/full_size_roots.json (tools/bench_configs.py)
            from tools.bench_configs import side_configs

            del items, ws
            pipe = None
            torch.cuda.empty_cache()
            log("side configs ...")
            out["side_configs"] = side_configs(dev, steps=args.side_steps, warmup=args.side_warmup,
                                               cpu=not args.no_cpu_baseline)
            if not all(e.get("root_matches_golden") for e in out["side_configs"].values()):
                log("ERROR: a side config's root differs from its golden (or it failed)")
                status = 1
        print(json.dumps(out), flush=True)
    if world > 1:
        st = torch.tensor([status], dtype=torch.int32, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        status = int(st.item())
        dist.destroy_process_group()
    return status


def single_gpu_step_ms(args, dev, n: int, item_len: int) -> float:
    """ms per step of the whole n-item tree on this GPU alone: the N = 1
    bench's step (one stream, device.merkle_hash), args.warmup untimed and
    args.steps timed steps, wall clock bracketed by synchronize()."""
    import torch

    from prysm_amd import device as D

    log(f"rank 0: the whole 2^{args.log2n} tree on one GPU (parallel_efficiency) ...")
    items = torch.empty(n * item_len, dtype=torch.uint8, device=dev)
    D.synth_fill(items, SEED)
    ws = D.merkle_workspace(n, item_len, dev)
    out = torch.empty(32, dtype=torch.uint8, device=dev)
    for _ in range(args.warmup):
        D.merkle_hash(items, n, item_len, out=out, ws=ws)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = D.merkle_hash(items, n, item_len, out=out, ws=ws)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    want = golden_root(args.log2n, item_len)
    if want is not None and bytes(r.cpu().numpy()).hex() != want:
        raise RuntimeError("single-GPU root differs from the golden root")
    del items, ws
    torch.cuda.empty_cache()
    return ms


def run_c5_ranks(args, world: int, rank: int, local: int) -> int:
    """BASELINE config 5 over N ranks: the depth-32 deposit
    trie of 2^20 x 280-B deposits split by subtree (parallel.trie_plan):
    every rank builds its 2^h-deposit subtree from deposits generated in its
    HBM, one all-gather of 32 B per rank, rank 0 builds the levels above.
    value = deposits of all ranks / max-over-ranks time; strong scaling."""
    import torch
    import torch.distributed as dist

    from prysm_amd import device as D
    from prysm_amd import parallel as P

    if world > 1 and args.backend == "gloo":
        P.init_process_group("gloo")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 and args.backend == "nccl":
        P.init_process_group("nccl", dev)
    n, dl, depth = 1 << 20, 280, 32
    seed = 0x5EED000000000000 + 5
    tp = P.trie_plan(n, world, depth)
    lo, hi = tp.items(rank)
    cnt = hi - lo
    data = torch.empty(max(cnt * dl, 16), dtype=torch.uint8, device=dev)
    if cnt:
        D.synth_fill(data[:cnt * dl], seed, word0=lo * dl // 8)
    sub_h = tp.height if tp.height else depth
    lv = torch.empty(D.deposit_trie_levels_bytes(max(cnt, 1), sub_h), dtype=torch.uint8, device=dev)
    root = torch.zeros(32, dtype=torch.uint8, device=dev)
    gathered = torch.zeros(32 * world, dtype=torch.uint8, device=dev)
    top_lv = torch.zeros(D.deposit_trie_levels_bytes(world, max(depth - tp.height, 1)), dtype=torch.uint8,
                         device=dev)
    out = torch.zeros(32, dtype=torch.uint8, device=dev)
    gloo = world > 1 and args.backend == "gloo"

    def step():
        if cnt:
            D.deposit_trie_build(lv, cnt, data, cnt, dl, sub_h, sub_h, root)
        if world == 1 or tp.height == 0:
            return root
        if gloo:
            host = torch.empty(32 * world, dtype=torch.uint8)
            dist.all_gather_into_tensor(host, root.cpu())
            gathered.copy_(host)
        else:
            dist.all_gather_into_tensor(gathered, root)
        if rank == 0:
            top_lv[:32 * tp.nonempty] = gathered[:32 * tp.nonempty]
            D.deposit_trie_levels(top_lv, world, tp.nonempty, 0, depth - tp.height, depth - tp.height, out)
            return out
        return None

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    status = 0
    if rank == 0:
        got = bytes(r.cpu().numpy()).hex()
        try:
            with open(os.path.join(ROOT, "tests", "golden", "full_size_roots.json")) as f:
                want = json.load(f)["c5"]["root"]
        except (OSError, KeyError, ValueError):
            want = None
        status = 0 if want is None or got == want else 1
        sec = t.item() / args.steps
        print(json.dumps({
            "metric": "deposit trie build, 2^20 x 280-B deposits, depth 32", "value": n / sec, "unit": "deposits/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": sec * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "u64 (Keccak lanes as u32 pairs)", "data": "synthetic (device SplitMix64, seed 0x5EED..05)",
            "config": {"workload": "C5 split by subtree: per-rank 2^h-deposit subtrees, 32-B all-gather, rank-0 top",
                       "n": n, "subtree_height": tp.height, "nonempty": tp.nonempty, "root": got,
                       "root_matches_golden": None if want is None else got == want,
                       "backend": str(dist.get_backend()) if world > 1 else None,
                       "world_size": dist.get_world_size() if world > 1 else 1}}), flush=True)
    if world > 1:
        st = torch.tensor([status], dtype=torch.int32, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(st, op=dist.ReduceOp.MAX)
        status = int(st.item())
        dist.destroy_process_group()
    return status


def run_single_process(args) -> int:
    """One process drives args.gpus devices through the library's
    single-process multi-device entry (mk_dev_ssz_merkle_hash_multi): shard d
    of the subtree plan lives on device d (generated there), every device
    reduces its shard to its 1024-node frontier on its own stream, the
    library all-gathers the frontiers over RCCL and device 0 finishes.  The
    whole step is inside the timed region (all devices synchronised)."""
    import torch

    from prysm_amd import device as D
    from prysm_amd import _lib

    ndev = args.gpus
    if _lib.device_count() < ndev:
        log(f"ERROR: {ndev} devices requested, {_lib.device_count()} visible")
        return 2
    n, item_len = 1 << args.log2n, args.item_len
    h, ne, begin = D.shard_plan(n, item_len, ndev)
    shards = []
    for d in range(ndev):
        nb = (begin[d + 1] - begin[d]) * item_len
        t = torch.empty(max(nb, 16), dtype=torch.uint8, device=f"cuda:{d}")
        if nb:
            D.synth_fill(t[:nb], SEED, word0=begin[d] * item_len // 8)
        shards.append(t)
    out = torch.empty(32, dtype=torch.uint8, device="cuda:0")

    def sync_all():
        for d in range(ndev):
            torch.cuda.synchronize(d)

    sync_all()
    log(f"single process, {ndev} device(s): shard height {h}, {ne} non-empty shards")
    for _ in range(args.warmup):
        D.merkle_hash_multi(shards, n, item_len, out)
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        D.merkle_hash_multi(shards, n, item_len, out)
    sync_all()
    elapsed = time.perf_counter() - t0
    root_hex = bytes(out.cpu().numpy()).hex()
    want = golden_root(args.log2n, item_len)
    res = {"metric": "tree-hash leaves/sec @2^28 chunks (ssz.merkleHash, 32-B leaves)",
           "value": n * args.steps / elapsed, "unit": "leaves/s", "n_gpus": ndev, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
           "scaling": "strong", "vs_baseline": None, "dtype": "u64 (Keccak lanes as u32 pairs)",
           "data": "synthetic (device SplitMix64, seed 0x5EED000000000004)",
           "config": {"workload": f"C4: ssz.merkleHash of 2^{args.log2n} x {item_len}-B items, one process, "
                                  f"mk_dev_ssz_merkle_hash_multi over {ndev} device(s)",
                      "n_items": n, "item_len": item_len, "parallelism": f"subtree{ndev}-single-process",
                      "shard_height": h, "root": root_hex,
                      "root_matches_golden": None if want is None else root_hex == want}}
    print(json.dumps(res), flush=True)
    return 1 if want is not None and root_hex != want else 0


if __name__ == "__main__":
    sys.exit(main())
