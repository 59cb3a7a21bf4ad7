"""The N>1 path (subtree sharding + one all-gather + rank-0 finish) with the
gloo backend on CPU, world_size 2 and 4.  The per-shard compute is the
oracle here (the HIP kernels are covered by tests/test_gpu_parity.py); this
checks the orchestration, the shard plan and the collective."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

SEED = 0x5EED000000000000 + 81


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _plan_cpu(n, item_len, world):
    """Shard plan restated in Python (the C planner is checked against this
    in test_boundary)."""
    per = 128 // item_len if item_len < 128 else 1
    cb = per * item_len
    chunks = -(-n * item_len // cb) if n else 0
    h = 0
    while (1 << h) * world < chunks:
        h += 1
    ne = -(-chunks // (1 << h)) if chunks else 0
    if h == 0 or ne <= 1:
        return h, 1, [0] + [n] * world
    return h, ne, [min(n, s * (1 << h) * per) for s in range(world + 1)]


def _worker(rank, world, port, n, item_len, q, frontier=0, pipe=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import oracle as O
        from prysm_amd import parallel as P

        sp = P.plan(n, item_len, world, plan_fn=_plan_cpu)
        lo, hi = sp.items(rank)
        full = O.splitmix_bytes(n * item_len, SEED)
        local = torch.from_numpy(full[lo * item_len:hi * item_len].copy())

        def subtree(items, sn, il, h, pad):
            # oracle subtree of shard `rank` of the synthetic tree
            return torch.frombuffer(bytearray(O.merkle_subtree_gen(n, il, SEED, rank, h)), dtype=torch.uint8)

        def full_fn(items, nn, il):
            return torch.frombuffer(bytearray(O.merkle_hash_flat(items.numpy(), nn, il)), dtype=torch.uint8)

        def finish(g, nr, nt):
            roots = [bytes(g[32 * i:32 * i + 32].numpy()) for i in range(nr)]
            chunks = roots
            while len(chunks) > 1:
                if len(chunks) % 2:
                    chunks = chunks + [bytes(128)]
                chunks = [O.keccak256(chunks[i] + chunks[i + 1]) for i in range(0, len(chunks), 2)]
            lenc = nt.to_bytes(8, "little") + bytes(24)
            return torch.frombuffer(bytearray(O.keccak256(chunks[0] + lenc)), dtype=torch.uint8)

        def frontier_fn(items, sn, il, h, k, pad):
            # the shard's level k below its root = the roots of its 2^k sub-shards
            cnt = P.frontier_count(sn, il, h, k)
            nodes = b"".join(O.merkle_subtree_gen(n, il, SEED, (rank << k) + j, h - k) for j in range(cnt))
            return torch.frombuffer(bytearray(nodes), dtype=torch.uint8)

        def finish_nodes(g, count, nt):
            return finish(g, count, nt)

        if pipe is not None:  # (gather_log2, leaf_levels[, slots]): ShardedMerklePipeline over several trees
            def node_frontier(level, cnt, hh, kk, pad, out):
                nodes = [bytes(level[32 * i:32 * i + 32].numpy()) for i in range(cnt)]
                for _ in range(hh - kk):  # the odd rule incl. a lone node (pad_at_one)
                    if len(nodes) % 2:
                        nodes = nodes + [bytes(128)]
                    nodes = [O.keccak256(nodes[i] + nodes[i + 1]) for i in range(0, len(nodes), 2)]
                return torch.frombuffer(bytearray(b"".join(nodes)), dtype=torch.uint8)

            pl = P.ShardedMerklePipeline(
                n, item_len, sp, rank, world, "cpu", gather_log2=pipe[0], leaf_levels=pipe[1],
                frontier_fn=lambda it, sn, il, h, k, pad, out: frontier_fn(it, sn, il, h, k, pad),
                node_frontier_fn=node_frontier,
                finish_nodes_fn=lambda g, c, nt, out: finish_nodes(g, c, nt),
                **({"slots": pipe[2]} if len(pipe) > 2 else {}))
            assert pl.ok
            roots = [pl.submit(local) for _ in range(max(3, pl.slots + 2))]
            if rank == 0:
                assert len({bytes(r.numpy()) for r in roots}) == 1
                q.put(bytes(roots[-1].numpy()))
            return
        root = P.sharded_merkle_hash(local, n, item_len, sp, rank, world, subtree_fn=subtree, full_fn=full_fn,
                                     finish_fn=finish, frontier_log2=frontier, frontier_fn=frontier_fn,
                                     finish_nodes_fn=finish_nodes)
        if rank == 0:
            q.put(bytes(root.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 4 * 1000 + 3), (2, 1 << 14), (4, 4 * 37), (4, 9), (4, 1 << 12)])
def test_sharded_root_equals_full_root(world, n):
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 32, q)) for r in range(world)]
    for p in procs:
        p.start()
    root = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert root == O.merkle_hash_gen(n, 32, SEED)


@pytest.mark.parametrize("world,n,k", [(2, 1 << 14, 3), (2, 4 * 1000 + 3, 2), (4, 4 * 1000 + 3, 4), (4, 1 << 12, 5),
                                       (4, 4 * 37, 1)])
def test_frontier_sharded_root_equals_full_root(world, n, k):
    """Frontier mode: ranks gather their 2^k-node level, rank 0 finishes the
    k + log2(world) top levels (ragged last shards included)."""
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 32, q, k)) for r in range(world)]
    for p in procs:
        p.start()
    root = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert root == O.merkle_hash_gen(n, 32, SEED)


@pytest.mark.parametrize("world,n,k,leaf,slots", [(2, 1 << 14, 3, 5, 3), (2, 4 * 1000 + 3, 2, 3, 3),
                                                  (4, 4 * 3000 + 3, 2, 5, 3), (4, 1 << 14, 1, 5, 3),
                                                  (2, 1 << 14, 3, 5, 2), (2, 4 * 1000 + 3, 2, 3, 4)])
def test_pipelined_sharded_root_equals_full_root(world, n, k, leaf, slots):
    """ShardedMerklePipeline: leaf pass to `leaf` levels above the chunks,
    node passes to the 2^k frontier, all-gather and rank-0 finish split off
    per tree (ragged last shards included), `slots` buffer sets rotating
    over slots + 2 trees."""
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, 32, q, 0, (k, leaf, slots))) for r in range(world)]
    for p in procs:
        p.start()
    root = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert root == O.merkle_hash_gen(n, 32, SEED)


def _phase_worker(rank, world, port, n, q, pipelined):
    """bench.py's N-rank phase record on the CPU path: K steps of the sharded
    step (one-stream or pipelined) with the oracle as the injected compute, a
    host-clock parallel.PhaseTimer, and the record bench.py prints."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import oracle as O
        from prysm_amd import parallel as P

        k, leaf = 3, 5
        sp = P.plan(n, 32, world, plan_fn=_plan_cpu)
        lo, hi = sp.items(rank)
        local = torch.from_numpy(O.splitmix_bytes(n * 32, SEED)[lo * 32:hi * 32].copy())

        def level_below(kk):  # the shard's level kk below its root = roots of its 2^kk sub-shards
            cnt = P.frontier_count(hi - lo, 32, sp.height, kk)
            nodes = b"".join(O.merkle_subtree_gen(n, 32, SEED, (rank << kk) + j, sp.height - kk)
                             for j in range(cnt))
            return torch.frombuffer(bytearray(nodes), dtype=torch.uint8)

        def node_frontier(level, cnt, hh, kk, pad, out):
            nodes = [bytes(level[32 * i:32 * i + 32].numpy()) for i in range(cnt)]
            for _ in range(hh - kk):
                if len(nodes) % 2:
                    nodes = nodes + [bytes(128)]
                nodes = [O.keccak256(nodes[i] + nodes[i + 1]) for i in range(0, len(nodes), 2)]
            return torch.frombuffer(bytearray(b"".join(nodes)), dtype=torch.uint8)

        def finish_nodes(g, count, nt):
            level = [bytes(g[32 * i:32 * i + 32].numpy()) for i in range(count)]
            while len(level) > 1:
                if len(level) % 2:
                    level = level + [bytes(128)]
                level = [O.keccak256(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
            return torch.frombuffer(bytearray(O.keccak256(level[0] + nt.to_bytes(8, "little") + bytes(24))),
                                    dtype=torch.uint8)

        timer = P.PhaseTimer(cuda=False)
        if pipelined:
            pl = P.ShardedMerklePipeline(
                n, 32, sp, rank, world, "cpu", gather_log2=k, leaf_levels=leaf,
                frontier_fn=lambda it, sn, il, h, kk, pad, out: level_below(kk),
                node_frontier_fn=node_frontier, finish_nodes_fn=lambda g, c, nt, out: finish_nodes(g, c, nt),
                timer=timer)
            assert pl.ok
            step = lambda: pl.submit(local)  # noqa: E731
        else:
            step = lambda: P.sharded_merkle_hash(  # noqa: E731
                local, n, 32, sp, rank, world, subtree_fn=lambda *a: None, full_fn=lambda *a: None,
                finish_fn=lambda *a: None, frontier_log2=k, frontier_fn=lambda it, sn, il, h, kk, pad: level_below(kk),
                finish_nodes_fn=finish_nodes, timer=timer)
        step()  # warmup: not marked
        dist.barrier()
        steps = 12
        t0 = time.perf_counter()
        for _ in range(steps):
            timer.start_step()
            r = step()
        dist.barrier()
        ms = (time.perf_counter() - t0) / steps * 1e3
        timer.stop()
        rec = timer.record(world)
        if rank == 0:
            rec["ms_per_step"] = ms
            rec["root"] = bytes(r.numpy())
            q.put(rec)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pipelined", [False, True])
def test_bench_phase_record_world2(pipelined):
    """bench.py's N > 1 record breaks the step into phases (leaf pass, node
    passes to the frontier, all-gather, finisher; parallel.PhaseTimer) for
    rank 0 and every rank.  On the CPU path (gloo, world 2, oracle compute)
    the phases run back to back, so they sum to within 15 % of the step
    (host scheduling noise of a loaded CPU runner aside)."""
    from oracle import oracle as O

    n = 1 << 15
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_phase_worker, args=(r, 2, port, n, q, pipelined)) for r in range(2)]
    for p in procs:
        p.start()
    rec = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert rec["root"] == O.merkle_hash_gen(n, 32, SEED)
    ph = rec["phases_ms"]
    assert set(ph) == {"leaf", "nodes", "gather", "finish", "sum"}
    assert len(rec["per_rank_phases_ms"]) == 2 and all(len(r) == 4 for r in rec["per_rank_phases_ms"])
    assert rec["per_rank_phases_ms"][0] == [ph[k] for k in ("leaf", "nodes", "gather", "finish")]
    assert ph["leaf"] > 0 and ph["finish"] > 0 and rec["per_rank_phases_ms"][1][3] == 0
    assert (ph["nodes"] > 0) == pipelined
    assert abs(ph["sum"] - rec["ms_per_step"]) <= 0.15 * rec["ms_per_step"], (ph, rec["ms_per_step"])


@pytest.mark.parametrize("n,item_len,world", [(4099, 32, 8), (1000, 8, 3), (41 * 4 + 3, 32, 4), (5, 32, 8),
                                              (100, 200, 8), (10**6, 32, 8), (1 << 28, 32, 8)])
def test_python_plan_matches_c_planner(n, item_len, world):
    import ctypes

    from prysm_amd import _lib

    h, ne = ctypes.c_uint32(), ctypes.c_uint32()
    begin = (ctypes.c_uint64 * (world + 1))()
    assert _lib.load().mk_ssz_merkle_shard_plan(None, n, item_len, world, ctypes.byref(h), ctypes.byref(ne), begin) == 0
    ph, pne, pbegin = _plan_cpu(n, item_len, world)
    assert (ne.value, list(begin)) == (pne, pbegin)
    if pne > 1:
        assert h.value == ph


def _trie_worker(rank, world, port, n, q, depth=32):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys

        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from oracle import oracle as O
        from prysm_amd import parallel as P

        dl = 280
        tp = P.trie_plan(n, world, depth)
        lo, hi = tp.items(rank)
        full = O.splitmix_bytes(max(n, 1) * dl, SEED + 5)
        local = torch.from_numpy(full[lo * dl:hi * dl].copy())

        def subtree(data, cnt, ln, h):
            deps = [bytes(data[i * ln:(i + 1) * ln].numpy()) for i in range(cnt)]
            return torch.frombuffer(bytearray(O.deposit_trie_levels(deps, h)[0]), dtype=torch.uint8)

        def top(g, ne, world_, above):
            level = [bytes(g[32 * i:32 * i + 32].numpy()) for i in range(ne)]
            for _ in range(above):  # absent right child = 0^32 (deposit_trie.go:35-37)
                if len(level) % 2:
                    level = level + [bytes(32)]
                level = [O.keccak256(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
            return torch.frombuffer(bytearray(level[0]), dtype=torch.uint8)

        def full_fn(data, cnt, ln, d):
            deps = [bytes(data[i * ln:(i + 1) * ln].numpy()) for i in range(cnt)]
            return torch.frombuffer(bytearray(O.deposit_trie_levels(deps, d)[0] if cnt else bytes(32)),
                                    dtype=torch.uint8)

        root = P.sharded_deposit_trie_root(local, dl, tp, rank, world, subtree_fn=subtree, top_fn=top,
                                           full_fn=full_fn)
        if rank == 0:
            q.put((bytes(root.numpy()), tp.height, tp.nonempty))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n", [(2, 1000), (4, 1024), (4, 777), (3, 100), (8, 5), (4, 0), (8, 2049)])
def test_sharded_deposit_trie_root(world, n):
    """SURVEY §8e's C5 split: every rank builds its power-of-two subtree of
    the depth-32 deposit trie, one 32-B all-gather, rank 0 builds the levels
    above (0^32 for absent nodes, then the zero-sibling levels); the root
    equals the one-piece build (ragged last shard, empty shards, too small to
    shard, empty trie)."""
    from oracle import oracle as O

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_trie_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    root, h, ne = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dl = 280
    full = O.splitmix_bytes(max(n, 1) * dl, SEED + 5)
    deps = [bytes(full[i * dl:(i + 1) * dl]) for i in range(n)]
    want = O.deposit_trie_levels(deps, 32)[0] if n else bytes(32)
    assert root == want
    if n >= 2 * world:
        assert h > 0 and ne > 1  # really sharded
