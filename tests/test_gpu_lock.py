"""GPU parity of the phase-locked kernels (1024-thread workgroups whose Keccak
rounds hold s_barriers; DESIGN.md §4 "Phase-locked rounds") at the shapes
where they hand over to the free-running kernels: whole groups of 1024
threads run locked, the persistent grid's workgroups take unequal numbers of
groups, and the rest (the spans after the last whole group, the ragged tail)
runs in k_reduce / k_keccak64 / k_keccak_rec / k_struct_reg.  Every result
against the CPU oracle, bit-exact.  The library build decides which kernels
are locked (mk_version); the tests hold for either build."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    _lib.init(0)
    return torch.device("cuda:0")


# merkleHash leaf passes: 2^20 windows (= 2^23 32-B items) is the smallest
# locked leaf pass; 4096 windows per locked workgroup, 1024 per k_reduce span
@pytest.mark.parametrize("n", [
    1 << 23,                          # 256 locked groups exactly, one per CU
    (1 << 23) + 8 * 1024 * 3 + 77,    # 3 k_reduce FAST spans after the groups + a ragged window
    5 * (1 << 21) + 12_345,           # 320 groups over 256 workgroups (uneven) + the rest
    (1 << 24) - 1,                    # odd item count: the last window is padded
])
def test_leaf_lock_merkle_vs_oracle(gpu, n):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    items = torch.empty(n * 32, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 41)
    root = D.merkle_hash(items, n, 32)
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()) == O.merkle_hash_gen(n, 32, SEED + 41, nthreads=16)


def test_leaf_lock_small_items(gpu):
    """8-B items: 16 per chunk, the same 256-B windows."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n = (1 << 25) + 1000
    items = torch.empty(n * 8, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 42)
    root = D.merkle_hash(items, n, 8)
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()) == O.merkle_hash_gen(n, 8, SEED + 42, nthreads=16)


@pytest.mark.parametrize("n,world", [(1 << 24, 2), ((1 << 25) + 99, 4)])
def test_leaf_lock_subtree_shards(gpu, n, world):
    """Subtree shards (the multi-GPU split) whose leaf passes are
    locked: every shard root against the oracle's subtree and the finished
    root against the full merkleHash."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    h, ne, begin = D.shard_plan(n, 32, world)
    items = torch.empty(n * 32, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 43)
    roots = torch.zeros(world * 32, dtype=torch.uint8, device=gpu)
    for s in range(ne):
        D.merkle_subtree(items[begin[s] * 32:begin[s + 1] * 32], begin[s + 1] - begin[s], 32, h, True,
                         out=roots[32 * s:32 * s + 32])
    got = D.merkle_finish(roots, ne, n)
    torch.cuda.synchronize()
    for s in range(ne):
        assert bytes(roots[32 * s:32 * s + 32].cpu().numpy()) == O.merkle_subtree_gen(
            n, 32, SEED + 43, s, h, nthreads=16), s
    assert bytes(got.cpu().numpy()) == O.merkle_hash_gen(n, 32, SEED + 43, nthreads=16)


# batched Keccak: locked for whole groups of 1024 messages once n >= 2^18
@pytest.mark.parametrize("msg_len,n", [(64, 1 << 18), (64, (1 << 18) + 1024 * 70 + 5),
                                       (280, 1 << 18), (280, (1 << 18) + 1024 * 70 + 5)])
def test_hash_batch_lock_vs_oracle(gpu, msg_len, n):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    msgs = torch.empty(n * msg_len, dtype=torch.uint8, device=gpu)
    D.synth_fill(msgs, SEED + 44 + msg_len)
    got = D.hash_batch(msgs, n, msg_len)
    torch.cuda.synchronize()
    want = O.keccak256_batch(msgs.cpu().numpy(), msg_len, nthreads=16)
    assert np.array_equal(got.cpu().numpy().reshape(n, 32), want)


# typed registry (ValidatorRecord, 160-B records): locked from 2^18 records
@pytest.mark.parametrize("n", [1 << 18, (1 << 18) + 1024 * 33 + 17])
def test_struct_lock_vs_oracle(gpu, n):
    from oracle import oracle as O
    from prysm_amd import registry as R

    reg = R.synthetic_registry(n, SEED + 45)
    raw = reg.records.view(np.uint8).reshape(-1)
    spec = [(k, o, l) for k, o, l in R.VALIDATOR_FIELDS]
    want = O.struct_roots(raw, n, 160, spec, nthreads=16)
    assert np.array_equal(R.struct_roots(reg.records), want)


def test_deposit_trie_lock_vs_oracle(gpu):
    """A 2^18 + 3-deposit batch build through the trie handle: the leaves are
    locked groups + the rest; root and one branch against the oracle."""
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    n, ln = (1 << 18) + 3, 280
    host = O.splitmix_bytes(n * ln, SEED + 46)
    deps = [bytes(host[i * ln:(i + 1) * ln]) for i in range(n)]
    trie = T.DepositTrie.build(deps)
    root, levels = O.deposit_trie_levels(deps)
    assert trie.Root() == root
    k = n - 2
    branch = trie.GenerateMerkleBranch(k)
    assert branch[0] == levels[0][k ^ 1]


# registry list root with the merkleHash leaf pass fused into the locked
# struct kernel (k_struct_lock gpw > 0): contiguous groups per workgroup, then
# one level-1 window per lane; the ragged last window (n % 8 != 0) hashes its
# r roots, plus 0^128 when they fill one chunk only (r <= 4)
@pytest.mark.parametrize("n", [
    1 << 18,                 # 256 groups, one per workgroup, 128 windows each
    (1 << 18) + 5,           # a partial group; last window 5 roots (two chunks)
    (1 << 18) + 1024 + 3,    # last window 3 roots: one chunk + 0^128
    1_000_000,               # C3: 977 groups, 4 per workgroup (245 workgroups)
    (1 << 20) + 7 * 1024 + 1,
])
def test_struct_list_root_windows_vs_oracle(gpu, n):
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd import registry as R

    reg = R.synthetic_registry(n, SEED + 47 + n % 13)
    raw = reg.records.view(np.uint8).reshape(-1)
    spec = [(k, o, l) for k, o, l in R.VALIDATOR_FIELDS]
    roots = O.struct_roots(raw, n, 160, spec, nthreads=16)
    want = O.merkle_hash_flat(roots.reshape(-1), n, 32, nthreads=16)
    drec = torch.from_numpy(raw.copy()).to(gpu)
    got = D.struct_list_root(drec, n, 160, R.VALIDATOR_FIELDS)
    torch.cuda.synchronize()
    assert bytes(got.cpu().numpy()) == want
    # the split form: roots + level-1 nodes, then the finisher
    assert D.struct_list_level1_ok(drec, n, 160, R.VALIDATOR_FIELDS)
    c1 = -(-n // 8)
    roots_d = torch.empty(32 * n, dtype=torch.uint8, device=gpu)
    nodes = torch.empty(32 * c1, dtype=torch.uint8, device=gpu)
    D.struct_list_level1(drec, n, 160, R.VALIDATOR_FIELDS, roots_d, nodes)
    got2 = D.merkle_finish_nodes(nodes, c1, n)
    torch.cuda.synchronize()
    assert bytes(got2.cpu().numpy()) == want
    assert np.array_equal(roots_d.cpu().numpy().reshape(n, 32), roots.reshape(n, 32))
    # with a second list's level-1 windows in the same launch (the State's
    # balances: 8-B items; and 32-B items), ragged or not
    for nv, vl in ((n, 8), (n + 3, 8), (1000, 32), (17, 8)):
        vals = O.splitmix_bytes(nv * vl, SEED + 49 + nv)
        dv = torch.from_numpy(vals.copy()).to(gpu)
        cv = -(-nv * vl // 256)
        vnodes = torch.empty(32 * cv, dtype=torch.uint8, device=gpu)
        D.struct_list_level1(drec, n, 160, R.VALIDATOR_FIELDS, roots_d, nodes, values=dv, nvalues=nv, value_len=vl,
                             value_nodes=vnodes)
        gv = D.merkle_finish_nodes(vnodes, cv, nv)
        gr = D.merkle_finish_nodes(nodes, c1, n)
        torch.cuda.synchronize()
        assert bytes(gr.cpu().numpy()) == want, (nv, vl)
        want_v = O.merkle_hash_flat(vals, nv, vl, nthreads=16)
        assert bytes(gv.cpu().numpy()) == want_v, (nv, vl)
        # the pair finisher: each field's root into its slot, the second to
        # complete hashes Keccak(slot 0 || slot 1); both orders on one stream,
        # then the two on two streams at once, each pair with a new epoch
        pb = torch.zeros(128, dtype=torch.uint8, device=gpu)
        want_s = O.keccak256(want + want_v)
        epoch = 0
        for order in ((0, 1), (1, 0)):
            pb[64:96].zero_()
            epoch += 1
            for slot in order:  # cv may be 1: the one-node finisher
                if slot == 0:
                    D.merkle_finish_nodes_pair(nodes, c1, n, pb, 0, epoch)
                else:
                    D.merkle_finish_nodes_pair(vnodes, cv, nv, pb, 1, epoch)
            torch.cuda.synchronize()
            got_pb = bytes(pb.cpu().numpy())
            assert got_pb[:32] == want and got_pb[32:64] == want_v, (nv, vl, order)
            assert got_pb[64:96] == want_s, (nv, vl, order)
            assert int.from_bytes(got_pb[96:100], "little") == (epoch << 2) | 3, (nv, vl, order)
        # a pair left half-done (only slot 0 ran) does not complete with the next
        pb[64:96].zero_()
        D.merkle_finish_nodes_pair(nodes, c1, n, pb, 0, epoch + 1)
        torch.cuda.synchronize()
        assert bytes(pb[64:96].cpu().numpy()) == bytes(32)
        D.merkle_finish_nodes_pair(nodes, c1, n, pb, 0, epoch + 2)
        torch.cuda.synchronize()
        assert bytes(pb[64:96].cpu().numpy()) == bytes(32), "slot 0 of a new epoch completed a stale pair"
        side = torch.cuda.Stream(device=gpu)
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        with torch.cuda.stream(side):
            D.merkle_finish_nodes_pair(vnodes, cv, nv, pb, 1, epoch + 2)
        D.merkle_finish_nodes_pair(nodes, c1, n, pb, 0, epoch + 2)  # slot 0 twice in one epoch: idempotent
        torch.cuda.synchronize()
        assert bytes(pb[64:96].cpu().numpy()) == want_s, (nv, vl)
        with pytest.raises(Exception):
            D.merkle_finish_nodes_pair(nodes, c1, n, pb, 2, epoch + 3)
        with pytest.raises(Exception):
            D.merkle_finish_nodes_pair(nodes, c1, n, pb, 0, 0)


def test_state_hasher_schedules_agree(gpu):
    """registry.DeviceStateHasher under its four schedules (level-1 front +
    both tops in one fused launch, level-1 front + the two finishers on two
    streams, the one-call list root, round 3's two-call schedule) against the
    host-buffer state root, three submits each."""
    import torch

    from prysm_amd import registry as R

    n = (1 << 18) + 77
    reg = R.synthetic_registry(n, SEED + 48)
    bal = R.synthetic_balances(n, SEED + 48)
    want = R.state_root(reg, bal)
    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(gpu)
    dbal = torch.from_numpy(bal.view(np.uint8).copy()).to(gpu)
    for sched in ("fused", "level1", "list", "two"):
        h = R.DeviceStateHasher(n, gpu, schedule=sched)
        for _ in range(3):
            out = h.submit(rec, dbal)
        torch.cuda.synchronize()
        assert bytes(out.cpu().numpy()) == want, sched


def test_state_hasher_misaligned_balances_fall_back(gpu):
    """"level1" needs the balances 16-B aligned (mk_dev_ssz_struct_list_level1);
    an 8-B-offset view falls back to the one-call list schedule (same root
    tensor) instead of raising MK_EINVAL, and aligned balances take level1
    again on the next submit."""
    import torch

    from prysm_amd import registry as R

    n = (1 << 18) + 3
    reg = R.synthetic_registry(n, SEED + 49)
    bal = R.synthetic_balances(n, SEED + 49)
    want = R.state_root(reg, bal)
    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(gpu)
    store = torch.empty(n * 8 + 16, dtype=torch.uint8, device=gpu)
    h = R.DeviceStateHasher(n, gpu)
    for off in (8, 0, 8):
        store[off:off + n * 8].copy_(torch.from_numpy(bal.view(np.uint8).copy()))
        out = h.submit(rec, store[off:off + n * 8])
        torch.cuda.synchronize()
        assert out.data_ptr() == h.out.data_ptr()
        assert bytes(out.cpu().numpy()) == want, off



def _finish_ref(nodes: bytes, n_total: int) -> bytes:
    """merkleHash's level loop over 32-B nodes and its length mix-in
    (hash.go:225-237: an odd level appends the 128-B zero chunk)."""
    from oracle import oracle as O

    lv = [nodes[32 * i:32 * i + 32] for i in range(len(nodes) // 32)]
    while len(lv) > 1:
        if len(lv) % 2:
            lv.append(bytes(128))
        lv = [O.keccak256(lv[2 * i] + lv[2 * i + 1]) for i in range(len(lv) // 2)]
    return O.keccak256(lv[0] + n_total.to_bytes(8, "little") + bytes(24))


def test_pair_finisher_many_pairs_random_order(gpu):
    """60 pairs through one pair block, the two finishers launched in a
    random order on two streams each time (sometimes slot 0 first, sometimes
    slot 1, sometimes concurrently), a new epoch per pair; one pair in five
    is preceded by a half-done pair of the epoch before it (a failed call's
    leftover: the block's root reads back as zeros, not the previous pair's),
    and one in seven is followed by a late finisher of an older epoch (it is
    ignored: the arrival word and the root stay).  Every struct root equals
    Keccak(root0 || root1) of that pair's inputs."""
    import random

    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    rng = random.Random(77)
    side = torch.cuda.Stream(device=gpu)
    pb = torch.zeros(128, dtype=torch.uint8, device=gpu)
    for e in range(1, 61):
        ep = 2 * e
        c0, c1 = rng.choice([1, 7, 100, 3000]), rng.choice([1, 64, 65, 2048])
        a = torch.from_numpy(O.splitmix_bytes(32 * c0, 9000 + e).copy()).to(gpu)
        b = torch.from_numpy(O.splitmix_bytes(32 * c1, 9500 + e).copy()).to(gpu)
        want0 = _finish_ref(bytes(a.cpu().numpy()), c0)
        want1 = _finish_ref(bytes(b.cpu().numpy()), c1)
        if e % 5 == 0:  # a stale half of the epoch before this pair's
            D.merkle_finish_nodes_pair(a, c0, c0, pb, rng.randrange(2), ep - 1)
            torch.cuda.synchronize()
            assert bytes(pb[64:96].cpu().numpy()) == bytes(32), e  # never a plausible old root
        order = rng.randrange(3)
        ev = torch.cuda.Event()
        ev.record()
        side.wait_event(ev)
        if order == 0:
            D.merkle_finish_nodes_pair(a, c0, c0, pb, 0, ep)
            D.merkle_finish_nodes_pair(b, c1, c1, pb, 1, ep)
        elif order == 1:
            D.merkle_finish_nodes_pair(b, c1, c1, pb, 1, ep)
            D.merkle_finish_nodes_pair(a, c0, c0, pb, 0, ep)
        else:
            with torch.cuda.stream(side):
                D.merkle_finish_nodes_pair(b, c1, c1, pb, 1, ep)
            D.merkle_finish_nodes_pair(a, c0, c0, pb, 0, ep)
        torch.cuda.synchronize()
        if e % 7 == 0:  # a late finisher of an older epoch: ignored
            D.merkle_finish_nodes_pair(b, c1, c1, pb, rng.randrange(2), ep - 3)
            torch.cuda.synchronize()
        got = bytes(pb.cpu().numpy())
        assert got[:32] == want0 and got[32:64] == want1, e
        assert got[64:96] == O.keccak256(want0 + want1), (e, order)
        assert int.from_bytes(got[96:100], "little") == (ep << 2) | 3, e


def test_pair_finisher_epoch_wraps(gpu):
    """Epochs are 30-bit counters: after 2^30 - 1 comes 1, which is newer
    (the state hasher's epoch % (2^30 - 1) + 1); the pair still completes."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    pb = torch.zeros(128, dtype=torch.uint8, device=gpu)
    a = torch.from_numpy(O.splitmix_bytes(32 * 5, 31).copy()).to(gpu)
    b = torch.from_numpy(O.splitmix_bytes(32 * 9, 32).copy()).to(gpu)
    want = O.keccak256(_finish_ref(bytes(a.cpu().numpy()), 5) + _finish_ref(bytes(b.cpu().numpy()), 9))
    for ep in ((1 << 30) - 1, 1, 2):
        D.merkle_finish_nodes_pair(a, 5, 5, pb, 0, ep)
        D.merkle_finish_nodes_pair(b, 9, 9, pb, 1, ep)
        torch.cuda.synchronize()
        assert bytes(pb[64:96].cpu().numpy()) == want, ep
        assert int.from_bytes(bytes(pb[96:100].cpu().numpy()), "little") == (ep << 2) | 3, ep
