"""GPU parity of the device-resident incremental deposit trie
(mk_deposit_trie_* handle, mk_dev_deposit_trie_append/branch) against the
literal dict restatement of shared/trieutil/deposit_trie.go:13-63
(oracle.DictTrie) and the oracle's batch build."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 500


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    assert _lib.device_count() >= 1
    return torch.device("cuda:0")


def _deposit(i: int, ln: int = 280) -> bytes:
    from oracle import oracle as O

    return bytes(O.splitmix_bytes(ln, SEED, 35 * i))


def test_read_root_then_update_2000(gpu):
    """powchain saveInTrie (service.go:379-386): Root() before every
    UpdateDepositTrie.  Each append recomputes the right edge only."""
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    t, ref = T.DepositTrie(), O.DictTrie()
    rng = np.random.default_rng(5)
    for i in range(2000):
        assert t.Root() == ref.root(), i
        d = _deposit(i)
        t.UpdateDepositTrie(d)
        ref.update(d)
        if i % 173 == 0:
            j = int(rng.integers(0, i + 1))
            assert t.GenerateMerkleBranch(j) == ref.branch(j), (i, j)
    assert t.Root() == ref.root()
    assert t.deposit_count == 2000
    for j in (0, 1, 1023, 1024, 1999):
        br = t.GenerateMerkleBranch(j)
        assert br == ref.branch(j)
        assert T.VerifyMerkleBranch(O.keccak256(_deposit(j)), br, 32, j, t.Root())


def test_variable_length_deposits_incremental(gpu):
    """Deposits of different lengths (the var-length leaf kernel), appended in
    uneven batches, past the initial capacity (1024) and a capacity doubling."""
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    t, ref = T.DepositTrie(), O.DictTrie()
    i = 0
    for batch in (1, 2, 5, 1, 100, 917, 1, 3000, 1):
        for _ in range(batch):
            d = _deposit(i, 1 + (i * 37) % 300)
            t.UpdateDepositTrie(d)
            ref.update(d)
            i += 1
        assert t.Root() == ref.root(), i
    for j in (0, 7, 1024, i - 1):
        assert t.GenerateMerkleBranch(j) == ref.branch(j)
        assert t.leaf(j) == O.keccak256(_deposit(j, 1 + (j * 37) % 300))


@pytest.mark.parametrize("batches", [(70_000,), (6_004, 70_000, 2), (1, 1, 1 << 17), ((1 << 17) + 5, 1023, 1024)])
def test_append_batches_equal_batch_build(gpu, batches):
    """Large appends take the wide-level path (k_trie_level on the right
    edge) before the one-workgroup top; every state equals the batch build."""
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    t = T.DepositTrie()
    deps = []
    for b in batches:
        new = [_deposit(len(deps) + k) for k in range(b)]
        deps += new
        for d in new:
            t.UpdateDepositTrie(d)
        root, levels = O.deposit_trie_levels(deps)
        assert t.Root() == root, len(deps)
        for j in sorted({0, len(deps) // 3, len(deps) - 1}):
            want = [levels[d][(j >> d) ^ 1] if ((j >> d) ^ 1) < len(levels[d]) else bytes(32) for d in range(32)]
            assert t.GenerateMerkleBranch(j) == want, (len(deps), j)


@pytest.mark.parametrize("depth", [1, 2, 5, 20, 33, 63])
def test_depths(gpu, depth):
    from oracle import oracle as O
    from prysm_amd import trieutil as T

    n = min(1 << depth, 37)
    t, ref = T.DepositTrie(depth), O.DictTrie(depth)
    for i in range(n):
        d = _deposit(i, 44)
        t.UpdateDepositTrie(d)
        ref.update(d)
        if i % 5 == 0:
            assert t.Root() == ref.root()
    assert t.Root() == ref.root()
    assert t.GenerateMerkleBranch(n - 1) == ref.branch(n - 1)


def test_trie_full_is_an_error(gpu):
    from prysm_amd import _lib
    from prysm_amd import trieutil as T

    t = T.DepositTrie(2)
    for i in range(4):
        t.UpdateDepositTrie(_deposit(i, 8))
    assert len(t.Root()) == 32
    t.UpdateDepositTrie(_deposit(4, 8))
    with pytest.raises(_lib.MerkleError) as ei:
        t.Root()
    assert "do not fit a depth-2 trie" in str(ei.value)


def test_dev_append_stream_of_blocks(gpu):
    """mk_dev_deposit_trie_append on device-resident 280-B deposits (fixed
    records, k_keccak_rec): blocks of deposits appended to one HBM trie;
    root and branches after every block equal the batch build of the prefix."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    depth, cap, ln = 32, 1 << 16, 280
    total = 41_000
    data = torch.empty(total * ln, dtype=torch.uint8, device=gpu)
    D.synth_fill(data, SEED + 7)
    host = data.cpu().numpy()
    levels = torch.zeros(D.deposit_trie_levels_bytes(cap, depth), dtype=torch.uint8, device=gpu)
    root = torch.empty(32, dtype=torch.uint8, device=gpu)
    count = 0
    for k in (16, 1, 3000, 5, 1021, 1022, 17_000, 18_935):
        D.deposit_trie_append(levels, cap, count, data[count * ln:(count + k) * ln], k, ln, depth, root)
        count += k
        deps = [bytes(host[i * ln:(i + 1) * ln]) for i in range(count)]
        want_root, lv = O.deposit_trie_levels(deps)
        br = D.deposit_trie_branch(levels, cap, count, depth, count - 1)
        torch.cuda.synchronize()
        assert bytes(root.cpu().numpy()) == want_root, count
        want_br = b"".join(lv[d][((count - 1) >> d) ^ 1] if (((count - 1) >> d) ^ 1) < len(lv[d]) else bytes(32)
                           for d in range(depth))
        assert bytes(br.cpu().numpy()) == want_br, count
    assert count == total


@pytest.mark.parametrize("n", [1, 5, 1000, (1 << 17) + 3, (1 << 19) + 7])
def test_trie_pipeline_stream_of_tries(gpu, n):
    """TriePipeline: leaves + wide levels on the current stream, the top on a
    side stream overlapping the next trie; 4 consecutive tries, each root and
    a branch against the oracle's batch build."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd.pipeline import TriePipeline

    ln, depth = 280, 32
    pipe = TriePipeline(n, ln, depth, gpu)
    datas = []
    for t in range(4):
        d = torch.empty(n * ln, dtype=torch.uint8, device=gpu)
        D.synth_fill(d, SEED + 900 + t)
        datas.append(d)
    roots = []
    for t, d in enumerate(datas):
        roots.append(pipe.submit(d))
        if t % 2 == 1:
            torch.cuda.synchronize()
            roots = [r if isinstance(r, bytes) else bytes(r.cpu().numpy()) for r in roots]
    for t, d in enumerate(datas):
        host = d.cpu().numpy()
        want = O.deposit_trie_levels([bytes(host[i * ln:(i + 1) * ln]) for i in range(n)])[0]
        assert roots[t] == want, (t, pipe.split)


@pytest.mark.parametrize("n,ln", [(1, 280), (2, 280), (3, 280), (5, 280), (6, 280), (7, 280), (9, 280),
                                  (1000, 280), (4095, 280), (1003, 44), (37, 281)])
@pytest.mark.parametrize("d_to", [0, 1, 2, 3, 12])
def test_build_front_levels(gpu, n, ln, d_to):
    """mk_dev_deposit_trie_build: leaf hashes + levels 1..d_to of a batch
    build (280-B deposits on the record kernel, 44-B on the word kernel,
    281-B on the byte kernel), every written level against the oracle's
    batch build, then levels d_to..depth and the root."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    depth = 12
    cap = 1 << 12
    data = torch.empty((n * ln + 15) // 8 * 8, dtype=torch.uint8, device=gpu)
    D.synth_fill(data, SEED + 31 * n + ln)
    lv = torch.zeros(D.deposit_trie_levels_bytes(cap, depth), dtype=torch.uint8, device=gpu)
    root = torch.empty(32, dtype=torch.uint8, device=gpu)
    D.deposit_trie_build(lv, cap, data, n, ln, d_to, depth, root if d_to == depth else None)
    host = data.cpu().numpy()
    want_root, want = O.deposit_trie_levels([bytes(host[i * ln:(i + 1) * ln]) for i in range(n)], depth)
    got = lv.cpu().numpy()
    off, capd = 0, cap
    for d in range(d_to + 1):
        c = len(want[d])
        assert [bytes(got[(off + i) * 32:(off + i + 1) * 32]) for i in range(c)] == want[d], (d, n)
        off += capd
        capd = (capd + 1) // 2
    if d_to < depth:
        D.deposit_trie_levels(lv, cap, n, d_to, depth, depth, root)
    assert bytes(root.cpu().numpy()) == want_root


@pytest.mark.parametrize("start,k,bad", [(0, 1, ()), (0, 40, (0,)), (5, 40, (3, 4, 17, 39)), (1000, 3000, (7, 1500, 2999)),
                                         (77, 64, tuple(range(0, 64, 2))), (10, 20, tuple(range(20)))])
def test_save_logs_matches_reference_loop(gpu, start, k, bad):
    """mk_deposit_trie_save_logs against the reference's per-log loop
    (ProcessDepositLog -> saveInTrie, powchain/service.go:248-258, 379-386)
    run on the dict restatement of deposit_trie.go: each log carries the root
    the trie had before its deposit, except the `bad` ones (a wrong root:
    the reference skips them and goes on).  Accept flags, Root() and
    branches must agree."""
    import random

    from oracle import oracle as O
    from prysm_amd import trieutil as T

    rng = random.Random(start * 7919 + k)
    t, ref = T.DepositTrie(32), O.DictTrie(32)
    for i in range(start):  # history before the batch
        d = _deposit(i)
        t.UpdateDepositTrie(d)
        ref.update(d)
    deps = [_deposit(start + i, 280 if i % 5 else 200) for i in range(k)]
    roots, want = [], []
    for j, d in enumerate(deps):
        r = ref.root()
        if j in bad:
            r = bytes(rng.getrandbits(8) for _ in range(32))
        roots.append(r)
        ok = ref.root() == r
        want.append(ok)
        if ok:
            ref.update(d)
    got = t.save_logs(deps, roots)
    assert got == want
    assert t.Root() == ref.root()
    n = ref.count
    for idx in sorted({0, n // 2, n - 1}):
        if n:
            assert t.GenerateMerkleBranch(idx) == ref.branch(idx), idx
    # the trie keeps working as a plain trie afterwards
    extra = _deposit(start + k + 1)
    t.UpdateDepositTrie(extra)
    ref.update(extra)
    assert t.Root() == ref.root()


@pytest.mark.parametrize("k,missed", [(1, None), (50, None), (50, 20), (300, 0)])
def test_save_logs_of_deposit_contract_events(gpu, k, missed):
    """The node side of the ETH1 contract: the Deposit events of the
    contract restatement (depositContract.v.py:36-52; each carries the
    contract's root before its deposit) fed to mk_deposit_trie_save_logs.
    Every log is accepted and the trie's Root() and branches equal the
    contract's get_deposit_root / get_branch.  With one log lost on the way
    (`missed`), the ones after it carry roots the trie never had: they are
    all skipped, and the trie stays at the root before the gap."""
    import random

    from oracle import oracle as O
    from prysm_amd import trieutil as T

    rng = random.Random(k * 31 + (missed or 0))
    c = O.DepositContract()
    events = [c.deposit(32 * 10**9, 1_540_000_000 + i, bytes(rng.getrandbits(8) for _ in range(264)))
              for i in range(k)]
    seen = [e for j, e in enumerate(events) if j != missed]
    t = T.DepositTrie(32)
    got = t.save_logs([e[1] for e in seen], [e[0] for e in seen])
    if missed is None:
        assert got == [True] * k
        assert t.Root() == c.get_deposit_root()
        for idx in sorted({0, k // 2, k - 1}):
            assert t.GenerateMerkleBranch(idx) == c.get_branch(idx), idx
    else:
        assert got == [True] * missed + [False] * (k - 1 - missed)
        assert t.Root() == events[missed][0]


@pytest.mark.parametrize("n", [4096, 5 * 4096, 1 << 18])
def test_trie_pipeline_pipelined_front(gpu, n):
    """TriePipeline's "pipe" front: trie t's leaves + levels 1-2 in one
    phase-locked launch that also builds levels 3-7 of trie t-1 in its
    lock-step slots, trie t-1's top beside trie t+1's front, the last trie by
    flush().  Every root and branches of three tries (the levels the slots
    wrote among them) against the oracle's batch build; bad shapes refused."""
    import torch

    from oracle import oracle as O
    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd.pipeline import TriePipeline

    ln, depth = 280, 32
    pipe = TriePipeline(n, ln, depth, gpu, front="pipe")
    datas = []
    for t in range(4):
        d = torch.empty(n * ln, dtype=torch.uint8, device=gpu)
        D.synth_fill(d, SEED + 950 + t)
        datas.append(d)
    assert D.deposit_trie_pipe_ok(datas[0], n, ln, depth)
    got, handles = [], []
    for t, d in enumerate(datas):
        handles.append(pipe.submit(d))
        if t:
            torch.cuda.synchronize()
            got.append(bytes(handles[t - 1].cpu().numpy()))
    assert pipe._last_pipe
    pipe.flush()
    torch.cuda.synchronize()
    got.append(bytes(handles[-1].cpu().numpy()))
    wants = []
    for t, d in enumerate(datas):
        host = d.cpu().numpy()
        root, levels = O.deposit_trie_levels([bytes(host[i * ln:(i + 1) * ln]) for i in range(n)])
        assert got[t] == root, (t, n)
        wants.append(levels)
    # tries 1..3 still hold their levels (sets 1, 2, 0)
    for t in (1, 2, 3):
        lv = pipe.levels[t % len(pipe.levels)]
        for idx in sorted({0, n // 3, n - 1}):
            br = torch.empty(32 * depth, dtype=torch.uint8, device=gpu)
            D.deposit_trie_branch(lv, n, n, depth, idx, br)
            torch.cuda.synchronize()
            want = b"".join(wants[t][d][(idx >> d) ^ 1] if ((idx >> d) ^ 1) < len(wants[t][d]) else bytes(32)
                            for d in range(depth))
            assert bytes(br.cpu().numpy()) == want, (t, idx)
    lv = pipe.levels[0]
    with pytest.raises(_lib.MerkleError):
        D.deposit_trie_build_pipe(lv, None, n + 1, datas[0], n + 1, ln, depth)  # not whole groups
    with pytest.raises(_lib.MerkleError):
        D.deposit_trie_build_pipe(lv, lv, n, datas[0], n, ln, depth)  # aliasing sets
    assert not D.deposit_trie_pipe_ok(datas[0], n, 200, depth)


def test_trie_pipeline_mixed_fronts_and_flush(gpu):
    """TriePipeline over a stream whose buffers switch between the pipelined
    front (16-B aligned) and the split front (an 8-B-offset view), with a
    flush in the middle: every root against the oracle's batch build."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd.pipeline import TriePipeline

    n, ln, depth = 4096, 280, 32
    pipe = TriePipeline(n, ln, depth, gpu, front="auto")
    store = torch.empty(n * ln + 16, dtype=torch.uint8, device=gpu)
    plan = ["pipe", "pipe", "split", "pipe", "flush", "pipe", "split", "split", "pipe", "pipe"]
    handles, wants = [], []
    for t, step in enumerate(plan):
        if step == "flush":
            pipe.flush()
            continue
        off = 0 if step == "pipe" else 8
        d = store[off:off + n * ln]
        D.synth_fill(store, SEED + 970 + t)
        assert D.deposit_trie_pipe_ok(d, n, ln, depth) == (step == "pipe")
        host = d.cpu().numpy()
        wants.append(O.deposit_trie_levels([bytes(host[i * ln:(i + 1) * ln]) for i in range(n)])[0])
        handles.append(pipe.submit(d))
        assert pipe._last_pipe == (step == "pipe")
        torch.cuda.synchronize()  # the next fill rewrites the shared buffer
        if len(handles) > 1:
            # a split root is final once its submit has run; a pipelined one
            # once the next submit (or flush) has
            assert bytes(handles[-2].cpu().numpy()) == wants[-2], (t, step)
    pipe.flush()
    torch.cuda.synchronize()
    assert bytes(handles[-1].cpu().numpy()) == wants[-1]


def test_trie_pipeline_default_root_ready_after_submit(gpu):
    """The default front is "split" at every shape, including the shapes the
    pipelined front takes (whole 4096-deposit groups): a root read after
    submit + synchronize is that trie's root (the pipelined form's deferred
    root is opt-in)."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd.pipeline import TriePipeline

    n, ln, depth = 8192, 280, 32
    pipe = TriePipeline(n, ln, depth, gpu)
    d = torch.empty(n * ln, dtype=torch.uint8, device=gpu)
    for t in range(3):
        D.synth_fill(d, SEED + 990 + t)
        assert D.deposit_trie_pipe_ok(d, n, ln, depth)
        r = pipe.submit(d)
        torch.cuda.synchronize()
        host = d.cpu().numpy()
        assert bytes(r.cpu().numpy()) == O.deposit_trie_levels([bytes(host[i * ln:(i + 1) * ln])
                                                                 for i in range(n)])[0], t
    assert not pipe._last_pipe


def test_trie_pipeline_pipe_submits_from_two_streams(gpu):
    """Pipelined fronts submitted alternately from two streams (each front
    reads the previous trie's levels 0-2, which the other stream wrote): the
    pipeline orders them, every root equals the oracle's."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D
    from prysm_amd.pipeline import TriePipeline

    n, ln, depth = 2 * 4096, 280, 32
    pipe = TriePipeline(n, ln, depth, gpu, front="pipe")
    streams = [torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu)]
    datas, handles = [], []
    for t in range(5):
        d = torch.empty(n * ln, dtype=torch.uint8, device=gpu)
        D.synth_fill(d, SEED + 995 + t)
        datas.append(d)
    torch.cuda.synchronize()
    got = []
    for t, d in enumerate(datas):
        with torch.cuda.stream(streams[t % 2]):
            handles.append(pipe.submit(d))
        if t:  # a root is produced by the next submit and valid for two more (four sets rotate)
            torch.cuda.synchronize()
            got.append(bytes(handles[t - 1].cpu().numpy()))
    with torch.cuda.stream(streams[1]):
        pipe.flush()
    torch.cuda.synchronize()
    got.append(bytes(handles[-1].cpu().numpy()))
    for t, d in enumerate(datas):
        host = d.cpu().numpy()
        want = O.deposit_trie_levels([bytes(host[i * ln:(i + 1) * ln]) for i in range(n)])[0]
        assert got[t] == want, t
