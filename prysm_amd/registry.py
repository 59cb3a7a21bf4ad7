"""Typed validator-registry path (BASELINE configs 1/3).

The reference tree-hashes a registry reflectively, one Keccak call per field
(shared/ssz/hash.go:118-159).  Its own plugin hook, ``ssz.Hashable``
(hash.go:18-20, checked first at :57-58), lets a typed registry hash itself:
``ValidatorRegistry.tree_hash_ssz()`` keeps the validators as one flat
fixed-layout array and hands it to the engine (``mk_*ssz_struct*``): one
launch hashes every bytes field (Keccak(le32(len)||bytes)), one hashes every
144-byte struct message, then the fused merkleHash kernels reduce the list.

Record layout (160 B, 4-byte aligned): the field order of ``pb.Validator``
(proto/beacon/p2p/v1/types.pb.go:661-671) with ``StatusFlags`` widened from
int32 to uint64 so SSZ accepts it (``makeEncoder`` rejects int32,
ssz/encode.go:107-108; recorded deviation).
"""
from __future__ import annotations

import ctypes
import struct as _st

import numpy as np

from . import _lib
from . import ssz as S
from .hashutil import _ptr

VALIDATOR_DTYPE = np.dtype([
    ("pubkey", "u1", 48),
    ("withdrawal_credentials_hash32", "u1", 32),
    ("randao_commitment_hash32", "u1", 32),
    ("randao_layers", "<u8"),
    ("activation_epoch", "<u8"),
    ("exit_epoch", "<u8"),
    ("withdrawal_epoch", "<u8"),
    ("penalized_epoch", "<u8"),
    ("status_flags", "<u8"),
])
assert VALIDATOR_DTYPE.itemsize == 160

# (kind, offset, len) in declaration order
VALIDATOR_FIELDS = [(_lib.MK_FIELD_BYTES, 0, 48), (_lib.MK_FIELD_BYTES, 48, 32), (_lib.MK_FIELD_BYTES, 80, 32)] + \
                   [(_lib.MK_FIELD_RAW, 112 + 8 * k, 8) for k in range(6)]

# The same type for the reflective mirror (prysm_amd.ssz), for cross-checks.
VALIDATOR_SSZ = S.Struct("ssz.ValidatorRecord", [
    ("Pubkey", S.Bytes()), ("WithdrawalCredentialsHash32", S.Bytes()), ("RandaoCommitmentHash32", S.Bytes()),
    ("RandaoLayers", S.Uint(64)), ("ActivationEpoch", S.Uint(64)), ("ExitEpoch", S.Uint(64)),
    ("WithdrawalEpoch", S.Uint(64)), ("PenalizedEpoch", S.Uint(64)), ("StatusFlags", S.Uint(64))])


def _fields(spec):
    arr = (_lib.Field * len(spec))()
    for i, (k, o, n) in enumerate(spec):
        arr[i].kind, arr[i].offset, arr[i].len = k, o, n
    return arr


def struct_roots(records: np.ndarray, spec=VALIDATOR_FIELDS) -> np.ndarray:
    """Struct hash of every record -> (n, 32) uint8."""
    rec = np.ascontiguousarray(records)
    n = len(rec)
    raw = rec.view(np.uint8).reshape(-1)
    out = np.empty((n, 32), dtype=np.uint8)
    f = _fields(spec)
    _lib.invoke("mk_ssz_struct_roots", _ptr(raw), n, rec.dtype.itemsize, f, len(spec), _ptr(out))
    return out


def struct_list_root(records: np.ndarray, spec=VALIDATOR_FIELDS) -> bytes:
    """TreeHash of a list of such structs (makeSliceHasher -> merkleHash)."""
    rec = np.ascontiguousarray(records)
    raw = rec.view(np.uint8).reshape(-1)
    out = ctypes.create_string_buffer(32)
    f = _fields(spec)
    _lib.invoke("mk_ssz_struct_list_root", _ptr(raw) if raw.size else None, len(rec), rec.dtype.itemsize, f,
                len(spec), out)
    return out.raw


class ValidatorRegistry:
    """[]*ValidatorRecord as one flat array; implements ssz.Hashable."""

    def __init__(self, records: np.ndarray):
        assert records.dtype == VALIDATOR_DTYPE
        self.records = records

    def __len__(self):
        return len(self.records)

    def tree_hash_ssz(self) -> bytes:
        return struct_list_root(self.records)

    TreeHashSSZ = tree_hash_ssz

    def as_dicts(self):
        """The same values in the reflective mirror's representation."""
        out = []
        for r in self.records:
            out.append({"Pubkey": bytes(r["pubkey"]),
                        "WithdrawalCredentialsHash32": bytes(r["withdrawal_credentials_hash32"]),
                        "RandaoCommitmentHash32": bytes(r["randao_commitment_hash32"]),
                        "RandaoLayers": int(r["randao_layers"]), "ActivationEpoch": int(r["activation_epoch"]),
                        "ExitEpoch": int(r["exit_epoch"]), "WithdrawalEpoch": int(r["withdrawal_epoch"]),
                        "PenalizedEpoch": int(r["penalized_epoch"]), "StatusFlags": int(r["status_flags"])})
        return out


# As a descriptor for prysm_amd.ssz.tree_hash (the Hashable hook is checked first).
REGISTRY_HASHABLE = S.Hashable("ssz.ValidatorRegistry", lambda reg: reg.tree_hash_ssz())


def state_root(registry: ValidatorRegistry, balances: np.ndarray) -> bytes:
    """TreeHash of the synthetic State{ValidatorRegistry []*ValidatorRecord;
    ValidatorBalances []uint64} (BASELINE config 3): Keccak(reg_root || bal_root)."""
    reg = registry.tree_hash_ssz()
    bal = np.ascontiguousarray(balances, dtype="<u8")
    bal_root = S.merkle_hash_flat(bal.view(np.uint8), len(bal), 8)
    from .hashutil import hash_batch_var

    return hash_batch_var([reg + bal_root])[0]


class DeviceStateHasher:
    """TreeHash of State{ValidatorRegistry, ValidatorBalances} from records and
    balances resident in HBM (BASELINE config 3, device-resident), with every
    buffer allocated once.  The struct kernel (5 permutations per validator,
    at the VALU issue ceiling) also hashes the level-1 windows of both trees;
    what is left after it is two narrow latency-bound trees (~17 levels of
    one permutation latency each), run side by side on two streams so they
    fill each other's idle issue slots."""

    def __init__(self, n: int, device, schedule: str = "fused"):
        """``schedule``:
        "fused" (default): the struct launch of "level1", then both trees
            above level 1 and the state root in ONE launch on the caller's
            stream (mk_dev_ssz_merkle_top_fused: each tree's lower levels
            reduced per workgroup over the whole chip, the last workgroup of
            each tree its top, the second tree to finish the state root; no
            side stream, no event);
        "level1": one launch for the struct roots and the level-1
            windows of BOTH trees (mk_dev_ssz_struct_list_level1: the
            balances' windows on the lanes the registry's leave free); then
            the two trees' latency-bound levels side by side on two streams,
            the second finisher to complete hashing the state root
            (mk_dev_ssz_merkle_finish_nodes_pair): nothing waits on an event
            between the struct kernel and the root;
        "list": the registry root in one call (mk_dev_ssz_struct_list_root:
            the struct kernel also hashes the registry tree's level-1 windows)
            with the whole balances tree started at once beside it, on the CUs
            the struct kernel's 245-workgroup grid leaves free, then
            Keccak(reg_root || bal_root) after both;
        "two": round 3's schedule (struct roots alone, then the two trees
            side by side).
        Registries the fused kernel does not take (fewer than 2^18 records)
        run "two"."""
        import torch

        from . import device as D

        if schedule not in ("fused", "level1", "list", "two"):
            raise ValueError(f"unknown schedule {schedule!r}")
        self.n, self.dev, self.schedule = n, device, schedule
        L = _lib.load()
        f = _fields(VALIDATOR_FIELDS)
        self.roots = torch.empty(max(32, 32 * n), dtype=torch.uint8, device=device)
        self.msg_ws = torch.empty(max(256, n * L.mk_ssz_struct_msg_len(f, len(VALIDATOR_FIELDS))), dtype=torch.uint8,
                                  device=device)
        self.reg_ws = D.merkle_workspace(n, 32, device)
        self.list_ws = torch.empty(L.mk_ssz_struct_list_workspace_bytes(n, f, len(VALIDATOR_FIELDS)) + 256,
                                   dtype=torch.uint8, device=device) if schedule == "list" else None
        lv1 = schedule in ("level1", "fused")
        self.c1 = -(-n // 8)  # level-1 nodes of the registry tree
        self.nodes = torch.empty(max(32, 32 * self.c1), dtype=torch.uint8, device=device)
        self.fin_ws = D.finish_workspace(self.c1, device) if lv1 else None
        self.cb1 = -(-8 * n // 256)  # level-1 nodes of the balances tree
        self.bnodes = torch.empty(max(32, 32 * self.cb1), dtype=torch.uint8, device=device)
        self.bfin_ws = D.finish_workspace(self.cb1, device) if lv1 else None
        self.top_ws = D.top_fused_workspace(self.c1, self.cb1, device) if (
            schedule == "fused" and self.c1 <= (1 << 20) and self.cb1 <= (1 << 20)) else None
        # reg_root || bal_root || state root || arrival word (zero before first use)
        self.pair_block = torch.zeros(128, dtype=torch.uint8, device=device) if lv1 else None
        self.epoch = 0  # one per submit (mk_dev_ssz_merkle_finish_nodes_pair)
        self.bal_ws = D.merkle_workspace(n, 8, device)
        self.pair = torch.empty(64, dtype=torch.uint8, device=device)  # reg_root || bal_root
        # the state root ("level1": the pair finisher writes it into the pair block)
        # (every schedule writes its root here, so a fallback returns the same tensor)
        self.out = self.pair_block[64:96] if lv1 else torch.empty(32, dtype=torch.uint8, device=device)
        self.side = torch.cuda.Stream(device=device, priority=-1)  # its own hardware queue
        self.ev_roots = torch.cuda.Event()
        self.ev_bal = torch.cuda.Event()

    def submit(self, records, balances):
        """records: (n*160,) uint8 device tensor; balances: (n*8,) uint8.
        Enqueues on the current stream and returns the 32-B root tensor."""
        import torch

        from . import device as D

        n = self.n
        cur = torch.cuda.current_stream(self.dev)
        sched = self.schedule
        if sched != "two" and not D.struct_list_level1_ok(records, n, 160, VALIDATOR_FIELDS):
            sched = "two"
        if sched == "fused" and self.top_ws is None:
            sched = "level1"
        # the level-1 front also takes the balances' windows: 16-B aligned, more
        # than one chunk (mk_dev_ssz_struct_list_level1); otherwise the one-call
        # list root with the balances tree beside it
        if sched in ("level1", "fused") and (balances.data_ptr() % 16 or n * 8 <= 128):
            sched = "list"
            if self.list_ws is None:
                L = _lib.load()
                self.list_ws = torch.empty(
                    L.mk_ssz_struct_list_workspace_bytes(n, _fields(VALIDATOR_FIELDS), len(VALIDATOR_FIELDS)) + 256,
                    dtype=torch.uint8, device=self.dev)
        if sched == "fused":
            # two launches on the caller's stream: struct roots + both trees'
            # level-1 windows, then both trees to the state root
            D.struct_list_level1(records, n, 160, VALIDATOR_FIELDS, self.roots, self.nodes, values=balances,
                                 nvalues=n, value_len=8, value_nodes=self.bnodes)
            self.epoch = self.epoch % ((1 << 30) - 1) + 1
            D.merkle_top_fused(self.nodes, self.c1, n, self.pair_block, self.bnodes, self.cb1, n, epoch=self.epoch,
                               ws=self.top_ws)
            return self.out
        if sched == "level1":
            # one launch: struct roots + the level-1 windows of BOTH trees (the
            # balances' on the lanes the registry's windows leave free)
            D.struct_list_level1(records, n, 160, VALIDATOR_FIELDS, self.roots, self.nodes, values=balances,
                                 nvalues=n, value_len=8, value_nodes=self.bnodes)
            self.ev_roots.record(cur)
            self.side.wait_event(self.ev_roots)
            # the two trees' latency-bound levels side by side; whichever
            # finisher completes second hashes Keccak(reg_root || bal_root)
            self.epoch = self.epoch % ((1 << 30) - 1) + 1
            with torch.cuda.stream(self.side):
                D.merkle_finish_nodes_pair(self.bnodes, self.cb1, n, self.pair_block, 1, self.epoch, ws=self.bfin_ws)
                self.ev_bal.record(self.side)
            D.merkle_finish_nodes_pair(self.nodes, self.c1, n, self.pair_block, 0, self.epoch, ws=self.fin_ws)
            cur.wait_event(self.ev_bal)
            return self.out
        if sched == "list":
            self.ev_roots.record(cur)  # the inputs are ready
            self.side.wait_event(self.ev_roots)
            balances.record_stream(self.side)
            with torch.cuda.stream(self.side):
                D.merkle_hash(balances, n, 8, out=self.pair[32:], ws=self.bal_ws)
                self.ev_bal.record(self.side)
            D.struct_list_root(records, n, 160, VALIDATOR_FIELDS, out=self.pair[:32], ws=self.list_ws)
            cur.wait_event(self.ev_bal)
            D.hash_batch(self.pair, 1, 64, out=self.out)
            return self.out
        D.struct_roots(records, n, 160, VALIDATOR_FIELDS, out=self.roots, ws=self.msg_ws)
        self.ev_roots.record(cur)
        self.side.wait_event(self.ev_roots)
        # balances is read on the side stream after this call returns: keep the
        # caching allocator from reusing its block on the caller's stream meanwhile
        balances.record_stream(self.side)
        with torch.cuda.stream(self.side):
            D.merkle_hash(balances, n, 8, out=self.pair[32:], ws=self.bal_ws)
            self.ev_bal.record(self.side)
        D.merkle_hash(self.roots, n, 32, out=self.pair[:32], ws=self.reg_ws)
        cur.wait_event(self.ev_bal)
        D.hash_batch(self.pair, 1, 64, out=self.out)
        return self.out


class StatePipeline:
    """TreeHash of a stream of States{ValidatorRegistry, ValidatorBalances}
    (BASELINE config 3, one state per ``submit``; hash.go:118-159) with each
    state's two trees folded into the NEXT state's struct launch.

    State i's launch (mk_dev_ssz_struct_list_level1_pipe) writes its struct
    roots and both trees' level-1 nodes, and in one extra lock-step
    permutation per wave levels 2..10 of state i-1's registry tree and levels
    2..4 of its balances tree.  Beside state i+1's launch, on
    the CUs its grid leaves free, one high-priority side stream finishes
    state i-1's trees in turn (the ragged last subtrees, the ~245-node
    registry top, the ~3,900-node balances top); the second of the two tops
    hashes the state root into the state's pair block.  Submits and flush()
    may come from different current streams: each waits for the previous
    launch's event when the stream changed.  **A state's root is therefore written
    one submit later**: the tensor ``submit`` returns is produced once the
    next ``submit`` or ``flush()`` has been called and the side stream has
    run (synchronise, or ``wait()``).  Four buffer sets rotate; a root stays
    valid for the next two submits after it is produced.  Takes what
    mk_ssz_struct_pipe_ok accepts (ValidatorRecords at a 16-B aligned
    address, 16-B aligned balances, 3 x 2^18 < n <= 2^20 on 256 CUs);
    ValueError otherwise."""

    SETS = 4

    def __init__(self, n: int, device):
        import torch

        from . import device as D

        self.n, self.dev = n, torch.device(device)
        self.c1 = -(-n // 8)          # registry level-1 nodes
        self.cb1 = -(-8 * n // 256)   # balances level-1 nodes
        mk = lambda nb: torch.empty(max(32, nb), dtype=torch.uint8, device=self.dev)  # noqa: E731
        self.roots = mk(32 * n)
        self.nodes = [mk(32 * self.c1) for _ in range(self.SETS)]
        self.bnodes = [mk(32 * self.cb1) for _ in range(self.SETS)]
        self.levels = [mk(D.struct_pipe_levels_bytes(n)) for _ in range(self.SETS)]
        self.blevels = [mk(D.struct_pipe_levels_bytes(n, n, 8, 1)) for _ in range(self.SETS)]
        self.pairs = [torch.zeros(128, dtype=torch.uint8, device=self.dev) for _ in range(self.SETS)]
        self.epochs = [0] * self.SETS
        self.top_ws = D.struct_pipe_top_workspace(n, self.dev)
        self.btop_ws = D.struct_pipe_top_workspace(n, self.dev, n, 8, 1)
        self.flush_ws = D.finish_workspace(self.c1, self.dev)
        self.bflush_ws = D.finish_workspace(self.cb1, self.dev)
        # ONE high-priority side stream for both tops, in order: the 245-
        # workgroup grid leaves 1-2 CUs free per XCD, and a kernel's first
        # workgroup goes to the same XCD each time, so two tops launched side
        # by side on two queues queue behind each other for that XCD's free
        # CU, the second until the struct launch ends (0.53 vs 0.49 ms/step,
        # profiles/r05/c3_stream/); in order, the chain (~250 us) fits
        # beside the launch
        self.side = torch.cuda.Stream(device=self.dev, priority=-1)
        self.reg_side = self.bal_side = self.side
        self._i = 0
        self._pending = None  # the set of the state whose trees' slot levels are not built yet
        self._done = {}       # state index -> (registry top event, balances top event)
        self._front_ev = None  # (stream, event) after the last struct launch

    def submit(self, records, balances):
        """records: (n*160,) uint8 device tensor; balances: (n*8,) uint8, both
        16-B aligned.  Returns the state's 32-B root tensor (see the class
        note: written once the next submit or flush() has run)."""
        import torch

        from . import device as D

        n = self.n
        if (not D.struct_pipe_ok(records, n, 160, VALIDATOR_FIELDS) or balances.data_ptr() % 16
                or balances.numel() < 8 * n):
            raise ValueError("StatePipeline: ValidatorRecords and balances at 16-B aligned addresses, "
                             "4 groups of 1024 records per workgroup")
        cur = torch.cuda.current_stream(self.dev)
        i = self._i
        s = i % self.SETS
        self._i += 1
        # set s was last used by state i - 4, set (i + 1) % 4 by state i - 3: one
        # wait every second submit on state i - 3's tops covers both (each side
        # stream runs in order); they ran beside launch i - 1
        if i % 2 == 0:
            for ev in self._done.get(i - self.SETS + 1, ()):
                cur.wait_event(ev)
        self._done.pop(i - self.SETS - 1, None)
        prev = self._pending
        p = prev is not None
        if p and self._front_ev is not None and self._front_ev[0] != cur:
            cur.wait_event(self._front_ev[1])  # launch i - 1 (its nodes are read here) ran on another stream
        D.struct_list_level1_pipe(records, n, 160, VALIDATOR_FIELDS, self.roots, self.nodes[s],
                                  self.nodes[prev] if p else None, self.levels[prev] if p else None,
                                  values=balances, nvalues=n, value_len=8, value_nodes=self.bnodes[s],
                                  prev_value_nodes=self.bnodes[prev] if p else None,
                                  prev_value_levels=self.blevels[prev] if p else None)
        self.epochs[s] = self.epochs[s] % ((1 << 30) - 1) + 1
        k_ev = torch.cuda.Event()
        k_ev.record(cur)
        self._front_ev = (cur, k_ev)
        if p:  # state i - 1's two tops: their slot levels were built by launch i
            self._tops(i - 1, prev, k_ev, pipelined=True)
        self._pending = s
        return self.pairs[s][64:96]

    def _tops(self, state: int, s: int, after, pipelined: bool) -> None:
        import torch

        from . import device as D

        evs = []
        for side, which in ((self.reg_side, 0), (self.bal_side, 1)):
            if which == 0 or side is not self.reg_side:
                side.wait_event(after)
            with torch.cuda.stream(side):
                if pipelined:
                    D.struct_pipe_top(self.nodes[s] if which == 0 else self.bnodes[s], self.n,
                                      self.levels[s] if which == 0 else self.blevels[s], self.pairs[s], which,
                                      self.epochs[s], self.top_ws if which == 0 else self.btop_ws,
                                      nvalues=self.n, value_len=8, which=which)
                elif which == 0:  # the last state: each tree from its level-1 nodes
                    D.merkle_finish_nodes_pair(self.nodes[s], self.c1, self.n, self.pairs[s], 0, self.epochs[s],
                                               ws=self.flush_ws)
                else:
                    D.merkle_finish_nodes_pair(self.bnodes[s], self.cb1, self.n, self.pairs[s], 1, self.epochs[s],
                                               ws=self.bflush_ws)
                ev = torch.cuda.Event()
                ev.record(side)
            evs.append(ev)
        self._done[state] = tuple(evs)

    def flush(self) -> None:
        """Finish the last submitted state's trees (from their level-1 nodes,
        on the side stream); a no-op when nothing is pending."""
        import torch

        if self._pending is not None:
            cur = torch.cuda.current_stream(self.dev)
            if self._front_ev is not None and self._front_ev[0] != cur:
                cur.wait_event(self._front_ev[1])  # the last launch ran on another stream
            ev = torch.cuda.Event()
            ev.record(cur)
            self._tops(self._i - 1, self._pending, ev, pipelined=False)
            self._pending = None

    def wait(self, stream=None) -> None:
        """Make ``stream`` (default: the current one) wait for every root
        produced so far (the side stream's work)."""
        import torch

        st = stream or torch.cuda.current_stream(self.dev)
        st.wait_stream(self.side)


FAR_FUTURE_EPOCH = (1 << 64) - 1  # shared/params/config.go:118
_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix_words(seed: int, word0: int, count: int) -> np.ndarray:
    """Words [word0, word0 + count) of the counter-based SplitMix64 stream of
    SURVEY.md §8d (x = seed + k * 0x9E3779B97F4A7C15, standard mix) —
    the same stream the device kernel k_synth writes (mk_dev_synth_fill)."""
    with np.errstate(over="ignore"):
        k = np.arange(word0, word0 + count, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + k * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _fix_records(w: np.ndarray, first: int = 0) -> np.ndarray:
    """Validator records from raw SplitMix64 words (n x 20 u64, record i =
    stream words 20i .. 20i+19): bytes fields keep the stream; the epochs are
    masked or FarFutureEpoch by index rule; StatusFlags = i % 4."""
    n = w.shape[0]
    i = np.arange(first, first + n, dtype=np.uint64)
    far = np.uint64(FAR_FUTURE_EPOCH)
    w[:, 14] &= np.uint64((1 << 20) - 1)                                          # RandaoLayers
    w[:, 15] &= np.uint64((1 << 30) - 1)                                          # ActivationEpoch
    w[:, 16] = np.where(i % 3 == 0, w[:, 16] & np.uint64((1 << 30) - 1), far)     # ExitEpoch
    w[:, 17] = far                                                                # WithdrawalEpoch
    w[:, 18] = np.where(i % 5 == 0, np.uint64(7), far)                            # PenalizedEpoch
    w[:, 19] = i % np.uint64(4)                                                   # StatusFlags
    return w


def synthetic_registry(n: int, seed: int) -> ValidatorRegistry:
    """SURVEY.md §8d synthetic registry from the SplitMix64 stream (record i
    = words 20i..20i+19 of the stream with `seed`, 160 B), so the same
    registry can be generated on the device (synthetic_registry_device):
    PRNG bytes fields; epochs PRNG or FarFutureEpoch; StatusFlags 0..3."""
    w = _fix_records(splitmix_words(seed, 0, 20 * n).reshape(n, 20))
    return ValidatorRegistry(w.astype("<u8").view(VALIDATOR_DTYPE).reshape(n))


def synthetic_balances(n: int, seed: int) -> np.ndarray:
    """31.5e9 Gwei + (PRNG mod 1e9) (32 ETH +- 0.5 ETH), from
    the SplitMix64 stream with seed + 1."""
    w = splitmix_words(seed + 1, 0, n)
    return (np.uint64(31_500_000_000) + (w & np.uint64((1 << 30) - 1)) % np.uint64(10**9)).astype("<u8")


def synthetic_registry_device(n: int, seed: int, device):
    """The same records as synthetic_registry, generated in HBM (k_synth +
    the index rules as torch integer ops): an (n*160,) uint8 tensor."""
    import torch

    from . import device as D

    raw = torch.empty(n * 160, dtype=torch.uint8, device=device)
    D.synth_fill(raw, seed)
    w = raw.view(torch.int64).view(n, 20)
    i = torch.arange(n, dtype=torch.int64, device=device)
    far = torch.full_like(i, -1)  # 2^64 - 1
    w[:, 14] &= (1 << 20) - 1
    w[:, 15] &= (1 << 30) - 1
    w[:, 16] = torch.where(i % 3 == 0, w[:, 16] & ((1 << 30) - 1), far)
    w[:, 17] = far
    w[:, 18] = torch.where(i % 5 == 0, torch.full_like(i, 7), far)
    w[:, 19] = i % 4
    return raw


def synthetic_balances_device(n: int, seed: int, device):
    import torch

    from . import device as D

    raw = torch.empty(n * 8, dtype=torch.uint8, device=device)
    D.synth_fill(raw, seed + 1)
    w = raw.view(torch.int64)
    w.copy_(31_500_000_000 + (w & ((1 << 30) - 1)) % 1_000_000_000)
    return raw
