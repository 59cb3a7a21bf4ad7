"""State tree hash: ssz.TreeHash of a whole
``pb.BeaconState`` on the engine.

The reference roots a state with ``Keccak(proto.Marshal(state))``
(beacon-chain/core/state/state.go:168-174) and leaves "Replace by state tree
hashing algorithm" TODOs at beacon-chain/blockchain/service.go:115 and :273.
This module is that replacement: the reference's own reflective TreeHash
(shared/ssz/hash.go:23-239) of the state struct, field by field in
declaration order (proto/beacon/p2p/v1/types.pb.go:50-79, the XXX_ fields
skipped as structFields does, ssz_utils_cache.go:100), computed with a fixed
number of batched library calls instead of one Keccak per field element:

  1. every 32-B bytes field of the state (randao mixes, block / batched /
     index roots, crosslink roots, attestation-data roots, eth1 hashes,
     seeds): hashedEncoding K(le32(32) || b), one 36-B batch; the variable
     length bitfields one var-length batch;
  2. the validator registry: typed struct roots + merkleHash
     (mk_ssz_struct_list_root, the Hashable fast path of registry.py);
  3. struct messages of the small structs (CrosslinkRecord, AttestationData,
     Eth1Data), one var-length batch; then PendingAttestationRecord and
     Eth1DataVote (their messages contain step-3 roots), one more batch;
  4. every list of the state (balances, the 8192-entry root arrays, penalized
     balances, crosslinks, attestations, eth1 votes) in ONE segmented
     merkleHash call (mk_ssz_merkle_many);
  5. the state struct: K(concatenation of the 25 field outputs).

SSZ legality: ``Validator.StatusFlags`` is an int32 enum,
which makeEncoder rejects (encode.go:107-108), so it is widened to uint64;
``LatestEth1Data`` and ``Fork`` are pointers, which must be non-nil
(hash.go:172-173).  ``STATE_SSZ`` is the same type for the reflective mirror
(prysm_amd.ssz.tree_hash), and the tests check both paths against the
oracle's restatement (oracle/ssz_ref.py).
"""
from __future__ import annotations

import struct as _st
from dataclasses import dataclass, field
from typing import List

import numpy as np

from . import registry as R
from . import ssz as S
from .hashutil import hash_batch, hash_batch_var

# shared/params/config.go:96-105
SHARD_COUNT = 1024
LATEST_BLOCK_ROOTS_LENGTH = 8192
LATEST_RANDAO_MIXES_LENGTH = 8192
LATEST_PENALIZED_EXIT_LENGTH = 8192
LATEST_INDEX_ROOTS_LENGTH = 8192

_U64 = S.Uint(64)
_B = S.Bytes()

CROSSLINK_SSZ = S.Struct("pb.CrosslinkRecord", [("Epoch", _U64), ("ShardBlockRootHash32", _B)])
ATTESTATION_DATA_SSZ = S.Struct("pb.AttestationData", [
    ("Slot", _U64), ("Shard", _U64), ("BeaconBlockRootHash32", _B), ("EpochBoundaryRootHash32", _B),
    ("ShardBlockRootHash32", _B), ("LatestCrosslinkRootHash32", _B), ("JustifiedEpoch", _U64),
    ("JustifiedBlockRootHash32", _B), ("JustifiedSlot", _U64)])
PENDING_ATTESTATION_SSZ = S.Struct("pb.PendingAttestationRecord", [
    ("Data", S.Ptr(ATTESTATION_DATA_SSZ)), ("AggregationBitfield", _B), ("CustodyBitfield", _B),
    ("SlotIncluded", _U64)])
ETH1_DATA_SSZ = S.Struct("pb.Eth1Data", [("DepositRootHash32", _B), ("BlockHash32", _B)])
ETH1_VOTE_SSZ = S.Struct("pb.Eth1DataVote", [("Eth1Data", S.Ptr(ETH1_DATA_SSZ)), ("VoteCount", _U64)])
FORK_SSZ = S.Struct("pb.Fork", [("PreviousVersion", _U64), ("CurrentVersion", _U64), ("Epoch", _U64)])

# pb.BeaconState field order (types.pb.go:50-79); XXX_ fields present and skipped
STATE_FIELDS = [
    ("ValidatorRegistry", S.Slice(S.Ptr(R.VALIDATOR_SSZ))),
    ("ValidatorRegistryUpdateEpoch", _U64),
    ("ValidatorBalances", S.Slice(_U64)),
    ("LatestRandaoMixesHash32S", S.Slice(_B)),
    ("PreviousEpochStartShard", _U64),
    ("CurrentEpochStartShard", _U64),
    ("PreviousCalculationEpoch", _U64),
    ("CurrentCalculationEpoch", _U64),
    ("PreviousEpochSeedHash32", _B),
    ("CurrentEpochSeedHash32", _B),
    ("PreviousJustifiedEpoch", _U64),
    ("JustifiedEpoch", _U64),
    ("JustificationBitfield", _U64),
    ("FinalizedEpoch", _U64),
    ("LatestCrosslinks", S.Slice(S.Ptr(CROSSLINK_SSZ))),
    ("LatestBlockRootHash32S", S.Slice(_B)),
    ("BatchedBlockRootHash32S", S.Slice(_B)),
    ("LatestPenalizedBalances", S.Slice(_U64)),
    ("LatestAttestations", S.Slice(S.Ptr(PENDING_ATTESTATION_SSZ))),
    ("LatestIndexRootHash32S", S.Slice(_B)),
    ("LatestEth1Data", S.Ptr(ETH1_DATA_SSZ)),
    ("Eth1DataVotes", S.Slice(S.Ptr(ETH1_VOTE_SSZ))),
    ("GenesisTime", _U64),
    ("Fork", S.Ptr(FORK_SSZ)),
    ("Slot", _U64),
    ("XXX_NoUnkeyedLiteral", S.Unsupported("struct {}")),
    ("XXX_unrecognized", _B),
    ("XXX_sizecache", S.Unsupported("int32")),
]
STATE_SSZ = S.Struct("pb.BeaconState", STATE_FIELDS)

_SCALARS = ["ValidatorRegistryUpdateEpoch", "PreviousEpochStartShard", "CurrentEpochStartShard",
            "PreviousCalculationEpoch", "CurrentCalculationEpoch", "PreviousJustifiedEpoch", "JustifiedEpoch",
            "JustificationBitfield", "FinalizedEpoch", "GenesisTime", "Slot"]


@dataclass
class Attestations:
    """[]*PendingAttestationRecord as columns (AttestationData inlined)."""
    slot: np.ndarray            # u64 (a,)
    shard: np.ndarray           # u64 (a,)
    roots: np.ndarray           # (a, 4, 32): beacon block / epoch boundary / shard block / latest crosslink
    justified_epoch: np.ndarray
    justified_root: np.ndarray  # (a, 32)
    justified_slot: np.ndarray
    aggregation_bitfield: List[bytes]
    custody_bitfield: List[bytes]
    slot_included: np.ndarray

    def __len__(self):
        return len(self.slot)


@dataclass
class BeaconState:
    """A synthetic, SSZ-legal pb.BeaconState with its lists as flat arrays."""
    registry: R.ValidatorRegistry
    balances: np.ndarray                 # u64 (n,)
    randao_mixes: np.ndarray             # (8192, 32)
    seeds: np.ndarray                    # (2, 32): previous, current epoch seed
    crosslink_epochs: np.ndarray         # u64 (1024,)
    crosslink_roots: np.ndarray          # (1024, 32)
    latest_block_roots: np.ndarray       # (8192, 32)
    batched_block_roots: np.ndarray      # (m, 32)
    penalized_balances: np.ndarray       # u64 (8192,)
    attestations: Attestations
    index_roots: np.ndarray              # (8192, 32)
    eth1_data: np.ndarray                # (2, 32): deposit root, block hash
    eth1_votes: np.ndarray               # (v, 2, 32)
    eth1_vote_counts: np.ndarray         # u64 (v,)
    fork: np.ndarray                     # u64 (3,)
    scalars: dict = field(default_factory=dict)

    # ---------------------------------------------------------------- the engine path
    def tree_hash_ssz(self) -> bytes:
        """ssz.TreeHash(state): 7 library calls, no per-element Python work."""
        att = self.attestations
        a, v = len(att), len(self.eth1_votes)
        # 1. hashedEncoding of every 32-B bytes field, one fixed-length batch
        b32 = np.concatenate([self.randao_mixes, self.seeds, self.crosslink_roots, self.latest_block_roots,
                              self.batched_block_roots, self.index_roots, att.roots.reshape(-1, 32),
                              att.justified_root, self.eth1_data, self.eth1_votes.reshape(-1, 32)])
        msgs = np.empty((len(b32), 36), dtype=np.uint8)
        msgs[:, :4] = np.frombuffer(_st.pack("<I", 32), dtype=np.uint8)
        msgs[:, 4:] = b32
        h = hash_batch(msgs, 36)
        cut = np.cumsum([0, len(self.randao_mixes), 2, len(self.crosslink_roots), len(self.latest_block_roots),
                         len(self.batched_block_roots), len(self.index_roots), 4 * a, a, 2, 2 * v])
        h_randao, h_seeds, h_cross, h_block, h_batched, h_index, h_att4, h_just, h_eth1, h_votes = (
            h[cut[i]:cut[i + 1]] for i in range(10))
        h_att4 = h_att4.reshape(a, 4 * 32)
        bits = hash_batch_var([_st.pack("<I", len(x)) + x for x in att.aggregation_bitfield + att.custody_bitfield])
        # 2. the registry (typed Hashable path: struct kernel + merkleHash)
        reg_root = self.registry.tree_hash_ssz()
        # 3. small structs: CrosslinkRecord, AttestationData, Eth1Data (latest + per vote)
        le = lambda x: np.ascontiguousarray(x, dtype="<u8").reshape(-1, 1).view(np.uint8)  # noqa: E731
        cross_msg = np.concatenate([le(self.crosslink_epochs), h_cross], axis=1)
        att_msg = np.concatenate([le(att.slot), le(att.shard), h_att4, le(att.justified_epoch), h_just,
                                  le(att.justified_slot)], axis=1)
        eth1_msg = np.concatenate([h_eth1.reshape(1, 64), h_votes.reshape(v, 64)])
        r3 = hash_batch_var([bytes(r) for r in cross_msg] + [bytes(r) for r in att_msg] + [bytes(r) for r in eth1_msg])
        cross_roots = b"".join(r3[:len(cross_msg)])
        att_data = r3[len(cross_msg):len(cross_msg) + a]
        eth1_root, vote_eth1 = r3[len(cross_msg) + a], r3[len(cross_msg) + a + 1:]
        # PendingAttestationRecord / Eth1DataVote messages hold step-3 roots
        rec_msgs = [att_data[i] + bits[i] + bits[a + i] + _st.pack("<Q", int(att.slot_included[i]))
                    for i in range(a)]
        vote_msgs = [vote_eth1[i] + _st.pack("<Q", int(self.eth1_vote_counts[i])) for i in range(v)]
        r4 = hash_batch_var(rec_msgs + vote_msgs)
        att_roots, vote_roots = b"".join(r4[:a]), b"".join(r4[a:])
        # 4. every list of the state in one segmented merkleHash call
        lists = [(self.balances.astype("<u8").view(np.uint8), len(self.balances), 8),
                 (h_randao, len(h_randao), 32), (np.frombuffer(cross_roots, np.uint8), len(cross_msg), 32),
                 (h_block, len(h_block), 32), (h_batched, len(h_batched), 32),
                 (self.penalized_balances.astype("<u8").view(np.uint8), len(self.penalized_balances), 8),
                 (np.frombuffer(att_roots, np.uint8), a, 32), (h_index, len(h_index), 32),
                 (np.frombuffer(vote_roots, np.uint8), v, 32)]
        buf, offs, pos = [], [], 0
        for arr, _, _ in lists:
            pad = (-pos) % 16
            buf.append(np.zeros(pad, np.uint8))
            pos += pad
            offs.append(pos)
            flat = np.ascontiguousarray(arr, dtype=np.uint8).reshape(-1)
            buf.append(flat)
            pos += flat.size
        roots = _merkle_many_mixed(np.concatenate(buf), offs, [x[1] for x in lists], [x[2] for x in lists])
        (bal_root, randao_root, cross_root, block_root, batched_root, pen_root, att_root, index_root,
         votes_root) = roots
        # 5. the state struct: field outputs in declaration order
        sc = self.scalars
        u = lambda name: _st.pack("<Q", int(sc[name]))  # noqa: E731
        fork_root = hash_batch_var([b"".join(_st.pack("<Q", int(x)) for x in self.fork)])[0]
        msg = b"".join([
            reg_root, u("ValidatorRegistryUpdateEpoch"), bal_root, randao_root, u("PreviousEpochStartShard"),
            u("CurrentEpochStartShard"), u("PreviousCalculationEpoch"), u("CurrentCalculationEpoch"),
            bytes(h_seeds[0]), bytes(h_seeds[1]), u("PreviousJustifiedEpoch"), u("JustifiedEpoch"),
            u("JustificationBitfield"), u("FinalizedEpoch"), cross_root, block_root, batched_root, pen_root,
            att_root, index_root, eth1_root, votes_root, u("GenesisTime"), fork_root, u("Slot")])
        return hash_batch_var([msg])[0]

    TreeHashSSZ = tree_hash_ssz

    # ---------------------------------------------------------------- reflective form
    def as_value(self) -> dict:
        """The same state as a value of STATE_SSZ (dicts / lists / bytes) for the
        reflective mirror and the oracle."""
        att = self.attestations
        b = lambda a: [bytes(r) for r in a]  # noqa: E731
        d = {
            "ValidatorRegistry": self.registry.as_dicts(),
            "ValidatorBalances": [int(x) for x in self.balances],
            "LatestRandaoMixesHash32S": b(self.randao_mixes),
            "PreviousEpochSeedHash32": bytes(self.seeds[0]), "CurrentEpochSeedHash32": bytes(self.seeds[1]),
            "LatestCrosslinks": [{"Epoch": int(e), "ShardBlockRootHash32": bytes(r)}
                                 for e, r in zip(self.crosslink_epochs, self.crosslink_roots)],
            "LatestBlockRootHash32S": b(self.latest_block_roots),
            "BatchedBlockRootHash32S": b(self.batched_block_roots),
            "LatestPenalizedBalances": [int(x) for x in self.penalized_balances],
            "LatestAttestations": [{
                "Data": {"Slot": int(att.slot[i]), "Shard": int(att.shard[i]),
                         "BeaconBlockRootHash32": bytes(att.roots[i, 0]),
                         "EpochBoundaryRootHash32": bytes(att.roots[i, 1]),
                         "ShardBlockRootHash32": bytes(att.roots[i, 2]),
                         "LatestCrosslinkRootHash32": bytes(att.roots[i, 3]),
                         "JustifiedEpoch": int(att.justified_epoch[i]),
                         "JustifiedBlockRootHash32": bytes(att.justified_root[i]),
                         "JustifiedSlot": int(att.justified_slot[i])},
                "AggregationBitfield": att.aggregation_bitfield[i], "CustodyBitfield": att.custody_bitfield[i],
                "SlotIncluded": int(att.slot_included[i])} for i in range(len(att))],
            "LatestIndexRootHash32S": b(self.index_roots),
            "LatestEth1Data": {"DepositRootHash32": bytes(self.eth1_data[0]), "BlockHash32": bytes(self.eth1_data[1])},
            "Eth1DataVotes": [{"Eth1Data": {"DepositRootHash32": bytes(x[0]), "BlockHash32": bytes(x[1])},
                               "VoteCount": int(c)} for x, c in zip(self.eth1_votes, self.eth1_vote_counts)],
            "Fork": {"PreviousVersion": int(self.fork[0]), "CurrentVersion": int(self.fork[1]),
                     "Epoch": int(self.fork[2])},
            "XXX_NoUnkeyedLiteral": None, "XXX_unrecognized": b"", "XXX_sizecache": 0,
        }
        for name in _SCALARS:
            d[name] = int(self.scalars[name])
        return d


def _merkle_many_mixed(buf: np.ndarray, offs, ns, item_lens) -> List[bytes]:
    """mk_ssz_merkle_many with per-list item lengths (host buffer)."""
    from . import _lib
    from .hashutil import _ptr

    k = len(ns)
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    n = np.ascontiguousarray(ns, dtype=np.uint64)
    il = np.ascontiguousarray(item_lens, dtype=np.uint32)
    out = np.empty((k, 32), dtype=np.uint8)
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    _lib.invoke("mk_ssz_merkle_many", _ptr(buf), _ptr(o), _ptr(n), _ptr(il), k, _ptr(out))
    return [bytes(r) for r in out]


def synthetic_state(n_validators: int, seed: int, n_attestations: int = 128, n_batched: int = 16,
                    n_votes: int = 4, lists_len: int = LATEST_BLOCK_ROOTS_LENGTH,
                    shards: int = SHARD_COUNT) -> BeaconState:
    """A synthetic BeaconState from the SplitMix64 stream:
    the registry and balances of registry.py, the 8192-entry root arrays,
    1024 crosslinks, `n_attestations` pending attestations with bitfields of
    16..48 bytes, `n_batched` batched block roots and `n_votes` eth1 votes."""
    words = iter(range(1, 1 << 20))

    def rnd(nbytes: int) -> np.ndarray:
        w = R.splitmix_words(seed + 1000 * next(words), 0, (nbytes + 7) // 8)
        return w.view(np.uint8)[:nbytes].copy()

    def u64(count: int, mask: int = (1 << 40) - 1) -> np.ndarray:
        return R.splitmix_words(seed + 1000 * next(words), 0, count) & np.uint64(mask)

    a = n_attestations
    agg_len = 16 + (u64(a, 31) & np.uint64(31)).astype(np.int64)
    cust_len = 16 + (u64(a, 31) & np.uint64(31)).astype(np.int64)
    att = Attestations(
        slot=u64(a), shard=u64(a, shards - 1), roots=rnd(a * 128).reshape(a, 4, 32), justified_epoch=u64(a),
        justified_root=rnd(a * 32).reshape(a, 32), justified_slot=u64(a),
        aggregation_bitfield=[bytes(rnd(int(L))) for L in agg_len],
        custody_bitfield=[bytes(rnd(int(L))) for L in cust_len], slot_included=u64(a))
    st = BeaconState(
        registry=R.synthetic_registry(n_validators, seed), balances=R.synthetic_balances(n_validators, seed),
        randao_mixes=rnd(lists_len * 32).reshape(lists_len, 32), seeds=rnd(64).reshape(2, 32),
        crosslink_epochs=u64(shards), crosslink_roots=rnd(shards * 32).reshape(shards, 32),
        latest_block_roots=rnd(lists_len * 32).reshape(lists_len, 32),
        batched_block_roots=rnd(n_batched * 32).reshape(n_batched, 32),
        penalized_balances=u64(lists_len, (1 << 45) - 1), attestations=att,
        index_roots=rnd(lists_len * 32).reshape(lists_len, 32), eth1_data=rnd(64).reshape(2, 32),
        eth1_votes=rnd(n_votes * 64).reshape(n_votes, 2, 32), eth1_vote_counts=u64(n_votes, 1023),
        fork=u64(3, 15))
    sc = u64(len(_SCALARS))
    st.scalars = {name: int(x) for name, x in zip(_SCALARS, sc)}
    return st
