"""Test helpers: JSON fixture type tuples -> prysm_amd.ssz descriptors, and
the synthetic validator registry of SURVEY.md §8d (pb.Validator field order,
proto/beacon/p2p/v1/types.pb.go:661-671, StatusFlags widened to uint64)."""
import numpy as np

from prysm_amd import ssz as S


def _hashable_fn(v):
    # hash_test.go:25-32: 28 zero bytes followed by the 4-byte value
    return (bytes(28) + bytes(v))[:32]


def to_ssz_type(t):
    k = t[0]
    if k == "nil":
        return None
    if k == "bool":
        return S.Bool()
    if k == "uint":
        return S.Uint(t[1])
    if k == "bytes":
        return S.Bytes()
    if k == "bytearray":
        return S.ByteArray(t[1])
    if k == "slice":
        return S.Slice(to_ssz_type(t[1]))
    if k == "array":
        return S.Array(to_ssz_type(t[1]), t[2])
    if k == "struct":
        return S.Struct(t[1], [(n, to_ssz_type(ft)) for n, ft in t[2]])
    if k == "ptr":
        return S.Ptr(to_ssz_type(t[1]))
    if k == "hashable":
        return S.Hashable(t[1], _hashable_fn)
    if k == "string":
        return S.Unsupported("string")
    raise ValueError(t)


def to_value(t, v):
    k = t[0]
    if v is None:
        return None
    if k in ("slice", "array"):
        return [to_value(t[1], e) for e in v]
    if k == "struct":
        return {n: to_value(ft, v[n]) for n, ft in t[2]}
    if k == "ptr":
        return to_value(t[1], v)
    if k in ("bytes", "bytearray"):
        return bytes(v)
    return v


VALIDATOR_FIELDS = [("Pubkey", "bytes"), ("WithdrawalCredentialsHash32", "bytes"),
                    ("RandaoCommitmentHash32", "bytes"), ("RandaoLayers", "u64"), ("ActivationEpoch", "u64"),
                    ("ExitEpoch", "u64"), ("WithdrawalEpoch", "u64"), ("PenalizedEpoch", "u64"),
                    ("StatusFlags", "u64"), ("XXX_unrecognized", "bytes")]


def validator_registry(n, seed):
    """(oracle type tuple, prysm_amd type, values) for []*ValidatorRecord."""
    rng = np.random.default_rng(seed & 0xFFFFFFFF)
    far = (1 << 64) - 1  # FarFutureEpoch, params/config.go:118
    vals = []
    for i in range(n):
        v = {"Pubkey": bytes(rng.integers(0, 256, 48, dtype=np.uint8)),
             "WithdrawalCredentialsHash32": bytes(rng.integers(0, 256, 32, dtype=np.uint8)),
             "RandaoCommitmentHash32": bytes(rng.integers(0, 256, 32, dtype=np.uint8)),
             "RandaoLayers": int(rng.integers(0, 1 << 20)),
             "ActivationEpoch": int(rng.integers(0, 1 << 30)),
             "ExitEpoch": far if i % 3 else int(rng.integers(0, 1 << 30)),
             "WithdrawalEpoch": far,
             "PenalizedEpoch": far if i % 5 else 7,
             "StatusFlags": int(i % 4),
             "XXX_unrecognized": b"ignored"}
        vals.append(v)
    ref_fields = [(n, ("bytes",) if k == "bytes" else ("uint", 64)) for n, k in VALIDATOR_FIELDS]
    t_ref = ("slice", ("ptr", ("struct", "ssz.ValidatorRecord", ref_fields)))
    ssz_fields = [(n, S.Bytes() if k == "bytes" else S.Uint(64)) for n, k in VALIDATOR_FIELDS]
    t_ssz = S.Slice(S.Ptr(S.Struct("ssz.ValidatorRecord", ssz_fields)))
    return t_ref, t_ssz, vals


def to_ref_type(t):
    """prysm_amd.ssz descriptor -> oracle/ssz_ref type tuple (inverse of to_ssz_type)."""
    if isinstance(t, S.Bool):
        return ("bool",)
    if isinstance(t, S.Uint):
        return ("uint", t.bits)
    if isinstance(t, S.Bytes):
        return ("bytes",)
    if isinstance(t, S.ByteArray):
        return ("bytearray", t.n)
    if isinstance(t, S.Slice):
        return ("slice", to_ref_type(t.elem))
    if isinstance(t, S.Array):
        return ("array", to_ref_type(t.elem), t.n)
    if isinstance(t, S.Struct):
        return ("struct", t.go_name, [(n, to_ref_type(ft)) for n, ft in t.fields])
    if isinstance(t, S.Ptr):
        return ("ptr", to_ref_type(t.elem))
    if isinstance(t, S.Hashable):
        return ("hashable", t.go_name, t.fn)
    return ("string",)
