"""ORACLE — TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of the reference's reflective SSZ tree-hash, used to
pin the product's host mirror (``prysm_amd.ssz``) against the reference's own
vectors.  Go types are modelled as tuples (Go reflect has no Python
counterpart):

    ("bool",) ("uint", bits) ("bytes",) ("bytearray", n) ("slice", T)
    ("array", T, n) ("struct", go_name, [(field, T), ...]) ("ptr", T)
    ("hashable", go_name, fn) ("string",)        # unsupported kind

Restated from (reference root):
  shared/ssz/hash.go:23-39     TreeHash + ToBytes32 (bytesutil/bytes.go:64-68)
  shared/ssz/hash.go:41-52     error text "hash error: <msg> for input type <T>"
  shared/ssz/hash.go:56-82     makeHasher dispatch (Hashable checked first)
  shared/ssz/hash.go:84-107    getEncoding (raw LE scalars) / hashedEncoding
                               (Keccak(le32(len) || bytes))
  shared/ssz/hash.go:118-139   slice hasher -> merkleHash
  shared/ssz/hash.go:141-159   struct hasher, fields in declaration order,
                               names containing "XXX" skipped
                               (ssz_utils_cache.go:97-111)
  shared/ssz/hash.go:165-178   pointer hasher, nil -> error
  shared/ssz/ssz_utils_cache.go:77-89 + encode.go:79-111  encoder is built
                               before the hasher, so unsupported kinds report
                               "type T is not serializable".
"""
from __future__ import annotations

import struct as _struct

from . import oracle as _o


class HashError(Exception):
    pass


def go_type_name(t) -> str:
    k = t[0]
    if k == "nil":
        return "<nil>"
    if k == "bool":
        return "bool"
    if k == "uint":
        return f"uint{t[1]}"
    if k == "bytes":
        return "[]uint8"
    if k == "bytearray":
        return f"[{t[1]}]uint8"
    if k == "slice":
        return "[]" + go_type_name(t[1])
    if k == "array":
        return f"[{t[2]}]" + go_type_name(t[1])
    if k in ("struct", "hashable"):
        return t[1]
    if k == "ptr":
        return "*" + go_type_name(t[1])
    if k == "string":
        return "string"
    raise ValueError(t)


def _check_serializable(t):
    """makeEncoder's recursive type walk (encode.go:79-111, 196-221, 255-260,
    297-302): returns an error message or None."""
    k = t[0]
    if k in ("bool", "uint", "bytes", "bytearray", "hashable"):
        return None
    if k in ("slice", "array"):
        e = _check_serializable(t[1])
        return None if e is None else f"failed to get ssz utils: {e}"
    if k == "struct":
        for name, ft in t[2]:
            if "XXX" in name:
                continue
            e = _check_serializable(ft)
            if e is not None:
                return f"failed to get ssz utils: {e}"
        return None
    if k == "ptr":
        return _check_serializable(t[1])
    return f"type {go_type_name(t)} is not serializable"


def _scalar_encoding(t, v) -> bytes:
    if t[0] == "bool":
        return b"\x01" if v else b"\x00"
    return int(v).to_bytes(t[1] // 8, "little")


def _hasher(t, v) -> bytes:
    k = t[0]
    if k == "hashable":
        return bytes(t[2](v))
    if k in ("bool", "uint"):
        return _scalar_encoding(t, v)
    if k in ("bytes", "bytearray"):
        b = bytes(v)
        return _o.keccak256(_struct.pack("<I", len(b)) + b)
    if k in ("slice", "array"):
        elems = []
        for e in v:
            try:
                elems.append(_hasher(t[1], e))
            except HashError as err:
                raise HashError(f"failed to hash element of slice/array: {err}")
        return _o.merkle_hash(elems)
    if k == "struct":
        parts = []
        for name, ft in t[2]:
            if "XXX" in name:
                continue
            try:
                parts.append(_hasher(ft, v[name]))
            except HashError as err:
                raise HashError(f"failed to hash field of struct: {err}")
        return _o.keccak256(b"".join(parts))
    if k == "ptr":
        if v is None:
            raise HashError("nil is not supported")
        return _hasher(t[1], v)
    raise HashError(f"type {go_type_name(t)} is not hashable")


def tree_hash(t, v) -> bytes:
    """ssz.TreeHash (hash.go:23-39).  Raises HashError with the reference's
    exact error text."""
    if t is None or t[0] == "nil":
        raise HashError("hash error: nil is not supported for input type <nil>")
    e = _check_serializable(t)
    if e is not None:
        raise HashError(f"hash error: {e} for input type {go_type_name(t)}")
    try:
        out = _hasher(t, v)
    except HashError as err:
        raise HashError(f"hash error: {err} for input type {go_type_name(t)}")
    return (out + b"\0" * 32)[:32]
