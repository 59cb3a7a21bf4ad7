"""Host mirror of ``shared/ssz`` tree-hashing over the HIP engine.

Reference (file:line under the reference root):
  TreeHash            shared/ssz/hash.go:23-39   (+ bytesutil.ToBytes32 bytes.go:64-68)
  hash error text     shared/ssz/hash.go:41-52
  makeHasher          shared/ssz/hash.go:56-82   (Hashable checked first: the plugin hook)
  getEncoding /       shared/ssz/hash.go:84-107  (raw LE scalars / Keccak(le32(len)||bytes))
  hashedEncoding
  makeSliceHasher     shared/ssz/hash.go:118-139 (element hashes -> merkleHash)
  makeStructHasher    shared/ssz/hash.go:141-159 (+ structFields ssz_utils_cache.go:97-111)
  makePtrHasher       shared/ssz/hash.go:165-178
  merkleHash          shared/ssz/hash.go:194-239
  encoder-first error ssz_utils_cache.go:77-89, encode.go:79-111

Go's reflection is replaced by explicit type descriptors (``Uint(16)``,
``Slice(T)``, ``Struct("ssz.simpleStruct", [("B", Uint(16)), ...])`` ...).
Evaluation is breadth-first and batched: all elements of a list are hashed
by one library call per nesting level (bytes fields -> one variable-length
Keccak batch, struct concatenations -> one batch, all lists of a nesting
level -> one segmented merkleHash call, mk_ssz_merkle_many), instead of one
Keccak call per field as in the reference's recursive hasher.  Errors carry
the reference's exact text.
"""
from __future__ import annotations

import ctypes
import struct as _st
from typing import Any, Callable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from .hashutil import _flatten, _ptr, hash_batch, hash_batch_var

SSZ_CHUNK_SIZE = 128  # hash.go:15
HASH_LENGTH = 32  # hash.go:14


class HashError(Exception):
    """Carries the reference's error text, e.g.
    ``hash error: nil is not supported for input type *[]uint8``."""


# ----------------------------------------------------------------- type model
class SSZType:
    go_name = "?"


class Bool(SSZType):
    go_name = "bool"


class Uint(SSZType):
    def __init__(self, bits: int):
        assert bits in (8, 16, 32, 64)
        self.bits = bits
        self.go_name = f"uint{bits}"


class Bytes(SSZType):
    go_name = "[]uint8"


class ByteArray(SSZType):
    def __init__(self, n: int):
        self.n = n
        self.go_name = f"[{n}]uint8"


class Slice(SSZType):
    def __init__(self, elem: SSZType):
        self.elem = elem
        self.go_name = "[]" + elem.go_name


class Array(SSZType):
    def __init__(self, elem: SSZType, n: int):
        self.elem, self.n = elem, n
        self.go_name = f"[{n}]{elem.go_name}"


class Struct(SSZType):
    def __init__(self, go_name: str, fields: Sequence[Tuple[str, SSZType]]):
        self.go_name = go_name
        self.fields = list(fields)

    def hashed_fields(self):
        # structFields skips names containing "XXX" (ssz_utils_cache.go:100)
        return [(n, t) for n, t in self.fields if "XXX" not in n]


class Ptr(SSZType):
    def __init__(self, elem: SSZType):
        self.elem = elem
        self.go_name = "*" + elem.go_name


class Hashable(SSZType):
    """A type implementing ssz.Hashable (hash.go:18-20): ``fn(value)`` plays
    TreeHashSSZ and returns 32 bytes (or raises HashError)."""

    def __init__(self, go_name: str, fn: Callable[[Any], bytes]):
        self.go_name, self.fn = go_name, fn


class Unsupported(SSZType):
    """Any other Go kind (string, int, map, ...): not serializable."""

    def __init__(self, go_name: str):
        self.go_name = go_name


# ----------------------------------------------------------------- helpers
def _field(v, name):
    return v[name] if isinstance(v, dict) else getattr(v, name)


def _check_serializable(t: SSZType) -> Optional[str]:
    """makeEncoder's recursive walk; the encoder is generated before the
    hasher, so unsupported kinds report "is not serializable"."""
    if isinstance(t, (Bool, Uint, Bytes, ByteArray, Hashable)):
        return None
    if isinstance(t, (Slice, Array)):
        e = _check_serializable(t.elem)
        return None if e is None else f"failed to get ssz utils: {e}"
    if isinstance(t, Struct):
        for _, ft in t.hashed_fields():
            e = _check_serializable(ft)
            if e is not None:
                return f"failed to get ssz utils: {e}"
        return None
    if isinstance(t, Ptr):
        return _check_serializable(t.elem)
    return f"type {t.go_name} is not serializable"


def _trivial(t: SSZType) -> bool:
    """True when no value of type t can make the hasher fail or call a
    Hashable hook (no pointers, no Hashable): validation can skip it."""
    tr = getattr(t, "_trivial", None)
    if tr is None:
        if isinstance(t, (Ptr, Hashable)):
            tr = False
        elif isinstance(t, (Slice, Array)):
            tr = _trivial(t.elem)
        elif isinstance(t, Struct):
            tr = all(_trivial(ft) for _, ft in t.hashed_fields())
        else:
            tr = True
        t._trivial = tr
    return tr


def _validate(t: SSZType, v, memo: dict) -> None:
    """Depth-first pass in the reference's evaluation order that raises the
    first error the recursive Go hasher would hit (nil pointers, Hashable
    errors), with the same nesting of messages.  Hashable results are
    memoised so TreeHashSSZ runs once.  Subtrees that cannot fail are
    skipped; a list of pointers to such a type only checks for nil."""
    if _trivial(t):
        return
    if isinstance(t, Hashable):
        memo[id(v)] = bytes(t.fn(v))
        return
    if isinstance(t, (Slice, Array)):
        if isinstance(t.elem, Ptr) and _trivial(t.elem.elem):
            for e in v:
                if e is None:
                    raise HashError("failed to hash element of slice/array: nil is not supported")
            return
        for e in v:
            try:
                _validate(t.elem, e, memo)
            except HashError as err:
                raise HashError(f"failed to hash element of slice/array: {err}")
        return
    if isinstance(t, Struct):
        for name, ft in t.hashed_fields():
            try:
                _validate(ft, _field(v, name), memo)
            except HashError as err:
                raise HashError(f"failed to hash field of struct: {err}")
        return
    if isinstance(t, Ptr):
        if v is None:
            raise HashError("nil is not supported")
        _validate(t.elem, v, memo)


def _scalar_bytes(t: SSZType, vals) -> np.ndarray:
    """getEncoding of bool/uintN: raw little-endian, not hashed (hash.go:84-98)."""
    if isinstance(t, Bool):
        return np.asarray([1 if x else 0 for x in vals] if not isinstance(vals, np.ndarray) else vals,
                          dtype=np.uint8).reshape(-1, 1)
    dt = np.dtype(f"<u{t.bits // 8}")
    a = np.asarray(vals, dtype=dt) if not isinstance(vals, np.ndarray) else vals.astype(dt, copy=False)
    return a.reshape(-1).view(np.uint8).reshape(-1, t.bits // 8)


def _hash_size(t: SSZType) -> int:
    """Length of the hasher's output for type t (hash.go:56-82)."""
    if isinstance(t, Bool):
        return 1
    if isinstance(t, Uint):
        return t.bits // 8
    if isinstance(t, Ptr):
        return _hash_size(t.elem)
    return 32


def _column(vals: Sequence, name: str) -> list:
    if vals and isinstance(vals[0], dict):
        return [v[name] for v in vals]
    return [_field(v, name) for v in vals]


def _hash_bytes_values(vals: Sequence) -> np.ndarray:
    """hashedEncoding of every value: Keccak(le32(len) || bytes) (hash.go:100-107,
    encode.go:148-159), one batched call; equal lengths take the fixed-length
    kernels."""
    bs = [bytes(v) for v in vals]
    L0 = len(bs[0])
    if all(len(b) == L0 for b in bs):
        msgs = np.empty((len(bs), 4 + L0), dtype=np.uint8)
        msgs[:, :4] = np.frombuffer(_st.pack("<I", L0), dtype=np.uint8)
        if L0:
            msgs[:, 4:] = np.frombuffer(b"".join(bs), dtype=np.uint8).reshape(len(bs), L0)
        return hash_batch(msgs, 4 + L0)
    return np.frombuffer(b"".join(hash_batch_var([_st.pack("<I", len(b)) + b for b in bs])),
                         dtype=np.uint8).reshape(len(bs), 32)


def _hash_many(t: SSZType, vals: Sequence, memo: dict) -> np.ndarray:
    """Hasher output of every value in ``vals`` (all of type t) as an
    (n, size) uint8 matrix, batched on the GPU: one library call per
    nesting level (bytes fields, struct messages, all lists of a level)."""
    n = len(vals)
    size = _hash_size(t)
    if n == 0:
        return np.zeros((0, size), dtype=np.uint8)
    if isinstance(t, Hashable):
        return np.frombuffer(b"".join(memo[id(v)] for v in vals), dtype=np.uint8).reshape(n, 32)
    if isinstance(t, (Bool, Uint)):
        return _scalar_bytes(t, vals)
    if isinstance(t, (Bytes, ByteArray)):
        return _hash_bytes_values(vals)
    if isinstance(t, Ptr):
        return _hash_many(t.elem, vals, memo)
    if isinstance(t, Struct):
        cols = [_hash_many(ft, _column(vals, name), memo) for name, ft in t.hashed_fields()]
        if not cols:  # Keccak of the empty concatenation
            return np.frombuffer(b"".join(hash_batch_var([b""] * n)), dtype=np.uint8).reshape(n, 32)
        return hash_batch(np.ascontiguousarray(np.concatenate(cols, axis=1)), sum(c.shape[1] for c in cols))
    if isinstance(t, (Slice, Array)):
        # one list of equal-length byte strings: element digests and the tree
        # in one library call (mk_ssz_tree_hash_bytes_list)
        if n == 1 and isinstance(t.elem, (Bytes, ByteArray)) and len(vals[0]):
            bs = [bytes(e) for e in vals[0]]
            if all(len(b) == len(bs[0]) for b in bs):
                flat = np.frombuffer(b"".join(bs), dtype=np.uint8) if len(bs[0]) else np.zeros(0, np.uint8)
                return np.frombuffer(tree_hash_bytes_list(flat, len(bs), len(bs[0])), dtype=np.uint8).reshape(1, 32)
        # every list of this nesting level in one library call (mk_ssz_merkle_many)
        if isinstance(t.elem, (Bool, Uint)):
            encs = [_scalar_bytes(t.elem, v) for v in vals]
            roots = merkle_many([e.reshape(-1) for e in encs], [len(e) for e in encs], _hash_size(t.elem))
        else:
            lens = [len(v) for v in vals]
            flat = [e for v in vals for e in v]
            hs = _hash_many(t.elem, flat, memo)  # the inner lists are consecutive rows
            size = _hash_size(t.elem)
            offs = np.cumsum([0] + lens[:-1], dtype=np.uint64) * np.uint64(size)
            return merkle_many_flat(hs, offs, lens, size)
        return np.frombuffer(b"".join(roots), dtype=np.uint8).reshape(n, 32)
    raise HashError(f"type {t.go_name} is not hashable")


# ----------------------------------------------------------------- public API
def merkle_hash_flat(items: np.ndarray, n: int, item_len: int) -> bytes:
    """merkleHash over n contiguous items of item_len bytes (one GPU call)."""
    a = np.ascontiguousarray(items, dtype=np.uint8).reshape(-1)
    if a.size < n * item_len:
        raise ValueError("items buffer shorter than n*item_len")
    if n and item_len == 0:
        raise ZeroDivisionError("integer divide by zero")  # hash.go:207 panics
    out = ctypes.create_string_buffer(32)
    _lib.invoke("mk_ssz_merkle_hash", _ptr(a) if a.size else None, n, item_len, out)
    return out.raw


def tree_hash_bytes_list(elems: np.ndarray, n: int, elem_len: int) -> bytes:
    """ssz.TreeHash of a slice of n byte strings of elem_len bytes each,
    contiguous in ``elems`` (makeSliceHasher + hashedEncoding, hash.go:100-107,
    118-139): merkleHash over Keccak(le32(elem_len) || element), one GPU call
    (mk_ssz_tree_hash_bytes_list)."""
    a = np.ascontiguousarray(elems, dtype=np.uint8).reshape(-1)
    if a.size < n * elem_len:
        raise ValueError("elements buffer shorter than n*elem_len")
    out = ctypes.create_string_buffer(32)
    _lib.invoke("mk_ssz_tree_hash_bytes_list", _ptr(a) if a.size else None, n, elem_len, out)
    return out.raw


def merkle_many(lists: Sequence[np.ndarray], ns: Sequence[int], item_len: int) -> List[bytes]:
    """merkleHash of every list (lists[i]: ns[i] items of item_len bytes) in
    one library call: all lists' windows in one launch, one launch per level."""
    k = len(lists)
    if k == 0:
        return []
    if item_len == 0 and any(ns):
        raise ZeroDivisionError("integer divide by zero")
    offs = np.zeros(k, dtype=np.uint64)
    parts, pos = [], 0
    for i, a in enumerate(lists):
        pad = (-pos) % 16  # 16-B aligned lists take the streaming window path
        if pad:
            parts.append(np.zeros(pad, np.uint8))
            pos += pad
        offs[i] = pos
        parts.append(np.ascontiguousarray(a, dtype=np.uint8).reshape(-1))
        pos += parts[-1].size
    buf = np.concatenate(parts) if pos else np.zeros(16, np.uint8)
    return [bytes(r) for r in merkle_many_flat(buf, offs, ns, item_len)]


def merkle_many_flat(buf: np.ndarray, offs, ns, item_len: int) -> np.ndarray:
    """merkleHash of list i = ns[i] items of item_len bytes at byte offset
    offs[i] of ``buf`` (one mk_ssz_merkle_many call): (k, 32) roots."""
    k = len(ns)
    if item_len == 0 and any(ns):
        raise ZeroDivisionError("integer divide by zero")
    buf = np.ascontiguousarray(buf, dtype=np.uint8).reshape(-1)
    if buf.size == 0:
        buf = np.zeros(16, np.uint8)
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    n = np.ascontiguousarray(ns, dtype=np.uint64)
    il = np.full(k, max(item_len, 1), dtype=np.uint32)
    out = np.empty((k, 32), dtype=np.uint8)
    if k:
        _lib.invoke("mk_ssz_merkle_many", _ptr(buf), _ptr(o), _ptr(n), _ptr(il), k, _ptr(out))
    return out


def merkle_hash(lst: Sequence[bytes]) -> bytes:
    """ssz.merkleHash (hash.go:194-239) over a list of byte strings.  Lists
    whose items all have len(list[0]) bytes (every list TreeHash builds) go
    to the GPU as one flat buffer."""
    n = len(lst)
    if n == 0:
        return merkle_hash_flat(np.zeros(0, np.uint8), 0, 1)
    L0 = len(lst[0])
    if L0 == 0:
        raise ZeroDivisionError("integer divide by zero")
    if all(len(x) == L0 for x in lst):
        return merkle_hash_flat(np.frombuffer(b"".join(bytes(x) for x in lst), dtype=np.uint8), n, L0)
    return _merkle_hash_ragged(lst)


def _merkle_hash_ragged(lst: Sequence[bytes]) -> bytes:
    """Items of different lengths (only Encodable elements of variable size
    produce this): level 0 chunks per hash.go:205-220, each level one batched
    GPU launch of variable-length messages."""
    zero = bytes(SSZ_CHUNK_SIZE)
    p = SSZ_CHUNK_SIZE // len(lst[0]) if len(lst[0]) < SSZ_CHUNK_SIZE else 1
    chunks = [b"".join(bytes(x) for x in lst[i:i + p]) for i in range(0, len(lst), p)]
    while len(chunks) > 1:
        if len(chunks) % 2:
            chunks.append(zero)
        chunks = hash_batch_var([chunks[i] + chunks[i + 1] for i in range(0, len(chunks), 2)])
    lenc = _st.pack("<Q", len(lst)) + bytes(24)
    return hash_batch_var([chunks[0] + lenc])[0]


def tree_hash(val: Any, typ: Optional[SSZType]) -> bytes:
    """ssz.TreeHash (hash.go:23-39): 32-byte tree hash of ``val`` of Go type
    ``typ`` (None models a nil interface).  Raises HashError with the
    reference's text."""
    if typ is None:
        raise HashError("hash error: nil is not supported for input type <nil>")
    e = _check_serializable(typ)
    if e is not None:
        raise HashError(f"hash error: {e} for input type {typ.go_name}")
    memo: dict = {}
    try:
        _validate(typ, val, memo)
    except HashError as err:
        raise HashError(f"hash error: {err} for input type {typ.go_name}")
    out = bytes(_hash_many(typ, [val], memo)[0])
    return (out + bytes(32))[:32]  # bytesutil.ToBytes32
