"""Host mirror of ``shared/hashutil`` over the HIP engine.

Reference: shared/hashutil/hash.go:11-25 (``Hash``), merkleRoot.go:12-30
(``MerkleRoot``).  Same names, argument meaning and return values; the
batched entry points are the new API the north star asks for (the reference
has no batch form).  Every digest is computed on the GPU; there is no CPU
fallback.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, List, Sequence

import numpy as np

from . import _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p) if a.size else None


def _flatten(msgs: Sequence[bytes]):
    msgs = [bytes(m) for m in msgs]
    offs = np.zeros(len(msgs) + 1, dtype=np.uint64)
    if msgs:
        offs[1:] = np.cumsum([len(m) for m in msgs], dtype=np.uint64)
    data = np.frombuffer(b"".join(msgs), dtype=np.uint8) if offs[-1] else np.zeros(1, np.uint8)
    return np.ascontiguousarray(data), offs


def Hash(data: bytes) -> bytes:
    """hashutil.Hash: legacy Keccak-256 of ``data`` (hash.go:11)."""
    data = bytes(data)
    out = ctypes.create_string_buffer(32)
    buf = ctypes.create_string_buffer(data, max(1, len(data)))
    _lib.invoke("mk_hash", buf, len(data), out)
    return out.raw


def hash_batch(msgs: np.ndarray, msg_len: int) -> np.ndarray:
    """Batched Hash of n fixed-length messages.  ``msgs``: uint8 array of
    n*msg_len bytes (any shape).  Returns (n, 32) uint8."""
    a = np.ascontiguousarray(msgs, dtype=np.uint8).reshape(-1)
    if msg_len == 0:
        raise ValueError("msg_len must be > 0 (use hash_batch_var for empty messages)")
    n = a.size // msg_len
    out = np.empty((n, 32), dtype=np.uint8)
    _lib.invoke("mk_hash_batch", _ptr(a), n, msg_len, _ptr(out))
    return out


def hash_batch_var(msgs: Sequence[bytes]) -> List[bytes]:
    """Batched Hash of variable-length messages, in order."""
    if not msgs:
        return []
    data, offs = _flatten(msgs)
    out = np.empty((len(msgs), 32), dtype=np.uint8)
    _lib.invoke("mk_hash_batch_var", _ptr(data), _ptr(offs), len(msgs), _ptr(out))
    return [bytes(r) for r in out]


def MerkleRoot(values: List[bytes]) -> bytes:
    """hashutil.MerkleRoot (merkleRoot.go:12-30), including its side effect:
    ``values[i]`` is replaced by ``Hash(values[i])`` (merkleRoot.go:16-19).

    One library call (``mk_merkle_root``): the leaves are hashed into the
    upper half of the heap o[1..2n), the partial top heap band is one
    pairwise level and the rest a power-of-two binary tree on the device.
    Like the reference, an empty list is an index-out-of-range panic
    (IndexError here)."""
    n = len(values)
    if n == 0:
        raise IndexError("index out of range [1] with length 0")
    data, offs = _flatten(values)
    leaves = np.empty((n, 32), dtype=np.uint8)
    out = ctypes.create_string_buffer(32)
    _lib.invoke("mk_merkle_root", _ptr(data), _ptr(offs), n, _ptr(leaves), out)
    for i in range(n):
        values[i] = bytes(leaves[i])
    return out.raw
