"""ctypes binding of libprysm_merkle.so (include/prysm_merkle.h).

This is the Python-side twin of the cgo binding a Go maintainer would add
(INTEGRATION.md).  The library is built in-tree (``prysm_amd/lib/``) by
``__graft_entry__.build()`` / ``make -C prysm_amd/csrc``.  There is no CPU
fallback anywhere in the product path: if the library is missing, or no
gfx950 device is visible, calls raise ``MerkleError`` loudly.
"""
from __future__ import annotations

import ctypes
import os
import re

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libprysm_merkle.so")
HEADER = os.path.join(os.path.dirname(HERE), "include", "prysm_merkle.h")

MK_OK = 0
MK_EINVAL = -22
MK_ENODEV = -19
MK_ENOMEM = -12
MK_EHIP = -5
MK_ECOMM = -71


class MerkleError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{msg} (code {code})")
        self.code = code


_c = ctypes
_vp = _c.c_void_p
_u64, _u32, _int = _c.c_uint64, _c.c_uint32, _c.c_int


class Call(ctypes.Structure):
    """mk_call: per-call device selection and error detail (include/prysm_merkle.h)."""
    _fields_ = [("device", ctypes.c_int32), ("code", ctypes.c_int32), ("err", ctypes.c_char * 256)]


_cp = _c.POINTER(Call)

# name -> (restype, argtypes); entry points taking a per-call context list it first
_SIGS = {
    "mk_init": (_int, [_int]),
    "mk_device_count": (_int, []),
    "mk_strerror": (_c.c_char_p, [_int]),
    "mk_last_error": (_c.c_char_p, []),
    "mk_version": (_c.c_char_p, []),
    "mk_hash": (_int, [_cp, _vp, _u64, _vp]),
    "mk_hash_batch": (_int, [_cp, _vp, _u64, _u32, _vp]),
    "mk_hash_batch_var": (_int, [_cp, _vp, _vp, _u64, _vp]),
    "mk_dev_hash_batch": (_int, [_cp, _vp, _u64, _u32, _vp, _vp]),
    "mk_dev_hash_batch_var": (_int, [_cp, _vp, _vp, _u64, _vp, _vp]),
    "mk_ssz_merkle_hash": (_int, [_cp, _vp, _u64, _u32, _vp]),
    "mk_ssz_merkle_workspace_bytes": (_u64, [_u64, _u32]),
    "mk_dev_ssz_merkle_hash": (_int, [_cp, _vp, _u64, _u32, _vp, _vp, _u64, _vp]),
    "mk_ssz_tree_hash_bytes_list_workspace_bytes": (_u64, [_u64, _u32]),
    "mk_dev_ssz_tree_hash_bytes_list": (_int, [_cp, _vp, _u64, _u32, _vp, _vp, _u64, _vp]),
    "mk_ssz_tree_hash_bytes_list": (_int, [_cp, _vp, _u64, _u32, _vp]),
    "mk_ssz_merkle_many_workspace_bytes": (_u64, [_vp, _vp, _u32]),
    "mk_dev_ssz_merkle_many": (_int, [_cp, _vp, _vp, _vp, _vp, _u32, _vp, _vp, _u64, _vp]),
    "mk_ssz_merkle_many": (_int, [_cp, _vp, _vp, _vp, _vp, _u32, _vp]),
    "mk_ssz_merkle_shard_plan": (_int, [_cp, _u64, _u32, _u32, _vp, _vp, _vp]),
    "mk_dev_ssz_merkle_subtree": (_int, [_cp, _vp, _u64, _u32, _u32, _int, _vp, _vp, _u64, _vp]),
    "mk_dev_ssz_merkle_finish": (_int, [_cp, _vp, _u64, _u64, _vp, _vp]),
    "mk_dev_ssz_merkle_subtree_frontier": (_int, [_cp, _vp, _u64, _u32, _u32, _u32, _int, _vp, _vp, _vp, _u64,
                                                  _vp]),
    "mk_ssz_merkle_node_frontier_workspace_bytes": (_u64, [_u64, _u32, _u32]),
    "mk_dev_ssz_merkle_node_frontier": (_int, [_cp, _vp, _u64, _u32, _u32, _int, _vp, _vp, _vp, _u64, _vp]),
    "mk_ssz_merkle_finish_workspace_bytes": (_u64, [_u64]),
    "mk_dev_ssz_merkle_finish_nodes": (_int, [_cp, _vp, _u64, _u64, _vp, _vp, _u64, _vp]),
    "mk_dev_ssz_merkle_finish_nodes_pair": (_int, [_cp, _vp, _u64, _u64, _vp, _u32, _u32, _vp, _u64, _vp]),
    "mk_ssz_merkle_top_fused_workspace_bytes": (_u64, [_u64, _u64]),
    "mk_dev_ssz_merkle_top_fused": (_int, [_cp, _vp, _u64, _u64, _vp, _u64, _u64, _vp, _u32, _vp, _u64, _vp]),
    "mk_ssz_merkle_hash_multi": (_int, [_cp, _vp, _u64, _u32, _int, _vp, _vp]),
    "mk_dev_ssz_merkle_hash_multi": (_int, [_cp, _vp, _u64, _u32, _int, _vp, _vp]),
    "mk_ssz_struct_msg_len": (_u64, [_vp, _u32]),
    "mk_ssz_struct_roots": (_int, [_cp, _vp, _u64, _u32, _vp, _u32, _vp]),
    "mk_ssz_struct_list_workspace_bytes": (_u64, [_u64, _vp, _u32]),
    "mk_dev_ssz_struct_list_root": (_int, [_cp, _vp, _u64, _u32, _vp, _u32, _vp, _vp, _u64, _vp]),
    "mk_dev_ssz_struct_roots": (_int, [_cp, _vp, _u64, _u32, _vp, _u32, _vp, _vp, _u64, _vp]),
    "mk_ssz_struct_list_level1_ok": (_int, [_vp, _u64, _u32, _vp, _u32]),
    "mk_dev_ssz_struct_list_level1": (_int, [_cp, _vp, _u64, _u32, _vp, _u32, _vp, _vp, _vp, _u64, _u32, _vp, _vp]),
    "mk_ssz_struct_pipe_ok": (_int, [_vp, _u64, _u32, _vp, _u32, _vp]),
    "mk_ssz_struct_pipe_levels_bytes": (_u64, [_u64, _u64, _u32, _u32]),
    "mk_ssz_struct_pipe_top_workspace_bytes": (_u64, [_u64, _u64, _u32, _u32]),
    "mk_dev_ssz_struct_list_level1_pipe": (_int, [_cp, _vp, _u64, _u32, _vp, _u32, _vp, _vp, _vp, _u64, _u32, _vp,
                                                  _vp, _vp, _vp, _vp, _vp]),
    "mk_dev_ssz_struct_pipe_top": (_int, [_cp, _vp, _u64, _u64, _u32, _u32, _vp, _vp, _u32, _u32, _vp, _u64, _vp]),
    "mk_ssz_struct_list_root": (_int, [_cp, _vp, _u64, _u32, _vp, _u32, _vp]),
    "mk_merkle_root": (_int, [_cp, _vp, _vp, _u64, _vp, _vp]),
    "mk_merkle_root_workspace_bytes": (_u64, [_u64]),
    "mk_dev_merkle_root": (_int, [_cp, _vp, _vp, _u64, _u32, _vp, _u64, _vp, _vp, _vp]),
    "mk_deposit_trie_levels_bytes": (_u64, [_u64, _u32]),
    "mk_deposit_trie_build": (_int, [_cp, _vp, _vp, _u64, _u32, _vp, _vp]),
    "mk_dev_deposit_trie_append": (_int, [_cp, _vp, _u64, _u64, _vp, _vp, _u64, _u32, _u32, _vp, _vp]),
    "mk_dev_deposit_trie_branch": (_int, [_cp, _vp, _u64, _u64, _u32, _u64, _vp, _vp]),
    "mk_deposit_trie_pipe_ok": (_int, [_vp, _u64, _u32, _u32, _vp]),
    "mk_dev_deposit_trie_build_pipe": (_int, [_cp, _vp, _vp, _u64, _vp, _u64, _u32, _u32, _vp]),
    "mk_dev_deposit_trie_pipe_top": (_int, [_cp, _vp, _u64, _u64, _u32, _vp, _vp]),
    "mk_dev_deposit_trie_levels": (_int, [_cp, _vp, _u64, _u64, _u32, _u32, _u32, _vp, _vp]),
    "mk_dev_deposit_trie_build": (_int, [_cp, _vp, _u64, _vp, _vp, _u64, _u32, _u32, _u32, _vp, _vp]),
    "mk_deposit_trie_new": (_int, [_cp, _u32, _u64, _vp]),
    "mk_deposit_trie_free": (None, [_vp]),
    "mk_deposit_trie_count": (_u64, [_vp]),
    "mk_deposit_trie_append": (_int, [_cp, _vp, _vp, _vp, _u64]),
    "mk_deposit_trie_save_logs": (_int, [_cp, _vp, _vp, _vp, _u64, _vp, _vp]),
    "mk_deposit_trie_root": (_int, [_cp, _vp, _vp]),
    "mk_deposit_trie_branch": (_int, [_cp, _vp, _u64, _vp]),
    "mk_deposit_trie_leaves": (_int, [_cp, _vp, _u64, _u64, _vp]),
    "mk_verify_merkle_branches": (_int, [_cp, _vp, _vp, _vp, _u64, _u32, _u32, _vp, _vp]),
    "mk_dev_synth_fill": (_int, [_cp, _vp, _u64, _u64, _u64, _vp]),
    "mk_prof_enable": (_int, [_int]),
    "mk_prof_read": (_int, [_cp, _vp, _vp, _vp, _vp]),
}

MK_FIELD_BYTES = 1
MK_FIELD_RAW = 2


class Field(ctypes.Structure):
    """mk_field: one field of a flat fixed-layout record."""
    _fields_ = [("kind", ctypes.c_uint32), ("offset", ctypes.c_uint32), ("len", ctypes.c_uint32)]


_lib = None


def header_symbols():
    """Every mk_* function declared in include/prysm_merkle.h."""
    with open(HEADER) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|uint64_t|void|const char\*)\s+(mk_[a-z0-9_]+)\s*\(", txt, re.M)))


def load():
    """Load the HIP library (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    # PRYSM_MERKLE_LIB: another build of the same library (A/B tooling, e.g.
    # prysm_amd/lib/variants/); never a different implementation
    path = os.environ.get("PRYSM_MERKLE_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise MerkleError(MK_ENODEV, f"{path} missing: run __graft_entry__.build() "
                                     "(no CPU fallback exists)")
    L = ctypes.CDLL(path)
    for name, (res, args) in _SIGS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int, what: str = "", call: "Call" = None) -> None:
    """Raise MerkleError for a failed call; the detail comes from the call's
    own context (never from another call on this thread)."""
    if rc != MK_OK:
        L = load()
        detail = call.err.decode(errors="replace") if call is not None else L.mk_last_error().decode(errors="replace")
        raise MerkleError(rc, f"{what}: {L.mk_strerror(rc).decode()}: {detail}")


def invoke(name: str, *args, device: int = -1) -> None:
    """Call entry point `name` with a fresh per-call context (device: -1 =
    the stream's / thread's current device) and raise on failure."""
    call = Call(device, 0, b"")
    rc = getattr(load(), name)(ctypes.byref(call), *args)
    check(rc, name, call)


def device_count() -> int:
    return load().mk_device_count()


def init(device: int = 0) -> None:
    check(load().mk_init(device), "mk_init")
