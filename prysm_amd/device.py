"""Device-resident entry points (inputs already in HBM), torch as plumbing.

torch provides device memory, the current HIP stream and torch.distributed;
every hash is computed by the HIP kernels behind the C-ABI
(``mk_dev_*`` in include/prysm_merkle.h).  Work is enqueued on torch's
current stream of the tensor's device and is not synchronised here.  Every
call passes its device in its own ``mk_call`` context (``_lib.invoke``).
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib


def _stream(dev: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _p(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def _np(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _dev(t: torch.Tensor) -> int:
    """Device index of a GPU tensor (passed in every call's context)."""
    if t.device.type != "cuda":
        raise _lib.MerkleError(_lib.MK_EINVAL, "device entry points need a GPU tensor")
    return t.device.index if t.device.index is not None else torch.cuda.current_device()


def synth_fill(dst: torch.Tensor, seed: int, word0: int = 0) -> torch.Tensor:
    """Fill ``dst`` (uint8, nbytes % 8 == 0) with bytes [8*word0, ...) of the
    SplitMix64 stream."""
    _lib.invoke("mk_dev_synth_fill", _p(dst), dst.numel() * dst.element_size(), seed, word0, _stream(dst.device),
                device=_dev(dst))
    return dst


def struct_roots(records: torch.Tensor, n: int, record_len: int, spec, out: torch.Tensor = None,
                 ws: torch.Tensor = None) -> torch.Tensor:
    """Struct root of each of n records (makeStructHasher per element,
    shared/ssz/hash.go:141-159; ``spec`` = [(kind, offset, len)] as in
    registry.VALIDATOR_FIELDS).  Returns an (n*32,) uint8 device tensor."""
    from .registry import _fields

    dev = _dev(records)
    if records.numel() < n * record_len:
        raise ValueError("records tensor shorter than n*record_len")
    f = _fields(spec)
    L = _lib.load()
    if out is None:
        out = torch.empty(max(32, 32 * n), dtype=torch.uint8, device=records.device)
    if ws is None:
        ws = torch.empty(max(256, n * L.mk_ssz_struct_msg_len(f, len(spec))), dtype=torch.uint8,
                         device=records.device)
    _lib.invoke("mk_dev_ssz_struct_roots", _p(records), n, record_len, f, len(spec), _p(out), _p(ws), ws.numel(),
                _stream(records.device), device=dev)
    return out


def struct_list_root(records: torch.Tensor, n: int, record_len: int, spec, out: torch.Tensor = None,
                     ws: torch.Tensor = None) -> torch.Tensor:
    """TreeHash of a list of n flat records (struct roots + merkleHash)."""
    from .registry import _fields

    dev = _dev(records)
    f = _fields(spec)
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=records.device)
    if ws is None:
        ws = torch.empty(_lib.load().mk_ssz_struct_list_workspace_bytes(n, f, len(spec)) + 256, dtype=torch.uint8,
                         device=records.device)
    _lib.invoke("mk_dev_ssz_struct_list_root", _p(records), n, record_len, f, len(spec), _p(out), _p(ws), ws.numel(),
                _stream(records.device), device=dev)
    return out


def struct_list_level1_ok(records: torch.Tensor, n: int, record_len: int, spec) -> bool:
    """Whether struct_list_level1 takes these records (the ValidatorRecord
    layout at a 16-B aligned address, n >= 2^18)."""
    from .registry import _fields

    return bool(_lib.load().mk_ssz_struct_list_level1_ok(_p(records), n, record_len, _fields(spec), len(spec)))


def struct_list_level1(records: torch.Tensor, n: int, record_len: int, spec, roots: torch.Tensor,
                       nodes: torch.Tensor, values: torch.Tensor = None, nvalues: int = 0, value_len: int = 8,
                       value_nodes: torch.Tensor = None) -> torch.Tensor:
    """The list root's first tree level in the struct-roots launch: the n
    struct roots into ``roots`` and the ceil(n/8) level-1 nodes of their
    merkleHash into ``nodes`` (finish with merkle_finish_nodes(nodes,
    ceil(n/8), n)); with ``values`` also the ceil(nvalues * value_len / 256)
    level-1 nodes of a second list's merkleHash into ``value_nodes``."""
    from .registry import _fields

    if roots.numel() < 32 * n or nodes.numel() < 32 * -(-n // 8):
        raise ValueError("roots / nodes buffers too small")
    if nvalues and (values is None or value_nodes is None or
                    value_nodes.numel() < 32 * -(-nvalues * value_len // 256)):
        raise ValueError("second list: values / value_nodes missing or too small")
    _lib.invoke("mk_dev_ssz_struct_list_level1", _p(records), n, record_len, _fields(spec), len(spec), _p(roots),
                _p(nodes), _p(values) if nvalues else None, nvalues, value_len,
                _p(value_nodes) if nvalues else None, _stream(records.device), device=_dev(records))
    return nodes


def struct_pipe_ok(records: torch.Tensor, n: int, record_len: int, spec) -> bool:
    """Whether struct_list_level1_pipe takes these records on the current
    stream (struct_list_level1_ok with 4 groups of 1024 per workgroup)."""
    from .registry import _fields

    return bool(_lib.load().mk_ssz_struct_pipe_ok(_p(records), n, record_len, _fields(spec), len(spec),
                                                  _stream(records.device)))


def struct_pipe_levels_bytes(n: int, nvalues: int = 0, value_len: int = 8, which: int = 0) -> int:
    """Bytes of one tree's slot-levels buffer (which 0: the registry of n
    records, 1: the second list of nvalues x value_len)."""
    return int(_lib.load().mk_ssz_struct_pipe_levels_bytes(n, nvalues, value_len, which))


def struct_pipe_top_workspace(n: int, device, nvalues: int = 0, value_len: int = 8, which: int = 0) -> torch.Tensor:
    nb = int(_lib.load().mk_ssz_struct_pipe_top_workspace_bytes(n, nvalues, value_len, which))
    return torch.empty(max(256, nb), dtype=torch.uint8, device=device)


def struct_list_level1_pipe(records: torch.Tensor, n: int, record_len: int, spec, roots: torch.Tensor,
                            nodes: torch.Tensor, prev_nodes, prev_levels, values: torch.Tensor = None,
                            nvalues: int = 0, value_len: int = 8, value_nodes: torch.Tensor = None,
                            prev_value_nodes=None, prev_value_levels=None) -> torch.Tensor:
    """struct_list_level1, and in the same launch levels 2..10 of the
    PREVIOUS state's registry tree (its level-1 ``prev_nodes``; None for the
    first state) into ``prev_levels`` and levels 2..4 of its second list's
    tree (``prev_value_nodes``) into ``prev_value_levels``."""
    from .registry import _fields

    if roots.numel() < 32 * n or nodes.numel() < 32 * -(-n // 8):
        raise ValueError("roots / nodes buffers too small")
    if prev_nodes is not None and (prev_nodes.numel() < 32 * -(-n // 8) or prev_levels is None or
                                   prev_levels.numel() < struct_pipe_levels_bytes(n)):
        raise ValueError("previous state's nodes / levels buffers too small")
    if nvalues and (values is None or value_nodes is None or
                    value_nodes.numel() < 32 * -(-nvalues * value_len // 256)):
        raise ValueError("second list: values / value_nodes missing or too small")
    if prev_value_nodes is not None and (
            prev_value_levels is None or
            prev_value_levels.numel() < struct_pipe_levels_bytes(n, nvalues, value_len, 1)):
        raise ValueError("previous state's second-list levels buffer too small")
    vp = lambda t: _p(t) if t is not None else None  # noqa: E731
    _lib.invoke("mk_dev_ssz_struct_list_level1_pipe", _p(records), n, record_len, _fields(spec), len(spec),
                _p(roots), _p(nodes), vp(values) if nvalues else None, nvalues, value_len,
                vp(value_nodes) if nvalues else None, vp(prev_nodes), vp(prev_levels) if prev_nodes is not None else None,
                vp(prev_value_nodes), vp(prev_value_levels) if prev_value_nodes is not None else None,
                _stream(records.device), device=_dev(records))
    return nodes


def struct_pipe_top(nodes: torch.Tensor, n: int, levels: torch.Tensor, pair_block: torch.Tensor, slot: int,
                    epoch: int, ws: torch.Tensor, nvalues: int = 0, value_len: int = 8, which: int = 0) -> None:
    """One tree's root of a state whose slot levels the next pipelined launch
    built (which 0: the registry, 1: the second list), into slot ``slot`` of a
    pair block (merkle_finish_nodes_pair semantics)."""
    if pair_block.numel() < 128:
        raise ValueError("pair block of 128 bytes")
    _lib.invoke("mk_dev_ssz_struct_pipe_top", _p(nodes), n, nvalues, value_len, which, _p(levels), _p(pair_block),
                slot, epoch, _p(ws), ws.numel(), _stream(nodes.device), device=_dev(nodes))


def merkle_workspace(n: int, item_len: int, device) -> torch.Tensor:
    nbytes = _lib.load().mk_ssz_merkle_workspace_bytes(n, item_len)
    return torch.empty(max(256, nbytes), dtype=torch.uint8, device=device)


def merkle_hash(items: torch.Tensor, n: int, item_len: int, out: torch.Tensor = None,
                ws: torch.Tensor = None) -> torch.Tensor:
    """ssz.merkleHash of n items of item_len bytes held in ``items`` (uint8,
    device).  Returns a (32,) uint8 device tensor."""
    dev = _dev(items)
    if items.numel() < n * item_len:
        raise ValueError("items tensor shorter than n*item_len")
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=items.device)
    if ws is None:
        ws = merkle_workspace(n, item_len, items.device)
    _lib.invoke("mk_dev_ssz_merkle_hash", _p(items), n, item_len, _p(out), _p(ws), ws.numel(), _stream(items.device),
                device=dev)
    return out


def tree_hash_bytes_list_workspace(n: int, elem_len: int, device, aligned16: bool = True) -> torch.Tensor:
    """Workspace of mk_dev_ssz_tree_hash_bytes_list.  The library's query
    plans for 16-B aligned elements; elements at another address take the
    two-phase form (element digests in the workspace first), which needs
    n x 32 more bytes (rounded to 256)."""
    nb = _lib.load().mk_ssz_tree_hash_bytes_list_workspace_bytes(n, elem_len)
    if not aligned16:
        nb += -(-n * 32 // 256) * 256
    return torch.empty(max(nb, 256), dtype=torch.uint8, device=device)


def tree_hash_bytes_list(elems: torch.Tensor, n: int, elem_len: int, out: torch.Tensor = None,
                         ws: torch.Tensor = None) -> torch.Tensor:
    """ssz.TreeHash of a list of n byte strings of elem_len bytes each
    (makeSliceHasher + hashedEncoding, shared/ssz/hash.go:100-107, 118-139):
    merkleHash over K(le32(elem_len) || element_i), in one call with the
    element digests fused into the leaf pass (32-B elements)."""
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=elems.device)
    if ws is None:
        ws = tree_hash_bytes_list_workspace(n, elem_len, elems.device, aligned16=elems.data_ptr() % 16 == 0)
    _lib.invoke("mk_dev_ssz_tree_hash_bytes_list", _p(elems), n, elem_len, _p(out), _p(ws), ws.numel(),
                _stream(elems.device), device=_dev(elems))
    return out


def merkle_many(items: torch.Tensor, offs, ns, item_lens, out: torch.Tensor = None,
                ws: torch.Tensor = None) -> torch.Tensor:
    """merkleHash of many lists in one call (list i = ns[i] items of
    item_lens[i] bytes at byte offset offs[i] of ``items``): an (nlists*32,)
    uint8 device tensor of roots."""
    dev = _dev(items)
    k = len(ns)
    o = np.ascontiguousarray(offs, dtype=np.uint64)
    n = np.ascontiguousarray(ns, dtype=np.uint64)
    il = np.ascontiguousarray(item_lens, dtype=np.uint32)
    if out is None:
        out = torch.empty(max(32, 32 * k), dtype=torch.uint8, device=items.device)
    if ws is None:
        ws = torch.empty(max(256, many_workspace_bytes(n, il)), dtype=torch.uint8, device=items.device)
    _lib.invoke("mk_dev_ssz_merkle_many", _p(items), _np(o), _np(n), _np(il), k, _p(out), _p(ws), ws.numel(),
                _stream(items.device), device=dev)
    return out[:32 * k]


def many_workspace_bytes(ns, item_lens) -> int:
    n = np.ascontiguousarray(ns, dtype=np.uint64)
    il = np.ascontiguousarray(item_lens, dtype=np.uint32)
    return _lib.load().mk_ssz_merkle_many_workspace_bytes(_np(n), _np(il), len(n))


def shard_plan(n: int, item_len: int, nshards: int):
    """(height, nonempty, item_begin[nshards+1]) of the subtree sharding."""
    h = ctypes.c_uint32()
    ne = ctypes.c_uint32()
    begin = (ctypes.c_uint64 * (nshards + 1))()
    _lib.invoke("mk_ssz_merkle_shard_plan", n, item_len, nshards, ctypes.byref(h), ctypes.byref(ne), begin)
    return h.value, ne.value, list(begin)


def subtree_workspace(shard_n: int, item_len: int, device) -> torch.Tensor:
    # the full-tree plan of the same item count bounds the subtree plan
    nbytes = _lib.load().mk_ssz_merkle_workspace_bytes(max(shard_n, 1), item_len) + 4096
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def merkle_subtree(items: torch.Tensor, shard_n: int, item_len: int, height: int, pad_at_one: bool,
                   out: torch.Tensor = None, ws: torch.Tensor = None) -> torch.Tensor:
    """32-B root of one shard at `height` levels above its chunks."""
    dev = _dev(items)
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=items.device)
    if ws is None:
        ws = subtree_workspace(shard_n, item_len, items.device)
    _lib.invoke("mk_dev_ssz_merkle_subtree", _p(items), shard_n, item_len, height, int(pad_at_one), _p(out), _p(ws),
                ws.numel(), _stream(items.device), device=dev)
    return out


def merkle_subtree_frontier(items: torch.Tensor, shard_n: int, item_len: int, height: int, frontier_log2: int,
                            pad_at_one: bool, out: torch.Tensor = None, ws: torch.Tensor = None) -> torch.Tensor:
    """The shard's tree level `frontier_log2` levels below its root: a
    (nodes*32,) uint8 device tensor (nodes = parallel.frontier_count(...))."""
    from .parallel import frontier_count

    dev = _dev(items)
    nodes = frontier_count(shard_n, item_len, height, frontier_log2)
    if out is None:
        out = torch.empty(32 << frontier_log2, dtype=torch.uint8, device=items.device)
    if out.numel() < 32 * nodes:
        raise ValueError("frontier output buffer too small")
    if ws is None:
        ws = subtree_workspace(shard_n, item_len, items.device)
    got = ctypes.c_uint64()
    _lib.invoke("mk_dev_ssz_merkle_subtree_frontier", _p(items), shard_n, item_len, height, frontier_log2,
                int(pad_at_one), _p(out), ctypes.byref(got), _p(ws), ws.numel(), _stream(items.device), device=dev)
    assert got.value == nodes, (got.value, nodes)
    return out[:32 * nodes]


def merkle_node_frontier(nodes: torch.Tensor, count: int, height: int, frontier_log2: int, pad_at_one: bool,
                         out: torch.Tensor = None, ws: torch.Tensor = None) -> torch.Tensor:
    """A subtree continued from one of its node levels: `count` 32-B nodes
    reduced `height` levels (odd rule, hash.go:225-235), stopping
    `frontier_log2` levels below the top; returns the (nodes*32,) level."""
    dev = _dev(nodes)
    lib = _lib.load()
    want = max(1, -(-count // (1 << (height - frontier_log2)))) if frontier_log2 else 1
    if out is None:
        out = torch.empty(32 << frontier_log2, dtype=torch.uint8, device=nodes.device)
    if out.numel() < 32 * want:
        raise ValueError("node frontier output buffer too small")
    if ws is None:
        ws = torch.empty(max(256, lib.mk_ssz_merkle_node_frontier_workspace_bytes(count, height, frontier_log2)),
                         dtype=torch.uint8, device=nodes.device)
    got = ctypes.c_uint64()
    _lib.invoke("mk_dev_ssz_merkle_node_frontier", _p(nodes), count, height, frontier_log2, int(pad_at_one), _p(out),
                ctypes.byref(got), _p(ws), ws.numel(), _stream(nodes.device), device=dev)
    assert got.value == want, (got.value, want)
    return out[:32 * want]


def finish_workspace(count: int, device) -> torch.Tensor:
    return torch.empty(max(256, _lib.load().mk_ssz_merkle_finish_workspace_bytes(count)), dtype=torch.uint8,
                       device=device)


def merkle_finish_nodes_pair(nodes: torch.Tensor, count: int, n_total: int, pair_block: torch.Tensor, slot: int,
                             epoch: int, ws: torch.Tensor = None) -> None:
    """merkle_finish_nodes for one list field of a two-field struct: the list
    root goes to pair_block[32 slot:32 slot + 32]; whichever of the pair's two
    finishers (slot 0 and 1, the same ``epoch``, any streams) completes
    second writes the struct root Keccak(pair_block[0:64]) to
    pair_block[64:96].  ``pair_block``: 128 bytes, zeroed before its first
    use; ``epoch``: 1 .. 2^30 - 1, a new one per pair."""
    dev = _dev(nodes)
    if pair_block.numel() < 128:
        raise ValueError("pair block of 128 bytes")
    if ws is None:
        ws = finish_workspace(count, nodes.device)
    _lib.invoke("mk_dev_ssz_merkle_finish_nodes_pair", _p(nodes), count, n_total, _p(pair_block), slot, epoch, _p(ws),
                ws.numel(), _stream(nodes.device), device=dev)


def top_fused_workspace(count0: int, count1: int, device) -> torch.Tensor:
    nb = _lib.load().mk_ssz_merkle_top_fused_workspace_bytes(count0, count1)
    if nb == 0:
        raise ValueError(f"fused top: bad counts {count0}, {count1}")
    return torch.empty(nb, dtype=torch.uint8, device=device)


def merkle_top_fused(nodes0: torch.Tensor, count0: int, n0: int, out: torch.Tensor, nodes1: torch.Tensor = None,
                     count1: int = 0, n1: int = 0, epoch: int = 0, ws: torch.Tensor = None) -> torch.Tensor:
    """The level loop + length mix-in of one list (count1 == 0: ``out`` gets
    the 32-B root) or of two lists side by side (``out`` a 128-B pair block,
    merkle_finish_nodes_pair semantics: the struct root at out[64:96],
    ``epoch`` 1 .. 2^30 - 1 a new one per pair), from a complete node level of
    each, in one launch (mk_dev_ssz_merkle_top_fused)."""
    dev = _dev(nodes0)
    if count1 and out.numel() < 128:
        raise ValueError("pair block of 128 bytes")
    if ws is None:
        ws = top_fused_workspace(count0, count1, nodes0.device)
    _lib.invoke("mk_dev_ssz_merkle_top_fused", _p(nodes0), count0, n0, _p(nodes1) if nodes1 is not None else None,
                count1, n1, _p(out), epoch, _p(ws), ws.numel(), _stream(nodes0.device), device=dev)
    return out


def merkle_finish_nodes(nodes: torch.Tensor, count: int, n_total: int, out: torch.Tensor = None,
                        ws: torch.Tensor = None) -> torch.Tensor:
    """Reference level loop over one gathered tree level of `count` nodes +
    length mix-in (the finisher of the frontier sharding)."""
    dev = _dev(nodes)
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=nodes.device)
    if ws is None:
        ws = finish_workspace(count, nodes.device)
    _lib.invoke("mk_dev_ssz_merkle_finish_nodes", _p(nodes), count, n_total, _p(out), _p(ws), ws.numel(),
                _stream(nodes.device), device=dev)
    return out


def merkle_finish(roots: torch.Tensor, nroots: int, n_total: int, out: torch.Tensor = None) -> torch.Tensor:
    """Reference level loop over gathered shard roots + length mix-in."""
    dev = _dev(roots)
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=roots.device)
    _lib.invoke("mk_dev_ssz_merkle_finish", _p(roots), nroots, n_total, _p(out), _stream(roots.device), device=dev)
    return out


def merkle_hash_multi(shards, n: int, item_len: int, out: torch.Tensor, streams=None) -> torch.Tensor:
    """Single-process multi-device merkleHash (the cgo caller's form):
    shards[d] on device d holds shard d of shard_plan(n, item_len,
    len(shards)); RCCL all-gather of the frontiers, device 0 finishes into
    ``out`` (a (32,) tensor on device 0)."""
    k = len(shards)
    ptrs = (ctypes.c_void_p * k)(*[s.data_ptr() for s in shards])
    sts = (ctypes.c_void_p * k)(*[(streams[d] if streams else torch.cuda.current_stream(shards[d].device)).cuda_stream
                                  for d in range(k)])
    _lib.invoke("mk_dev_ssz_merkle_hash_multi", ptrs, n, item_len, k, _p(out), sts, device=0)
    return out


def hash_batch(msgs: torch.Tensor, n: int, msg_len: int, out: torch.Tensor = None) -> torch.Tensor:
    """Batched Hash of n fixed-length messages resident on the device."""
    dev = _dev(msgs)
    if out is None:
        out = torch.empty(n * 32, dtype=torch.uint8, device=msgs.device)
    _lib.invoke("mk_dev_hash_batch", _p(msgs), n, msg_len, _p(out), _stream(msgs.device), device=dev)
    return out


def deposit_trie_levels_bytes(capacity: int, depth: int) -> int:
    return _lib.load().mk_deposit_trie_levels_bytes(capacity, depth)


def deposit_trie_append(levels: torch.Tensor, capacity: int, count: int, data: torch.Tensor, k: int,
                        fixed_len: int, depth: int, root: torch.Tensor, offs: torch.Tensor = None) -> None:
    """Append k deposits (fixed_len-byte records in ``data``, or variable
    length with device ``offs``) to the device trie holding ``count``
    deposits: UpdateDepositTrie (deposit_trie.go:29-40) batched, right edge
    of every level only; count == 0 is the batch build."""
    dev = _dev(levels)
    if offs is None and data.numel() < k * fixed_len:
        raise ValueError(f"deposit buffer holds {data.numel()} bytes < {k} x {fixed_len}")
    if levels.numel() < deposit_trie_levels_bytes(capacity, depth):
        raise ValueError("level buffer smaller than mk_deposit_trie_levels_bytes(capacity, depth)")
    _lib.invoke("mk_dev_deposit_trie_append", _p(levels), capacity, count, _p(data),
                _p(offs) if offs is not None else None, k, fixed_len, depth, _p(root), _stream(levels.device),
                device=dev)


def deposit_trie_build(levels: torch.Tensor, capacity: int, data: torch.Tensor, n: int, deposit_len: int,
                       d_to: int, depth: int, root: torch.Tensor = None) -> torch.Tensor:
    """Batch build front (deposit_trie.go:29-40): Hash of n fixed-length
    deposits into level 0 of an empty trie and levels 1..d_to (the root too
    when d_to == depth).  Returns ``levels``."""
    dev = _dev(levels)
    if n > capacity or levels.numel() < deposit_trie_levels_bytes(capacity, depth):
        raise ValueError("level array smaller than the capacity layout")
    if data.numel() * data.element_size() < n * deposit_len:
        raise ValueError("deposit buffer shorter than n * deposit_len")
    if d_to == depth and root is None:
        root = torch.empty(32, dtype=torch.uint8, device=levels.device)
    _lib.invoke("mk_dev_deposit_trie_build", _p(levels), capacity, _p(data), None, n, deposit_len, d_to, depth,
                _p(root) if root is not None else None, _stream(levels.device), device=dev)
    return levels


def deposit_trie_pipe_ok(data: torch.Tensor, n: int, deposit_len: int, depth: int) -> bool:
    """Whether deposit_trie_build_pipe takes this stream shape."""
    return bool(_lib.load().mk_deposit_trie_pipe_ok(_p(data), n, deposit_len, depth, _stream(data.device)))


def deposit_trie_build_pipe(levels: torch.Tensor, prev_levels, capacity: int, data: torch.Tensor, n: int,
                            deposit_len: int, depth: int) -> None:
    """Levels 0..2 of this trie and levels 3..7 of the previous trie of the
    stream (``prev_levels``, None for the first) in one launch
    (mk_dev_deposit_trie_build_pipe)."""
    _lib.invoke("mk_dev_deposit_trie_build_pipe", _p(levels), None if prev_levels is None else _p(prev_levels),
                capacity, _p(data), n, deposit_len, depth, _stream(levels.device), device=_dev(levels))


def deposit_trie_pipe_top(levels: torch.Tensor, capacity: int, count: int, depth: int, root: torch.Tensor) -> None:
    """Levels 8 .. depth and the root of a pipelined front's previous trie,
    in launches that fit beside the next front (mk_dev_deposit_trie_pipe_top)."""
    _lib.invoke("mk_dev_deposit_trie_pipe_top", _p(levels), capacity, count, depth, _p(root), _stream(levels.device),
                device=_dev(levels))


def deposit_trie_levels(levels: torch.Tensor, capacity: int, count: int, d_from: int, d_to: int, depth: int,
                        root: torch.Tensor = None) -> None:
    """Levels d_from+1 .. d_to of the batch build (level d_from complete);
    the root to ``root`` when d_to == depth."""
    dev = _dev(levels)
    _lib.invoke("mk_dev_deposit_trie_levels", _p(levels), capacity, count, d_from, d_to, depth,
                _p(root) if root is not None else None, _stream(levels.device), device=dev)


def deposit_trie_branch(levels: torch.Tensor, capacity: int, count: int, depth: int, index: int,
                        out: torch.Tensor = None) -> torch.Tensor:
    """GenerateMerkleBranch(index) of a device trie: (depth*32,) uint8."""
    dev = _dev(levels)
    if out is None:
        out = torch.empty(32 * depth, dtype=torch.uint8, device=levels.device)
    _lib.invoke("mk_dev_deposit_trie_branch", _p(levels), capacity, count, depth, index, _p(out),
                _stream(levels.device), device=dev)
    return out


def prof_enable(on: bool = True) -> None:
    _lib.check(_lib.load().mk_prof_enable(int(on)), "mk_prof_enable")


def prof_read():
    """(summed ms, launches, algorithmic permutations, digests) of the recorded leaf passes."""
    ms = ctypes.c_double()
    cnt = ctypes.c_uint64()
    perms = ctypes.c_double()
    hashes = ctypes.c_double()
    _lib.invoke("mk_prof_read", ctypes.byref(ms), ctypes.byref(cnt), ctypes.byref(perms), ctypes.byref(hashes))
    return ms.value, cnt.value, perms.value, hashes.value
