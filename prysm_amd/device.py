"""Device-resident entry points (inputs already in HBM), torch as plumbing.

torch provides device memory, the current HIP stream and torch.distributed;
every hash is computed by the HIP kernels behind the C-ABI
(``mk_dev_*`` in include/prysm_merkle.h).  Work is enqueued on torch's
current stream of the tensor's device and is not synchronised here.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib


def _stream(dev: torch.device):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def _p(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def _bind(t: torch.Tensor):
    if t.device.type != "cuda":
        raise _lib.MerkleError(_lib.MK_EINVAL, "device entry points need a GPU tensor")
    _lib.init(t.device.index or 0)


def synth_fill(dst: torch.Tensor, seed: int, word0: int = 0) -> torch.Tensor:
    """Fill ``dst`` (uint8, nbytes % 8 == 0) with bytes [8*word0, ...) of the
    SplitMix64 stream."""
    _bind(dst)
    _lib.check(_lib.load().mk_dev_synth_fill(_p(dst), dst.numel() * dst.element_size(), seed, word0,
                                             _stream(dst.device)), "mk_dev_synth_fill")
    return dst


def struct_roots(records: torch.Tensor, n: int, record_len: int, spec, out: torch.Tensor = None,
                 ws: torch.Tensor = None) -> torch.Tensor:
    """Struct root of each of n records (makeStructHasher per element,
    shared/ssz/hash.go:141-159; ``spec`` = [(kind, offset, len)] as in
    registry.VALIDATOR_FIELDS).  Returns an (n*32,) uint8 device tensor."""
    from .registry import _fields

    _bind(records)
    if records.numel() < n * record_len:
        raise ValueError("records tensor shorter than n*record_len")
    f = _fields(spec)
    L = _lib.load()
    if out is None:
        out = torch.empty(max(32, 32 * n), dtype=torch.uint8, device=records.device)
    if ws is None:
        ws = torch.empty(max(256, n * L.mk_ssz_struct_msg_len(f, len(spec))), dtype=torch.uint8,
                         device=records.device)
    _lib.check(L.mk_dev_ssz_struct_roots(_p(records), n, record_len, f, len(spec), _p(out), _p(ws), ws.numel(),
                                         _stream(records.device)), "mk_dev_ssz_struct_roots")
    return out


def merkle_workspace(n: int, item_len: int, device) -> torch.Tensor:
    nbytes = _lib.load().mk_ssz_merkle_workspace_bytes(n, item_len)
    return torch.empty(max(256, nbytes), dtype=torch.uint8, device=device)


def merkle_hash(items: torch.Tensor, n: int, item_len: int, out: torch.Tensor = None,
                ws: torch.Tensor = None) -> torch.Tensor:
    """ssz.merkleHash of n items of item_len bytes held in ``items`` (uint8,
    device).  Returns a (32,) uint8 device tensor."""
    _bind(items)
    if items.numel() < n * item_len:
        raise ValueError("items tensor shorter than n*item_len")
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=items.device)
    if ws is None:
        ws = merkle_workspace(n, item_len, items.device)
    _lib.check(_lib.load().mk_dev_ssz_merkle_hash(_p(items), n, item_len, _p(out), _p(ws), ws.numel(),
                                                  _stream(items.device)), "mk_dev_ssz_merkle_hash")
    return out


def shard_plan(n: int, item_len: int, nshards: int):
    """(height, nonempty, item_begin[nshards+1]) of the subtree sharding."""
    h = ctypes.c_uint32()
    ne = ctypes.c_uint32()
    begin = (ctypes.c_uint64 * (nshards + 1))()
    _lib.check(_lib.load().mk_ssz_merkle_shard_plan(n, item_len, nshards, ctypes.byref(h), ctypes.byref(ne),
                                                    begin), "mk_ssz_merkle_shard_plan")
    return h.value, ne.value, list(begin)


def subtree_workspace(shard_n: int, item_len: int, device) -> torch.Tensor:
    # the full-tree plan of the same item count bounds the subtree plan
    nbytes = _lib.load().mk_ssz_merkle_workspace_bytes(max(shard_n, 1), item_len) + 4096
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def merkle_subtree(items: torch.Tensor, shard_n: int, item_len: int, height: int, pad_at_one: bool,
                   out: torch.Tensor = None, ws: torch.Tensor = None) -> torch.Tensor:
    """32-B root of one shard at `height` levels above its chunks."""
    _bind(items)
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=items.device)
    if ws is None:
        ws = subtree_workspace(shard_n, item_len, items.device)
    _lib.check(_lib.load().mk_dev_ssz_merkle_subtree(_p(items), shard_n, item_len, height, int(pad_at_one), _p(out),
                                                     _p(ws), ws.numel(), _stream(items.device)),
               "mk_dev_ssz_merkle_subtree")
    return out


def merkle_subtree_frontier(items: torch.Tensor, shard_n: int, item_len: int, height: int, frontier_log2: int,
                            pad_at_one: bool, out: torch.Tensor = None, ws: torch.Tensor = None) -> torch.Tensor:
    """The shard's tree level `frontier_log2` levels below its root: a
    (nodes*32,) uint8 device tensor (nodes = parallel.frontier_count(...))."""
    _bind(items)
    from .parallel import frontier_count

    nodes = frontier_count(shard_n, item_len, height, frontier_log2)
    if out is None:
        out = torch.empty(32 << frontier_log2, dtype=torch.uint8, device=items.device)
    if out.numel() < 32 * nodes:
        raise ValueError("frontier output buffer too small")
    if ws is None:
        ws = subtree_workspace(shard_n, item_len, items.device)
    got = ctypes.c_uint64()
    _lib.check(_lib.load().mk_dev_ssz_merkle_subtree_frontier(
        _p(items), shard_n, item_len, height, frontier_log2, int(pad_at_one), _p(out), ctypes.byref(got), _p(ws),
        ws.numel(), _stream(items.device)), "mk_dev_ssz_merkle_subtree_frontier")
    assert got.value == nodes, (got.value, nodes)
    return out[:32 * nodes]


def merkle_node_frontier(nodes: torch.Tensor, count: int, height: int, frontier_log2: int, pad_at_one: bool,
                         out: torch.Tensor = None, ws: torch.Tensor = None) -> torch.Tensor:
    """A subtree continued from one of its node levels: `count` 32-B nodes
    reduced `height` levels (odd rule, hash.go:225-235), stopping
    `frontier_log2` levels below the top; returns the (nodes*32,) level."""
    _bind(nodes)
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
    _lib.check(lib.mk_dev_ssz_merkle_node_frontier(_p(nodes), count, height, frontier_log2, int(pad_at_one), _p(out),
                                                   ctypes.byref(got), _p(ws), ws.numel(), _stream(nodes.device)),
               "mk_dev_ssz_merkle_node_frontier")
    assert got.value == want, (got.value, want)
    return out[:32 * want]


def finish_workspace(count: int, device) -> torch.Tensor:
    return torch.empty(max(256, _lib.load().mk_ssz_merkle_finish_workspace_bytes(count)), dtype=torch.uint8,
                       device=device)


def merkle_finish_nodes(nodes: torch.Tensor, count: int, n_total: int, out: torch.Tensor = None,
                        ws: torch.Tensor = None) -> torch.Tensor:
    """Reference level loop over one gathered tree level of `count` nodes +
    length mix-in (the finisher of the frontier sharding)."""
    _bind(nodes)
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=nodes.device)
    if ws is None:
        ws = finish_workspace(count, nodes.device)
    _lib.check(_lib.load().mk_dev_ssz_merkle_finish_nodes(_p(nodes), count, n_total, _p(out), _p(ws), ws.numel(),
                                                          _stream(nodes.device)), "mk_dev_ssz_merkle_finish_nodes")
    return out


def merkle_finish(roots: torch.Tensor, nroots: int, n_total: int, out: torch.Tensor = None) -> torch.Tensor:
    """Reference level loop over gathered shard roots + length mix-in."""
    _bind(roots)
    if out is None:
        out = torch.empty(32, dtype=torch.uint8, device=roots.device)
    _lib.check(_lib.load().mk_dev_ssz_merkle_finish(_p(roots), nroots, n_total, _p(out), _stream(roots.device)),
               "mk_dev_ssz_merkle_finish")
    return out


def hash_batch(msgs: torch.Tensor, n: int, msg_len: int, out: torch.Tensor = None) -> torch.Tensor:
    """Batched Hash of n fixed-length messages resident on the device."""
    _bind(msgs)
    if out is None:
        out = torch.empty(n * 32, dtype=torch.uint8, device=msgs.device)
    _lib.check(_lib.load().mk_dev_hash_batch(_p(msgs), n, msg_len, _p(out), _stream(msgs.device)),
               "mk_dev_hash_batch")
    return out


def prof_enable(on: bool = True) -> None:
    _lib.check(_lib.load().mk_prof_enable(int(on)), "mk_prof_enable")


def prof_read():
    """(summed ms, launches, algorithmic permutations, digests) of the recorded leaf passes."""
    ms = ctypes.c_double()
    cnt = ctypes.c_uint64()
    perms = ctypes.c_double()
    hashes = ctypes.c_double()
    _lib.check(_lib.load().mk_prof_read(ctypes.byref(ms), ctypes.byref(cnt), ctypes.byref(perms), ctypes.byref(hashes)),
               "mk_prof_read")
    return ms.value, cnt.value, perms.value, hashes.value
