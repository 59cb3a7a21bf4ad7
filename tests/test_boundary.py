"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports
every symbol include/prysm_merkle.h declares, and its pure-host logic (the
shard planner, workspace sizing, argument errors) behaves — no GPU compute."""
import ctypes
import os

import pytest

from prysm_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__

        __graft_entry__.build()
    return _lib.load()


def test_header_declares_the_boundary():
    syms = _lib.header_symbols()
    for s in ("mk_init", "mk_hash", "mk_hash_batch", "mk_ssz_merkle_hash", "mk_dev_ssz_merkle_hash",
              "mk_dev_ssz_merkle_subtree", "mk_dev_ssz_merkle_finish", "mk_ssz_merkle_hash_multi",
              "mk_deposit_trie_build", "mk_verify_merkle_branches"):
        assert s in syms
    assert set(syms) == set(_lib._SIGS), "ctypes signature table out of sync with the header"


def test_library_exports_every_header_symbol(lib):
    missing = [s for s in _lib.header_symbols() if not hasattr(lib, s)]
    assert not missing
    assert lib.mk_version().decode().startswith("prysm_merkle")
    assert lib.mk_strerror(_lib.MK_ENODEV) == b"no usable gfx950 device"


def test_library_is_gfx950_code_object(lib):
    with open(_lib.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"gfx950" in blob
    assert b"k_reduce" in blob


def _plan(lib, n, item_len, world):
    h, ne = ctypes.c_uint32(), ctypes.c_uint32()
    begin = (ctypes.c_uint64 * (world + 1))()
    rc = lib.mk_ssz_merkle_shard_plan(None, n, item_len, world, ctypes.byref(h), ctypes.byref(ne), begin)
    return rc, h.value, ne.value, list(begin)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_shard_plan_c4(lib, world):
    n = 1 << 28
    rc, h, ne, begin = _plan(lib, n, 32, world)
    assert rc == 0
    chunks = n // 4
    assert (1 << h) * world == chunks or world == 1
    assert begin[0] == 0 and begin[-1] == n
    if world > 1:
        assert ne == world
        assert all(begin[i + 1] - begin[i] == n // world for i in range(world))


@pytest.mark.parametrize("n,item_len,world", [(4099, 32, 8), (1000, 8, 3), (41 * 4 + 3, 32, 4), (5, 32, 8),
                                              (0, 32, 4), (100, 200, 8), (10**6, 32, 8)])
def test_shard_plan_properties(lib, n, item_len, world):
    rc, h, ne, begin = _plan(lib, n, item_len, world)
    assert rc == 0
    per = 128 // item_len if item_len < 128 else 1
    chunks = -(-n * item_len // (per * item_len)) if n else 0
    assert begin[0] == 0 and begin[-1] == n and begin == sorted(begin)
    if ne > 1:
        assert (1 << h) * (ne - 1) < chunks <= (1 << h) * ne
        assert (1 << h) * world >= chunks
        for s in range(ne - 1):  # every non-last non-empty shard is full
            assert begin[s + 1] - begin[s] == (1 << h) * per
    else:
        assert begin[1] == n


def test_workspace_sizing(lib):
    assert lib.mk_ssz_merkle_workspace_bytes(0, 32) >= 32
    ws = lib.mk_ssz_merkle_workspace_bytes(1 << 28, 32)
    if b"leaf_lock=1" in lib.mk_version():
        # phase-locked leaf pass (3 levels): pass outputs 2^23 + 2^18 nodes of 32 B
        assert 32 * ((1 << 23) + (1 << 18)) <= ws < 300 << 20
    else:
        # fused leaf pass (5 levels): pass outputs 2^21 + 2^16 nodes of 32 B
        assert 32 * ((1 << 21) + (1 << 16)) <= ws < 80 << 20
    assert lib.mk_ssz_merkle_workspace_bytes(10, 0) == 0  # item_len 0 is invalid
    assert lib.mk_deposit_trie_levels_bytes(0, 32) == 0
    assert lib.mk_deposit_trie_levels_bytes(5, 2) == 32 * (5 + 3 + 2)


def test_node_frontier_planner(lib):
    """mk_dev_ssz_merkle_node_frontier's planner (no GPU needed for the
    workspace query): the per-rank split of the 8-GPU C4 shard (2^18 leaf-pass
    nodes, 18 levels to the shard root, frontier 10) plans; a frontier at or
    above the top, or more nodes than the height allows, does not."""
    assert lib.mk_ssz_merkle_node_frontier_workspace_bytes(1 << 18, 18, 10) >= 256
    assert lib.mk_ssz_merkle_node_frontier_workspace_bytes(1 << 18, 18, 0) >= 256
    assert lib.mk_ssz_merkle_node_frontier_workspace_bytes((1 << 18) - 7, 18, 10) >= 256  # ragged shard
    assert lib.mk_ssz_merkle_node_frontier_workspace_bytes(1, 18, 10) >= 256  # lone node (pad_at_one)
    assert lib.mk_ssz_merkle_node_frontier_workspace_bytes(1 << 18, 18, 18) == 0
    assert lib.mk_ssz_merkle_node_frontier_workspace_bytes((1 << 18) + 1, 18, 10) == 0


def test_oracle_is_not_imported_by_product():
    """The product package never touches oracle/ (it is test infrastructure)."""
    pkg = os.path.join(ROOT, "prysm_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f
                assert "liboracle" not in txt, f


def test_c99_harness_compiles_against_the_header(lib, tmp_path):
    """The header is plain C99 (what cgo compiles): the pthread harness
    builds with -std=c99 -Wall -Werror and links libprysm_merkle.so."""
    import subprocess

    src = os.path.join(ROOT, "tests", "c_abi", "harness.c")
    libdir = os.path.join(ROOT, "prysm_amd", "lib")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-pedantic", "-I" + os.path.join(ROOT, "include"), src,
                    "-L" + libdir, "-lprysm_merkle", "-lpthread", "-Wl,-rpath," + libdir,
                    "-o", str(tmp_path / "harness")], check=True)


def test_call_context_carries_errors_without_a_gpu(lib):
    """Errors come back in the failing call's own mk_call (cgo may move a
    goroutine between OS threads between two C calls)."""
    call = _lib.Call(-1, 0, b"")
    h, ne = ctypes.c_uint32(), ctypes.c_uint32()
    begin = (ctypes.c_uint64 * 2)()
    rc = lib.mk_ssz_merkle_shard_plan(ctypes.byref(call), 10, 32, 0, ctypes.byref(h), ctypes.byref(ne), begin)
    assert rc == _lib.MK_EINVAL and call.code == rc and call.err == b"nshards == 0"
    rc = lib.mk_ssz_merkle_shard_plan(ctypes.byref(call), 10, 32, 1, ctypes.byref(h), ctypes.byref(ne), begin)
    assert rc == 0 and call.code == 0 and call.err == b""
    if _lib.device_count() == 0:
        out = ctypes.create_string_buffer(32)
        rc = lib.mk_hash(ctypes.byref(call), b"abc", 3, out)
        assert rc == _lib.MK_ENODEV and call.err == b"no gfx950 device visible"
