"""GPU tests of the single-process multi-device entry points (the cgo
caller's form) and of the per-call context (mk_call) the C
ABI uses for device selection and error detail, plus the C99 pthread
harness (tests/c_abi/harness.c) against committed fixtures."""
import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x5EED000000000000 + 650


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    assert _lib.device_count() >= 1
    return torch.device("cuda:0")


def _multi_host(items: np.ndarray, n: int, item_len: int, devs):
    from prysm_amd import _lib

    out = ctypes.create_string_buffer(32)
    arr = (ctypes.c_int * len(devs))(*devs)
    _lib.invoke("mk_ssz_merkle_hash_multi", items.ctypes.data_as(ctypes.c_void_p), n, item_len, len(devs), arr, out)
    return out.raw


@pytest.mark.parametrize("n,nshards", [(12_345, 1), (1 << 20, 2), (1 << 20, 8), (999_999, 4), (5, 8),
                                       ((1 << 22) + 7, 8), (100_003, 3)])
def test_multi_shards_on_one_device(gpu, n, nshards):
    """Every shard on device 0: per-device upload thread, pinned staging,
    two alternating shard regions (upload of shard i+1 overlaps the passes of
    shard i), frontier blocks gathered by copy, finisher on device 0."""
    from oracle import oracle as O

    items = O.splitmix_bytes(n * 32, SEED + nshards)
    assert _multi_host(items, n, 32, [0] * nshards) == O.merkle_hash_flat(items, n, 32, nthreads=16)


def test_multi_shards_item_sizes(gpu):
    from oracle import oracle as O

    for n, il, k in ((300_001, 8, 4), (77_777, 3, 2), (20_000, 200, 4)):
        items = O.splitmix_bytes(n * il + 8, SEED + il)[:n * il]
        assert _multi_host(items, n, il, [0] * k) == O.merkle_hash_flat(items, n, il, nthreads=16), (n, il)


def test_multi_golden_2p26_eight_shards(gpu):
    """2^26 x 32-B items (2 GiB host buffer) as 8 shards through the
    host-buffer multi path; root vs the generator oracle."""
    from oracle import oracle as O

    n = 1 << 26
    items = O.splitmix_bytes(n * 32, SEED + 26)
    assert _multi_host(items, n, 32, [0] * 8) == O.merkle_hash_gen(n, 32, SEED + 26, nthreads=16)


@pytest.mark.parametrize("ndev", [2, 4, 8])
def test_multi_rccl_devices(gpu, ndev):
    """One shard per device, RCCL all-gather of the frontiers (xGMI): a ragged
    n and 2^24 items (host and device-resident forms, vs the oracle), then the
    golden-size C4 tree (2^28 items generated shard by shard on the devices,
    vs tests/golden/full_size_roots.json)."""
    import torch

    from oracle import oracle as O
    from prysm_amd import _lib
    from prysm_amd import device as D

    if _lib.device_count() < ndev:
        pytest.skip(f"needs {ndev} GPUs, {_lib.device_count()} visible")
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "full_size_roots.json")))["c4"]
    n, il = g["n"], g["item_len"]
    h, ne, begin = D.shard_plan(n, il, ndev)
    shards = []
    for d in range(ndev):
        t = torch.empty((begin[d + 1] - begin[d]) * il, dtype=torch.uint8, device=f"cuda:{d}")
        D.synth_fill(t, g["seed"], begin[d] * il // 8)
        shards.append(t)
    out = torch.empty(32, dtype=torch.uint8, device="cuda:0")
    D.merkle_hash_multi(shards, n, il, out)
    for d in range(ndev):
        torch.cuda.synchronize(d)
    assert bytes(out.cpu().numpy()).hex() == g["root"]
    del shards
    for n in (999_999, 1 << 24):
        items = O.splitmix_bytes(n * 32, SEED + 77)
        want = O.merkle_hash_flat(items, n, 32, nthreads=16)
        assert _multi_host(items, n, 32, list(range(ndev))) == want
        h, ne, begin = D.shard_plan(n, 32, ndev)
        shards = [torch.from_numpy(items[begin[d] * 32:max(begin[d + 1], begin[d] + 1) * 32].copy()).to(f"cuda:{d}")
                  for d in range(ndev)]
        out = torch.empty(32, dtype=torch.uint8, device="cuda:0")
        D.merkle_hash_multi(shards, n, 32, out)
        for d in range(ndev):
            torch.cuda.synchronize(d)
        assert bytes(out.cpu().numpy()) == want


def test_dev_multi_single_device(gpu):
    """mk_dev_ssz_merkle_hash_multi with one device is the plain plan on the
    caller's stream."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n = 300_007
    items = torch.empty(n * 32, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 5)
    out = torch.empty(32, dtype=torch.uint8, device=gpu)
    D.merkle_hash_multi([items], n, 32, out)
    torch.cuda.synchronize()
    assert bytes(out.cpu().numpy()) == O.merkle_hash_gen(n, 32, SEED + 5, nthreads=16)


def test_dev_multi_then_host_call_unsynchronised(gpu):
    """A host-buffer merkleHash issued right after a device-resident multi
    call, with no synchronisation in between: the multi path has its own
    per-device buffers, so neither root is disturbed (the host call runs on
    the library's stream while the multi call's work is still queued on the
    caller's)."""
    import torch

    from oracle import oracle as O
    from prysm_amd import device as D

    n1, n2 = 1 << 20, 200_003
    items = torch.empty(n1 * 32, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 31)
    host = O.splitmix_bytes(n2 * 32, SEED + 32)
    out = torch.empty(32, dtype=torch.uint8, device=gpu)
    torch.cuda.synchronize()
    for _ in range(3):
        D.merkle_hash_multi([items], n1, 32, out)
        got2 = _host_merkle(host, n2, 32)
        torch.cuda.synchronize()
        assert bytes(out.cpu().numpy()) == O.merkle_hash_gen(n1, 32, SEED + 31, nthreads=16)
        assert got2 == O.merkle_hash_flat(host, n2, 32, nthreads=16)


def _host_merkle(items: np.ndarray, n: int, item_len: int) -> bytes:
    from prysm_amd import _lib

    out = ctypes.create_string_buffer(32)
    _lib.invoke("mk_ssz_merkle_hash", items.ctypes.data_as(ctypes.c_void_p), n, item_len, out)
    return out.raw


def test_call_context_errors_and_device_restore(gpu):
    import torch

    from prysm_amd import _lib

    L = _lib.load()
    call = _lib.Call(-1, 0, b"")
    out = ctypes.create_string_buffer(32)
    rc = L.mk_ssz_merkle_hash(ctypes.byref(call), None, 5, 0, out)
    assert rc == _lib.MK_EINVAL and call.code == rc and b"divide by zero" in call.err
    call = _lib.Call(77, 0, b"")
    rc = L.mk_hash(ctypes.byref(call), b"abc", 3, out)
    assert rc == _lib.MK_ENODEV and b"device 77 out of range" in call.err
    # a device-resident call on a stream: the stream's device wins; a
    # conflicting call->device is an error, not a silent retarget
    if _lib.device_count() >= 2:
        st = torch.cuda.Stream(device="cuda:1")
        buf = torch.zeros(64, dtype=torch.uint8, device="cuda:1")
        call = _lib.Call(0, 0, b"")
        rc = L.mk_dev_hash_batch(ctypes.byref(call), buf.data_ptr(), 1, 64, buf.data_ptr(), st.cuda_stream)
        assert rc == _lib.MK_EINVAL and b"stream belongs to device 1" in call.err
    # the thread's current device is unchanged by a call that targets another one
    cur = torch.cuda.current_device()
    call = _lib.Call(_lib.device_count() - 1, 0, b"")
    assert L.mk_hash(ctypes.byref(call), b"abc", 3, out) == 0
    assert torch.cuda.current_device() == cur
    assert out.raw.hex() == "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"


def test_c_abi_harness_8_threads(gpu):
    """tests/c_abi/harness.c (C99 against include/prysm_merkle.h, linked to
    libprysm_merkle.so): 8 pthreads x 2 rounds of merkleHash, Hash batches,
    the deposit-trie handle, many lists and per-call errors, vs fixtures."""
    exe = _build_harness()
    with open(os.path.join(ROOT, "tests", "golden", "c_abi_fixture.json")) as f:
        fx = json.load(f)
    args = [exe, "8", "2"] + fx["merkle"] + fx["batch"] + [fx["trie_root"], fx["branch"]] + fx["many"]
    r = subprocess.run(args, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: 8 threads x 2 rounds" in r.stdout


def test_c_abi_cgo_replay(gpu):
    """`harness cgo`: the call sequences of INTEGRATION.md's Go wrappers
    replayed from C99 exactly as cgo makes them (NULL for an empty Go slice),
    every early-return branch included -- merkleHash over a flattened
    [][]byte with n = 0, 1, 2, 5, 10 and len(list[0]) == 0;
    TreeHashBytesList with n = 0 and elemLen = 0; MerkleHashMany with k = 0;
    HashBatch with n = 0; trie Append / SaveLogs of nothing -- against the
    reference's vectors (hash_test.go:80-81,151-178) and oracle fixtures."""
    exe = _build_harness()
    with open(os.path.join(ROOT, "tests", "golden", "c_abi_fixture.json")) as f:
        cg = json.load(f)["cgo"]
    keys = ["m0", "m1", "m2", "m5", "m10x16", "m10x32", "t0", "tz4", "t1x6"]
    r = subprocess.run([exe, "cgo"] + [cg[k] for k in keys], capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: cgo replay" in r.stdout and "MISMATCH" not in r.stdout


def test_c_abi_injected_failure_surfaces(gpu):
    """With the library's failure-injection hook (MK_INJECT_EHIP=1), every
    compute family returns MK_EHIP with the detail in its own mk_call: the
    cgo binding turns that into an error and never into
    a CPU answer."""
    exe = _build_harness()
    r = subprocess.run([exe, "inject"], capture_output=True, text=True, timeout=110,
                       env=dict(os.environ, MK_INJECT_EHIP="1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: injected failures surfaced as MK_EHIP" in r.stdout


def _build_harness() -> str:
    out = os.path.join(ROOT, "tests", "c_abi", "harness")
    src = os.path.join(ROOT, "tests", "c_abi", "harness.c")
    if not os.path.exists(out) or os.path.getmtime(out) < os.path.getmtime(src):
        lib = os.path.join(ROOT, "prysm_amd", "lib")
        subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"), src,
                        "-L" + lib, "-lprysm_merkle", "-lpthread", "-Wl,-rpath," + lib, "-o", out], check=True)
    return out
