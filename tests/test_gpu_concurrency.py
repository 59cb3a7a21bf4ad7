"""The C ABI's threading contract (Go may call from any OS
thread, concurrently; every entry binds its device and takes the per-device
lock): 8 host threads call the host-buffer entry points at once — ctypes
drops the GIL for the foreign call, so the calls overlap inside the library
— and every result is checked against the oracle."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 901


@pytest.fixture(scope="module")
def gpu():
    import torch

    from prysm_amd import _lib

    assert torch.cuda.is_available()
    _lib.init(0)
    return torch.device("cuda:0")


def test_concurrent_host_entry_points(gpu):
    from oracle import oracle as O
    from prysm_amd import hashutil as H
    from prysm_amd import ssz
    from prysm_amd import trieutil as T

    jobs = []
    for t in range(8):
        n = 5_000 + 977 * t
        items = O.splitmix_bytes(n * 32, SEED + t)
        msgs = O.splitmix_bytes(300 * 136, SEED + 100 + t)
        deps = [bytes(O.splitmix_bytes(280, SEED + 200 + t, 35 * i)) for i in range(33 + t)]
        jobs.append((n, items, msgs, deps, O.merkle_hash_flat(items, n, 32), O.keccak256_batch(msgs, 136),
                     O.deposit_trie_levels(deps)[0]))
    errors = []
    start = threading.Barrier(len(jobs))

    def worker(j):
        n, items, msgs, deps, want_root, want_hashes, want_trie = jobs[j]
        try:
            start.wait()
            for _ in range(10):
                assert ssz.merkle_hash_flat(items, n, 32) == want_root
                assert np.array_equal(H.hash_batch(msgs, 136), want_hashes)
                assert T.build_levels(deps)[0] == bytes(want_trie)
        except Exception as e:  # noqa: BLE001 - reported below
            errors.append((j, repr(e)))

    threads = [threading.Thread(target=worker, args=(j,)) for j in range(len(jobs))]
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in threads), "a worker hung"
    assert not errors, errors
