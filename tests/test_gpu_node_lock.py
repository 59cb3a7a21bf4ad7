"""The phase-locked node pass (k_node_lock, merkle_kernels.hip) against the
oracle.  A node pass of complete pairs runs it for whole multiples of 256
groups of 16,384 pairs (a level of >= 2^23 nodes: whole 2^28-item trees);
the pairs past the last group, the odd node and the levels above run the
ordinary passes.  Checked bit-exactly against or_merkle_nodes (hash.go's
level loop from a node level, oracle/merkle_ref.c) and or_merkle_hash_gen.
"""
import os

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SEED = 0x5EED0000000000AB
NTHREADS = min(16, os.cpu_count() or 1)


@pytest.fixture(scope="module")
def gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


def _nodes(gpu, count, seed=SEED):
    import torch

    from prysm_amd import device as D

    t = torch.empty(32 * count, dtype=torch.uint8, device=gpu)
    D.synth_fill(t, seed)
    return t


# 2^23: exactly 256 groups; + 2^15 + 7: two more k_reduce spans and an odd
# node after the groups; 2^24 + 3: 512 groups (2 per CU); 3 x 2^23 + 1: 768
# groups and an odd node; 2^23 - 2: below the threshold (255 groups' worth:
# k_reduce only), the control
@pytest.mark.parametrize("count", [1 << 23, (1 << 23) + (1 << 15) + 7, (1 << 24) + 3, 3 * (1 << 23) + 1,
                                   (1 << 23) - 2])
def test_finish_nodes_wide(gpu, count):
    import torch

    from prysm_amd import device as D

    nodes = _nodes(gpu, count)
    n_total = (count << 5) + 11
    root = D.merkle_finish_nodes(nodes, count, n_total)
    torch.cuda.synchronize()
    want = O.merkle_nodes(nodes.cpu().numpy(), count, n_total, nthreads=NTHREADS)
    assert bytes(root.cpu().numpy()) == want


@pytest.mark.parametrize("count,h", [(1 << 23, 23), ((1 << 24) - 5, 24)])
def test_node_frontier_wide(gpu, count, h):
    """Subtree mode (the sharded path's node passes): a 2^23-node level (256
    locked groups) or a ragged 2^24 - 5 one (256 locked groups, then k_reduce
    spans and an odd node) to a 1024-node frontier with the odd rule kept at
    count 1, then the finisher: equals the whole level's root."""
    import torch

    from prysm_amd import device as D

    k = 10
    nodes = _nodes(gpu, count, SEED + 1)
    lvl = D.merkle_node_frontier(nodes, count, h, k, True)
    root = D.merkle_finish_nodes(lvl, 1 << k, 12345)
    torch.cuda.synchronize()
    assert bytes(root.cpu().numpy()) == O.merkle_nodes(nodes.cpu().numpy(), count, 12345, nthreads=NTHREADS)


@pytest.mark.parametrize("n,item_len", [((1 << 28) + 12345, 32), ((1 << 28) - 31, 32), ((1 << 29) + 7, 32),
                                        ((1 << 26) + 5, 128)])
def test_whole_tree_ragged(gpu, n, item_len):
    """merkleHash of ragged 8-16 GiB trees: the locked leaf pass with its
    ragged last windows, then the locked node pass (2^23 nodes for the
    2^28-item trees, 2^24 -- two groups per CU -- for 2^29 + 7) followed by
    k_reduce spans and an odd node; 2^26 + 5 items of 128 B (one chunk per
    item) reach the same node level through the other chunk packing."""
    import torch

    from prysm_amd import device as D

    items = torch.empty(n * item_len + 8, dtype=torch.uint8, device=gpu)
    D.synth_fill(items, SEED + 2)
    root = D.merkle_hash(items[:n * item_len], n, item_len)
    torch.cuda.synchronize()
    got = bytes(root.cpu().numpy())
    del items
    torch.cuda.empty_cache()
    assert got == O.merkle_hash_gen(n, item_len, SEED + 2, nthreads=NTHREADS)
