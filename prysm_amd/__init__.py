"""prysm_amd — MI355X-native Merkleization engine for the Keccak-era Prysm
SSZ tree-hash path (shared/ssz, shared/hashutil, shared/trieutil).

Layout:
  csrc/        hand-written gfx950 HIP kernels + the C-ABI (libprysm_merkle.so)
  _lib.py      ctypes binding of include/prysm_merkle.h
  hashutil.py  Hash / batched Hash / MerkleRoot      (shared/hashutil)
  ssz.py       TreeHash / merkleHash                  (shared/ssz)
  trieutil.py  DepositTrie / VerifyMerkleBranch       (shared/trieutil)
  device.py    HBM-resident entry points (torch tensors + streams)
  parallel.py  subtree sharding across GPUs (torch.distributed / RCCL)
"""
from . import _lib  # noqa: F401

__all__ = ["hashutil", "ssz", "trieutil", "device", "parallel"]
