"""Rank body for tests/test_gpu_nccl.py: one rank of backend "nccl" (RCCL)
on cuda:0.  RCCL refuses two ranks on one device ("Duplicate GPU detected",
profiles/r02g/nccl_share2.err), so a one-GPU box can only run world 1; this
runs rank 0's exact frontier path with a real RCCL all-gather: the shard's
1024-node frontier (mk_dev_ssz_merkle_subtree_frontier), the all-gather
issued on a high-priority side stream through the process group's own
high-priority stream, the finisher on that side stream — twice, double-
buffered like ShardedMerklePipeline — and prints {"root", "want"} where
want is the one-call merkleHash of the same items."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from prysm_amd import device as D  # noqa: E402
from prysm_amd import parallel as P  # noqa: E402


def lib_main(log2n: int, n_extra: int):
    """The library's own RCCL code (MK_FORCE_COLLECTIVE=1, set by the test
    before this process loads the library): mk_dev_ssz_merkle_hash_multi and
    mk_ssz_merkle_hash_multi over one device run the one-shard sharded path
    (frontier, ncclCommInitAll + in-place ncclAllGather, finisher)."""
    import ctypes

    from prysm_amd import _lib

    assert os.environ.get("MK_FORCE_COLLECTIVE") == "1"
    dev = torch.device("cuda", 0)
    n, il = (1 << log2n) + n_extra, 32
    items = torch.empty(n * il, dtype=torch.uint8, device=dev)
    D.synth_fill(items, 0x5EED000000000000 + 778)
    want = bytes(D.merkle_hash(items, n, il).cpu().numpy()).hex()
    out = torch.empty(32, dtype=torch.uint8, device=dev)
    got_dev = [bytes(D.merkle_hash_multi([items], n, il, out).cpu().numpy()).hex() for _ in range(2)]
    host = items.cpu().numpy()
    buf = ctypes.create_string_buffer(32)
    devs = (ctypes.c_int * 1)(0)
    _lib.invoke("mk_ssz_merkle_hash_multi", host.ctypes.data_as(ctypes.c_void_p), n, il, 1, devs, buf)
    print(json.dumps({"root": got_dev + [buf.raw.hex()], "want": want}), flush=True)


def main():
    if sys.argv[1] == "lib":
        return lib_main(int(sys.argv[2]), int(sys.argv[3]))
    log2n, k = int(sys.argv[1]), int(sys.argv[2])
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    P.init_process_group("nccl", dev)
    assert dist.get_world_size() == 1 and dist.get_backend() == "nccl"
    n, il = 1 << log2n, 32
    items = torch.empty(n * il, dtype=torch.uint8, device=dev)
    D.synth_fill(items, 0x5EED000000000000 + 777)
    want = bytes(D.merkle_hash(items, n, il).cpu().numpy()).hex()
    # one shard holding the whole tree: its height is the tree's chunk height
    height = (n * il // 128 - 1).bit_length()
    assert D.shard_plan(n, il, 1)[0] in (0, height)  # the planner's view of the same tree
    side = torch.cuda.Stream(device=dev, priority=-1)
    ws = D.subtree_workspace(n, il, dev)
    fws = D.finish_workspace(1 << k, dev)
    blocks = [torch.empty(32 << k, dtype=torch.uint8, device=dev) for _ in range(2)]
    gathered = [torch.empty(32 << k, dtype=torch.uint8, device=dev) for _ in range(2)]
    outs = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(2)]
    cur = torch.cuda.current_stream(dev)
    roots = []
    for i in range(2):
        D.merkle_subtree_frontier(items, n, il, height, k, True, out=blocks[i], ws=ws)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            dist.all_gather_into_tensor(gathered[i], blocks[i])
            roots.append(D.merkle_finish_nodes(gathered[i], 1 << k, n, out=outs[i], ws=fws))
    torch.cuda.synchronize()
    got = [bytes(r.cpu().numpy()).hex() for r in roots]
    dist.destroy_process_group()
    print(json.dumps({"root": got, "want": want, "height": height, "frontier": k,
                      "rccl": ".".join(map(str, torch.cuda.nccl.version()))}), flush=True)


if __name__ == "__main__":
    main()
