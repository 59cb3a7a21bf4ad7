"""TriePipeline split-level A/B (which level the side stream starts at) on
the 2^20-deposit C5 trie, rounds interleaved; every root must agree.

  python tools/trie_split_ab.py
"""
import sys, time, json, torch
sys.path.insert(0, '.')
from prysm_amd import device as D
from prysm_amd.pipeline import TriePipeline
dev = torch.device('cuda:0')
n, ln, depth = 1 << 20, 280, 32
data = torch.empty(n * ln, dtype=torch.uint8, device=dev)
D.synth_fill(data, 0x5EED000000000005)
roots = set()
for rnd in range(3):
    for split in (0, 1, 2, 3, 4, 5, 6):
        p = TriePipeline(n, ln, depth, dev, split=split)
        for _ in range(20): p.submit(data)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(30): r = p.submit(data)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) / 30 * 1e3
        roots.add(bytes(r.cpu().numpy()))
        print(json.dumps({"round": rnd, "split": split, "ms_per_trie": ms}), flush=True)
assert len(roots) == 1
