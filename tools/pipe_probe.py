"""Times the trie fronts alone (hipEvents around each launch, one stream):
the locked front k_trie_rec_lock<1024,4,false> (inside a whole-trie append:
front + top, and the top alone for the difference) against the pipelined
front <1024,4,true> without and with a previous trie."""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from prysm_amd import device as D  # noqa: E402

n, ln, depth = 1 << 20, 280, 32
dev = torch.device("cuda:0")
data = torch.empty(n * ln, dtype=torch.uint8, device=dev)
D.synth_fill(data, 0x5EED000000000005)
nb = D.deposit_trie_levels_bytes(n, depth)
A = torch.empty(nb, dtype=torch.uint8, device=dev)
B = torch.empty(nb, dtype=torch.uint8, device=dev)
root = torch.empty(32, dtype=torch.uint8, device=dev)


def t(fn, reps=20):
    out = []
    for r in range(reps + 3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        if r >= 3:
            out.append(e0.elapsed_time(e1) * 1e3)
    return round(statistics.median(out), 1), round(min(out), 1)


res = {}
res["append_whole_trie_us"] = t(lambda: D.deposit_trie_append(A, n, 0, data, n, ln, depth, root))
res["top_from_level2_us"] = t(lambda: D.deposit_trie_levels(A, n, n, 2, depth, depth, root))
res["pipe_front_no_prev_us"] = t(lambda: D.deposit_trie_build_pipe(A, None, n, data, n, ln, depth))
D.deposit_trie_build_pipe(B, None, n, data, n, ln, depth)
res["pipe_front_with_prev_us"] = t(lambda: D.deposit_trie_build_pipe(A, B, n, data, n, ln, depth))
res["pipe_top_from_level7_us"] = t(lambda: D.deposit_trie_pipe_top(B, n, n, depth, root))
print(json.dumps(res))
