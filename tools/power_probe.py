"""Keeps one config's hot path busy for --seconds (C4: merkleHash of 2^28
x 32-B items; C5: the stream of 2^20-deposit tries) so rocm-smi can read the
package power and shader clock under sustained load."""
import argparse
import sys
import time

import torch

sys.path.insert(0, ".")
from prysm_amd import device as D  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c4")
ap.add_argument("--seconds", type=float, default=40)
a = ap.parse_args()
dev = torch.device("cuda:0")
if a.config == "c4":
    n = 1 << 28
    items = torch.empty(n * 32, dtype=torch.uint8, device=dev)
    D.synth_fill(items, 0x5EED000000000004)
    ws = D.merkle_workspace(n, 32, dev)
    out = torch.empty(32, dtype=torch.uint8, device=dev)
    step = lambda: D.merkle_hash(items, n, 32, out=out, ws=ws)  # noqa: E731
else:
    from prysm_amd.pipeline import TriePipeline

    n = 1 << 20
    data = torch.empty(n * 280, dtype=torch.uint8, device=dev)
    D.synth_fill(data, 0x5EED000000000005)
    pipe = TriePipeline(n, 280, 32, dev, front="pipe")
    step = lambda: pipe.submit(data)  # noqa: E731
step()
torch.cuda.synchronize()
print("busy", flush=True)
t0, k = time.time(), 0
while time.time() - t0 < a.seconds:
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    k += 20
print(f"steps {k} in {time.time() - t0:.1f} s", flush=True)
