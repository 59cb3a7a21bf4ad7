"""Where the C3 step's tree phase goes (1M-validator State, device-resident):
median times, one process, interleaved rounds, of
  struct   the struct-roots kernel alone
  reg      the registry tree (merkleHash of 10^6 32-B roots) alone
  bal      the balances tree (merkleHash of 10^6 u64) alone
  side     both trees side by side (DeviceStateHasher's schedule)
  seq_rb   both trees on one stream, registry first
  seq_br   both trees on one stream, balances first
  step     DeviceStateHasher.submit (struct + trees + the state hash)

  python tools/c3_tree_probe.py [--rounds 7] [--steps 20]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    import numpy as np
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd import registry as R

    dev = torch.device("cuda:0")
    n, seed = 1_000_000, 0x5EED000000000003
    reg, bal = R.synthetic_registry(n, seed), R.synthetic_balances(n, seed)
    rec = torch.from_numpy(reg.records.view(np.uint8).reshape(-1).copy()).to(dev)
    dbal = torch.from_numpy(bal.view(np.uint8).copy()).to(dev)
    want = R.state_root(reg, bal)
    h = R.DeviceStateHasher(n, dev)
    got = bytes(h.submit(rec, dbal).cpu().numpy())
    assert got == want, "state root"
    side = torch.cuda.Stream(device=dev, priority=-1)
    ev = torch.cuda.Event()

    def tree_reg():
        D.merkle_hash(h.roots, n, 32, out=h.pair[:32], ws=h.reg_ws)

    def tree_bal():
        D.merkle_hash(dbal, n, 8, out=h.pair[32:], ws=h.bal_ws)

    def both_side():
        cur = torch.cuda.current_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            tree_bal()
            ev.record(side)
        tree_reg()
        cur.wait_event(ev)

    cases = {
        "struct": lambda: D.struct_roots(rec, n, 160, R.VALIDATOR_FIELDS, out=h.roots, ws=h.msg_ws),
        "reg": tree_reg,
        "bal": tree_bal,
        "side": both_side,
        "seq_rb": lambda: (tree_reg(), tree_bal()),
        "seq_br": lambda: (tree_bal(), tree_reg()),
        "step": lambda: h.submit(rec, dbal),
    }
    times = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, f in cases.items():
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.steps):
                f()
            t1.record()
            torch.cuda.synchronize()
            times[k].append(t0.elapsed_time(t1) / a.steps)
    assert bytes(h.submit(rec, dbal).cpu().numpy()) == want
    torch.cuda.synchronize()
    ver = _lib.load().mk_version().decode()
    for k, t in times.items():
        print(json.dumps({"case": k, "median_ms": round(statistics.median(t), 4), "min_ms": round(min(t), 4),
                          "lib": os.environ.get("PRYSM_MERKLE_LIB") or "main", "version": ver}))


if __name__ == "__main__":
    main()
