"""C3 as a stream of states: state i's record roots on the main stream, its
two trees (registry merkleHash over the roots, balances merkleHash) and the
State hash on a high-priority side stream overlapping state i+1's record
roots; `slots` buffer sets (a submit waits for the side work `slots` states
back).  Compares ms/state against the one-state step bench.py --config c3
times, in one process; every root must equal the one-state root.

  PRYSM_MERKLE_LIB=<lib> python tools/c3_stream_probe.py [--slots 2 3 4]
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--slots", type=int, nargs="+", default=[2, 3, 4])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    import torch

    from prysm_amd import _lib
    from prysm_amd import device as D
    from prysm_amd import registry as R

    dev = torch.device("cuda:0")
    L = _lib.load()
    n = 1_000_000
    seed = 0x5EED000000000000 + 3
    rec = R.synthetic_registry_device(n, seed, dev)
    bal = R.synthetic_balances_device(n, seed, dev)
    spec = R._fields(R.VALIDATOR_FIELDS)
    nf = len(R.VALIDATOR_FIELDS)
    st = lambda: ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)  # noqa: E731
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731

    # the one-state step of bench.py --config c3
    ws1 = torch.empty(L.mk_ssz_struct_list_workspace_bytes(n, spec, nf) + 4096, dtype=torch.uint8, device=dev)
    bws1 = D.merkle_workspace(n, 8, dev)
    roots1 = torch.empty(64, dtype=torch.uint8, device=dev)
    out1 = torch.empty(32, dtype=torch.uint8, device=dev)
    side1 = torch.cuda.Stream(device=dev, priority=-1)

    def one_state():
        cur = torch.cuda.current_stream(dev)
        side1.wait_stream(cur)
        with torch.cuda.stream(side1):
            D.merkle_hash(bal, n, 8, out=roots1[32:], ws=bws1)
        _lib.check(L.mk_dev_ssz_struct_list_root(None, P(rec), n, 160, spec, nf, P(roots1), P(ws1), ws1.numel(),
                                                 st()), "registry")
        cur.wait_stream(side1)
        _lib.check(L.mk_dev_hash_batch(None, P(roots1), 1, 64, P(out1), st()), "state")
        return out1

    def timeit(fn):
        for _ in range(a.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            r = fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.steps * 1e3, bytes(r.cpu().numpy()).hex()

    def make_stream(S):
        side = torch.cuda.Stream(device=dev, priority=-1)
        rts = [torch.empty(32 * n, dtype=torch.uint8, device=dev) for _ in range(S)]
        rws = [D.merkle_workspace(n, 32, dev) for _ in range(S)]
        bws = [D.merkle_workspace(n, 8, dev) for _ in range(S)]
        pair = [torch.empty(64, dtype=torch.uint8, device=dev) for _ in range(S)]
        outs = [torch.empty(32, dtype=torch.uint8, device=dev) for _ in range(S)]
        sws = torch.empty(max(256, n * L.mk_ssz_struct_msg_len(spec, nf)), dtype=torch.uint8, device=dev)
        done = [None] * S
        state = {"i": 0}

        def submit():
            s = state["i"] % S
            state["i"] += 1
            cur = torch.cuda.current_stream(dev)
            if done[s] is not None:
                cur.wait_event(done[s])
            D.struct_roots(rec, n, 160, R.VALIDATOR_FIELDS, out=rts[s], ws=sws)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                D.merkle_hash(rts[s], n, 32, out=pair[s][:32], ws=rws[s])
                D.merkle_hash(bal, n, 8, out=pair[s][32:], ws=bws[s])
                _lib.check(L.mk_dev_hash_batch(None, P(pair[s]), 1, 64, P(outs[s]),
                                               ctypes.c_void_p(side.cuda_stream)), "state")
                ev = torch.cuda.Event()
                ev.record(side)
            done[s] = ev
            return outs[s]
        return submit

    res = {"lib": os.path.basename(os.environ.get("PRYSM_MERKLE_LIB") or "main")}
    for r in range(a.rounds):
        ms, root = timeit(one_state)
        res.setdefault("one_state_ms", []).append(round(ms, 4))
        res["root"] = root
        for S in a.slots:
            ms, got = timeit(make_stream(S))
            assert got == root, (S, got, root)
            res.setdefault(f"stream{S}_ms", []).append(round(ms, 4))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
