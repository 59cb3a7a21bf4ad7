"""registry.StatePipeline (BASELINE config 3 as a stream of states): each
state's struct launch also builds levels 2..10 of the previous state's
registry tree in its lock-step slots (k_struct_lock<true>), the rest of the
previous registry tree and the balances tree run on side streams.  Every
state root against the one-state path / the golden, the slot-built levels
against the oracle, the ragged last subtree, flush mid-stream, bad shapes."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED000000000000 + 1300


@pytest.fixture(scope="module")
def gpu():
    import torch

    assert torch.cuda.is_available()
    return torch.device("cuda:0")


def _states(n, seeds, dev):
    from prysm_amd import registry as R

    return [(R.synthetic_registry_device(n, s, dev), R.synthetic_balances_device(n, s, dev)) for s in seeds]


def _one_state_roots(n, states, dev):
    """The same states through DeviceStateHasher (one state per call)."""
    import torch

    from prysm_amd import registry as R

    h = R.DeviceStateHasher(n, dev)
    out = []
    for rec, bal in states:
        r = h.submit(rec, bal)
        torch.cuda.synchronize()
        out.append(bytes(r.cpu().numpy()))
    return out


@pytest.mark.parametrize("n", [1_000_000, 1 << 20, 786_433, 1_000_003])
def test_state_pipeline_roots(gpu, n):
    import torch

    from prysm_amd import device as D
    from prysm_amd import registry as R

    states = _states(n, [SEED + 7 * t + n % 97 for t in range(6)], gpu)
    assert D.struct_pipe_ok(states[0][0], n, 160, R.VALIDATOR_FIELDS)
    want = _one_state_roots(n, states, gpu)
    assert len(set(want)) == len(want)
    p = R.StatePipeline(n, gpu)
    got = []
    for t, (rec, bal) in enumerate(states):
        h = p.submit(rec, bal)
        if t:
            p.wait()
            torch.cuda.synchronize()
            got.append(bytes(prev.cpu().numpy()))
        prev = h
    p.flush()
    p.wait()
    torch.cuda.synchronize()
    got.append(bytes(prev.cpu().numpy()))
    assert got == want


def test_state_pipeline_golden_1m(gpu):
    """The C3 configuration: 10^6 validators of the golden seed, three states
    in a stream, every root equal to the committed golden state root."""
    import json
    import os

    import torch

    from prysm_amd import registry as R

    g = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "full_size_roots.json")))["c3"]
    rec = R.synthetic_registry_device(g["n"], g["seed"], gpu)
    bal = R.synthetic_balances_device(g["n"], g["seed"], gpu)
    p = R.StatePipeline(g["n"], gpu)
    handles = [p.submit(rec, bal) for _ in range(3)]
    p.flush()
    p.wait()
    torch.cuda.synchronize()
    for h in handles:
        assert bytes(h.cpu().numpy()).hex() == g["state_root"]


def test_state_pipeline_slot_levels_vs_oracle(gpu):
    """The slot levels the second launch built for the first state -- the
    registry's 2..10 and the balances' 2..4 -- subtree by subtree (first,
    middle, last complete one), against the oracle's node hashes over the
    first launch's level-1 nodes."""
    import torch

    from oracle import oracle as O
    from prysm_amd import registry as R

    n = 1_000_000
    states = _states(n, [SEED + 101, SEED + 102], gpu)
    p = R.StatePipeline(n, gpu)
    p.submit(*states[0])
    p.submit(*states[1])
    p.flush()
    p.wait()
    torch.cuda.synchronize()
    for nodes, levels, c1, sub, top in ((p.nodes[0], p.levels[0], p.c1, 512, 10),
                                        (p.bnodes[0], p.blevels[0], p.cb1, 128, 4)):
        l1 = nodes.cpu().numpy()[:32 * c1].reshape(-1, 32)
        lv = levels.cpu().numpy().reshape(-1, 32)
        nfull = c1 // sub
        offs, o = {}, 0
        for k in range(2, top + 1):
            offs[k] = o
            o += (sub >> (k - 1)) * nfull
        for b in (0, nfull // 2, nfull - 1):
            level = [bytes(x) for x in l1[sub * b:sub * b + sub]]
            for k in range(2, top + 1):
                level = [O.keccak256(level[2 * j] + level[2 * j + 1]) for j in range(len(level) // 2)]
                per = sub >> (k - 1)
                got = [bytes(x) for x in lv[offs[k] + per * b:offs[k] + per * b + per]]
                assert got == level, (sub, b, k)


def test_state_pipeline_flush_mid_stream_and_refusals(gpu):
    """A flush between submits (the next launch then has no previous state),
    roots still right; shapes the pipelined launch does not take are refused."""
    import torch

    from prysm_amd import registry as R

    n = 800_001
    states = _states(n, [SEED + 200 + t for t in range(4)], gpu)
    want = _one_state_roots(n, states, gpu)
    p = R.StatePipeline(n, gpu)
    hs = [p.submit(*states[0]), p.submit(*states[1])]
    p.flush()
    hs += [p.submit(*states[2]), p.submit(*states[3])]
    p.flush()
    p.wait()
    torch.cuda.synchronize()
    assert [bytes(h.cpu().numpy()) for h in hs] == want
    rec, bal = states[0]
    with pytest.raises(ValueError):
        p.submit(rec, torch.cat([bal, bal[:8]])[8:])  # balances 8 B off alignment
    with pytest.raises(ValueError):
        R.StatePipeline(1 << 18, gpu).submit(*_states(1 << 18, [SEED], gpu)[0])  # 1 group per workgroup


def test_state_pipeline_submits_from_two_streams(gpu):
    """Submits alternating between two current streams, and flush() from a
    third: each launch waits for the previous one's event when the stream
    changed (it reads that launch's level-1 nodes), so every root equals the
    one-state path's (no cross-stream dependency before)."""
    import torch

    from prysm_amd import registry as R

    n = 1 << 20
    states = _states(n, [SEED + 900 + t for t in range(5)], gpu)
    want = _one_state_roots(n, states, gpu)
    p = R.StatePipeline(n, gpu)
    streams = [torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu)]
    handles = []
    for t, (rec, bal) in enumerate(states):
        with torch.cuda.stream(streams[t % 2]):
            handles.append(p.submit(rec, bal))
    with torch.cuda.stream(streams[2]):
        p.flush()
        p.wait()
    torch.cuda.synchronize()
    # roots stay valid for two submits after they are produced: read the last three
    got = [bytes(h.cpu().numpy()) for h in handles[-3:]]
    assert got == want[-3:]
