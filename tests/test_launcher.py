"""bench.py's self-launch (CPU, gloo): `launch_ranks(N, ...)` starts N ranks
of one node through torch.distributed.run in a child process; the 8-rank
frontier-sharded root equals the 1-rank root and the oracle's root."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SEED = 0x5EED000000000000 + 88


@pytest.mark.parametrize("nproc", [1, 8])
def test_launch_ranks_roots_agree(nproc, tmp_path, monkeypatch):
    from oracle import oracle as O

    n, k = 4 * 4096 + 3, 3
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch_ranks(%d, [%r, %r, %r], script=%r))"
            % (ROOT, nproc, str(n), str(SEED), str(k), os.path.join(ROOT, "tests", "rank_probe.py")))
    env = {kk: v for kk, v in os.environ.items() if kk not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["world"] == nproc
    assert bytes.fromhex(lines[0]["root"]) == O.merkle_hash_gen(n, 32, SEED)


def test_bench_refuses_world_mismatch(monkeypatch):
    """Launched externally with WORLD_SIZE != --gpus, bench.py fails loudly
    instead of measuring a different GPU count."""
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--no-cpu-baseline"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 2 and "WORLD_SIZE 2" in r.stderr


def test_bench_rank_that_never_joins_fails_fast():
    """An N-rank run whose peer never joins ends within the process-group
    timeout (PRYSM_DIST_TIMEOUT) with an error JSON line and a non-zero
    status, instead of hanging for torch's 10-minute default: rank 0 of a
    world-2 gloo run started alone."""
    import socket
    import time

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), PRYSM_DIST_TIMEOUT="6")
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=120, env=env)
    dt = time.time() - t0
    assert r.returncode != 0 and dt < 60, (r.returncode, dt, r.stderr[-2000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["value"] is None and lines[0]["world_size"] == 2
    assert lines[0]["backend"] == "gloo" and lines[0]["error"]


def test_bench_deadline_ends_a_hung_rank():
    """The host-side deadline (PRYSM_BENCH_DEADLINE) ends a rank stuck
    longer than every timeout with status 124 and the error line."""
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), PRYSM_DIST_TIMEOUT="100", PRYSM_BENCH_DEADLINE="5")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--no-cpu-baseline"], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and "deadline" in lines[0]["error"]
