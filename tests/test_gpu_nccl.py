"""The RCCL path on hardware as far as one GPU allows: a
world-1 "nccl" process group runs rank 0's frontier all-gather and finisher
on a high-priority side stream (tests/nccl_world1.py, its own process so the
process group never touches the other tests).  RCCL refuses two ranks on one
device, so world > 1 over nccl needs the driver's multi-GPU node."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("log2n,k", [(20, 10), (16, 3)])
def test_rccl_world1_frontier_gather(log2n, k):
    out = _run([str(log2n), str(k)])
    assert out["root"] == [out["want"]] * 2, out


@pytest.mark.parametrize("log2n,extra", [(20, 0), (18, 12_345)])
def test_library_rccl_one_device(log2n, extra):
    """The library's ncclCommInitAll + in-place ncclAllGather (forced onto one
    device by the MK_FORCE_COLLECTIVE test hook), device and host forms."""
    out = _run(["lib", str(log2n), str(extra)], MK_FORCE_COLLECTIVE="1")
    assert out["root"] == [out["want"]] * 3, out


def _run(args, **extra_env):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0", **extra_env)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "nccl_world1.py")] + args,
                       env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
