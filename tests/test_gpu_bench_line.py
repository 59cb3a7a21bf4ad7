"""bench.py's records on the GPU: the N > 1 line is self-sufficient (two
gloo ranks sharing cuda:0: aggregate fraction, every rank's leaf fraction,
rank 0's single-GPU time and the parallel efficiency it implies), and the
N = 1 line carries every side config with its golden check.  Each runs
bench.py as a child process under its own time limit."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _line(stdout: str):
    lines = [json.loads(x) for x in stdout.splitlines() if x.startswith("{")]
    assert lines, stdout[-2000:]
    return lines[-1]


def test_bench_world2_line_is_self_sufficient():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo", "--share-device",
           "--log2n", "22", "--steps", "4", "--warmup", "2", "--no-cpu-baseline"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = _line(r.stdout)
    cfg, roof = out["config"], out["roofline"]
    assert out["n_gpus"] == 2 and cfg["world_size"] == 2
    assert 0 < roof["step_frac_aggregate"] < 1
    assert roof["tree_perms"] == 3 << 19  # 2^22 items: 2^19 windows x 2 + 2^19 - 1 nodes + 1
    assert len(cfg["per_rank_leaf_frac"]) == 2 and all(0 < f < 1 for f in cfg["per_rank_leaf_frac"])
    assert cfg["single_gpu_ms"] > 0
    assert 0 < cfg["parallel_efficiency"] <= 1.2
    assert abs(cfg["parallel_efficiency"] - cfg["single_gpu_ms"] / (2 * out["ms_per_step"])) < 1e-9


def test_bench_world1_side_configs():
    """The driver's N = 1 line at a small headline size: side_configs holds
    C2, C3, C5 and C1, each with its full-size root equal to the golden."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--log2n", "22", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--side-steps", "5", "--side-warmup", "1"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    side = _line(r.stdout)["side_configs"]
    assert set(side) == {"c1", "c2", "c3", "c5"}
    for c, e in side.items():
        assert e["root_matches_golden"] is True, (c, e)
        assert e["ms_per_step"] > 0 and 0 < e["frac"] < 1, (c, e)
    assert side["c5"]["single_trie_ms"] > 0 and side["c5"]["reference_incremental_perms"] == 35 << 20
