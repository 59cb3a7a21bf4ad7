"""ASan/UBSan build of the host planner (SURVEY.md §5 sanitizers): the pass
planner, shard plan, many-lists plan and trie layout (prysm_amd/csrc/planner.cpp,
plain C++) built host-only with -fsanitize=address,undefined and fuzzed by
tests/c_abi/planner_fuzz.cpp; its shard plans and frontier sizes are checked
against the Python restatements."""
import os
import subprocess

import pytest

from prysm_amd import parallel as P
from tests.test_distributed import _plan_cpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# the default build, and one with the phase-locked leaf pass (k_leaf_lock_sc)
# enabled down to 2^12 windows so the fuzz sizes reach it (-Werror: an
# override the source ignores, a redefined macro, fails the build)
@pytest.fixture(scope="module", params=[(), ("-DMK_LEAF_LOCK=1", "-DMK_LEAF_LOCK_MIN_LOG2=12")],
                ids=["default", "leaf_lock"])
def fuzz_exe(tmp_path_factory, request):
    out = str(tmp_path_factory.mktemp("fuzz") / ("planner_fuzz_" + ("leaf_lock" if request.param else "default")))
    csrc = os.path.join(ROOT, "prysm_amd", "csrc")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-fno-omit-frame-pointer", "-Werror", *request.param, "-I" + csrc, "-I" + os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c_abi", "planner_fuzz.cpp"), os.path.join(csrc, "planner.cpp"),
                    "-o", out], check=True)
    return out


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_planner_fuzz_sanitized(fuzz_exe, seed):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([fuzz_exe, str(seed), "400"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    assert "cases clean" in r.stderr
    if "leaf_lock" in fuzz_exe:
        assert " 0 phase-locked" not in r.stderr, r.stderr[-300:]
    assert " 0 node passes" not in r.stderr, r.stderr[-300:]  # the wide k_node_lock plans
    nshard = nfront = 0
    for line in r.stdout.splitlines():
        f = line.split()
        if f[0] == "S":
            n, il, world, h, ne = map(int, f[1:6])
            begin = list(map(int, f[6:]))
            ph, pne, pbegin = _plan_cpu(n, il, world)
            assert (ne, begin) == (pne, pbegin), line
            if pne > 1:
                assert h == ph, line
            nshard += 1
        elif f[0] == "F":
            sn, il, h, k, nodes = map(int, f[1:])
            assert nodes == P.frontier_count(sn, il, h, k), line
            nfront += 1
    assert nshard == 400 and nfront > 100
