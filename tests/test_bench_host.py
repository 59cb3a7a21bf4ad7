"""Host-side pieces of bench.py that need no GPU: the sysfs clock parser
the live clock sample relies on, and the golden-root lookup."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_sclk_parser(tmp_path):
    f = tmp_path / "pp_dpm_sclk"
    f.write_text("0: 500Mhz\n1: 2246Mhz *\n2: 2400Mhz\n")
    assert bench.ClockSampler._read(str(f)) == 2246.0
    f.write_text("S: 114Mhz *\n0: 500Mhz\n1: 2400Mhz\n")  # the idle form seen on other cards
    assert bench.ClockSampler._read(str(f)) == 114.0
    f.write_text("0: 500Mhz\n1: 2400Mhz\n")  # no current level marked
    assert bench.ClockSampler._read(str(f)) is None
    assert bench.ClockSampler._read(str(tmp_path / "missing")) is None


def test_golden_root_lookup():
    assert bench.golden_root(28, 32) == "54a62269279a90e4bda5a9da4b5bb0d5f3126bb3aacb1456cc0b0e47b9f50ba9"
    assert bench.golden_root(24, 32) is None


def test_tree_work_counts():
    """bench.tree_work: permutations and hashes of merkleHash (hash.go:194-
    239), used for the N-GPU line's aggregate fraction: the SURVEY §8d C4
    count, the small shapes by a literal level-by-level walk."""
    assert bench.tree_work(1 << 28, 32) == (100_663_296, 1 << 26)

    def walk(n, s):
        perms_of = lambda m: m // 136 + 1  # noqa: E731
        if n == 0:
            return perms_of(128 + 32), 1
        cb = (128 // s) * s if s < 128 else s
        data = n * s
        chunks = [min(cb, data - o) for o in range(0, data, cb)]
        if len(chunks) == 1:
            return perms_of(chunks[0] + 32), 1
        perms = hashes = 0
        level = chunks
        while len(level) > 1:
            if len(level) % 2:
                level = level + [128]
            level = [perms_of(level[i] + level[i + 1]) for i in range(0, len(level), 2)]
            perms += sum(level)
            hashes += len(level)
            level = [32] * len(level)
        return perms + 1, hashes + 1

    for s in (1, 3, 8, 32, 48, 128, 200):
        for n in list(range(0, 70)) + [255, 256, 257, 1000, 4099]:
            assert bench.tree_work(n, s) == walk(n, s), (n, s)
