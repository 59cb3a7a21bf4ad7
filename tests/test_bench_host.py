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
