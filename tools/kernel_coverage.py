"""Which kernels compiled into libprysm_merkle.so did a traced run launch?

  python tools/kernel_coverage.py ROCPROF_DIR [LIB] > coverage.json

ROCPROF_DIR: the -d directory of `rocprofv3 --kernel-trace --stats -- python
-m pytest tests -m gpu` (its *kernel_stats.csv); LIB: the library (default the
in-tree build).  Kernel names are compared up to their argument list (the
demangled form rocprofv3 and `nm -C` share)."""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def base(name: str) -> str:
    name = name.strip().strip('"')
    if name.startswith("void "):
        name = name[5:]
    return name.split("(", 1)[0].strip()


def main():
    d = sys.argv[1]
    lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "prysm_amd", "lib", "libprysm_merkle.so")
    nm = subprocess.run(["nm", "-C", lib], capture_output=True, text=True, check=True).stdout
    compiled = sorted({base(line.split(" ", 2)[2]) for line in nm.splitlines()
                       if len(line.split(" ", 2)) == 3 and " mk::k_" in " " + line.split(" ", 2)[2]})
    ran = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ran[base(r["Name"])] = ran.get(base(r["Name"]), 0) + int(r["Calls"])
    out = {"compiled": len(compiled), "launched": sorted(k for k in compiled if k in ran),
           "never_launched": [k for k in compiled if k not in ran],
           "calls": {k: ran[k] for k in compiled if k in ran}}
    print(json.dumps(out, indent=1))
    return 1 if out["never_launched"] else 0


if __name__ == "__main__":
    sys.exit(main())
