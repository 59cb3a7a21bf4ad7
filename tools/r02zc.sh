#!/bin/bash
# r02zc: plain (L2-allocating) vs non-temporal loads -- all configs' A/B and
# the leaf kernel's HBM fetch for each (one FETCH_SIZE pass per library)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02zc
mkdir -p $O
for args in "--log2n 28" "--log2n 25" "--c2 --log2n 24" "--trie --log2n 20" "--struct"; do
  timeout -k 10 300 python tools/ab_leaf.py $args --rounds 9 main plainld > $O/ab.tmp 2>&1 || { cat $O/ab.tmp; exit 1; }
  grep variant $O/ab.tmp | sed "s/^/[$args] /" | tee -a $O/ab.txt | cut -c1-150
done
for lib in main plainld; do
  if [ $lib = main ]; then L=""; else L=prysm_amd/lib/variants/libprysm_merkle_$lib.so; fi
  PRYSM_MERKLE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch_$lib -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/fetch_$lib.log 2>&1 || { tail -5 $O/fetch_$lib.log; exit 1; }
  python3 - $O/fetch_$lib $lib <<'PY'
import csv, glob, sys
vals = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void mk::k_reduce<true, true, 2>") and r["Counter_Name"] == "FETCH_SIZE":
            vals.append(float(r["Counter_Value"]))
# FETCH_SIZE in KiB, x2 gfx950 correction (MI355X_MICROARCH.md), per dispatch
print(sys.argv[2], "leaf FETCH GB/launch (x2 corrected):", round(sum(vals) / len(vals) * 1024 * 2 / 1e9, 3), "dispatches", len(vals))
PY
done
