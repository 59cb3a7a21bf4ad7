#!/bin/bash
# r02zm: split leaf form with line 0 of each window read non-temporally
# (MK_LEAF_NT_LINE0=1, so L2 keeps line 1 for block 2) vs plain loads:
# A/B at 2^25..2^28 and the leaf FETCH/WRITE per launch
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02zm
mkdir -p $O
for n in 25 26 27 28 28; do
  timeout -k 10 300 python tools/ab_leaf.py --log2n $n --rounds 9 main nt0 > $O/ab.tmp 2>&1 || { cat $O/ab.tmp; exit 1; }
  grep variant $O/ab.tmp | cut -c1-150 | tee -a $O/ab.txt
done
for lib in main nt0; do
  if [ $lib = main ]; then L=""; else L=prysm_amd/lib/variants/libprysm_merkle_$lib.so; fi
  for ctr in FETCH_SIZE WRITE_SIZE; do
    PRYSM_MERKLE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $ctr -d $O/${ctr}_$lib -o run --output-format csv -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/${ctr}_$lib.log 2>&1 || { tail -5 $O/${ctr}_$lib.log; exit 1; }
    python3 - $O/${ctr}_$lib $lib $ctr <<'PY' | tee -a $O/pmc.txt
import csv, glob, sys
vals = []
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith("void mk::k_reduce<true, true, 2>") and r["Counter_Name"] == sys.argv[3]:
            vals.append(float(r["Counter_Value"]))
mult = 2 if sys.argv[3] == "FETCH_SIZE" else 1  # gfx950 FETCH_SIZE x2 correction (MI355X_MICROARCH.md)
print(sys.argv[2], sys.argv[3], "GB/launch:", round(sum(vals) / len(vals) * 1024 * mult / 1e9, 3), "dispatches", len(vals))
PY
  done
done
