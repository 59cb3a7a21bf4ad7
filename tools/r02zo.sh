#!/bin/bash
# r02zo: MK_ROUND_UNROLL 1 vs 2 (default) confirmation on another box: leaf
# A/B at 2^25/2^26/2^28 and the C2 / C3 / C5 bench lines with each library
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02zo
mkdir -p $O
for n in 25 26 25 28; do
  timeout -k 10 300 python tools/ab_leaf.py --log2n $n --rounds 9 main u1 > $O/ab.tmp 2>&1 || { cat $O/ab.tmp; exit 1; }
  grep variant $O/ab.tmp | cut -c1-150 | tee -a $O/ab.txt
done
for rep in 1 2; do
  for lib in main u1; do
    if [ $lib = main ]; then L=""; else L=prysm_amd/lib/variants/libprysm_merkle_$lib.so; fi
    for c in c2 c3 c5; do
      PRYSM_MERKLE_LIB=$L timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
      python3 -c "import json,sys; b=json.loads(open('$O/$c.json').readline()); print('$rep $lib $c', round(b['ms_per_step'],4))" | tee -a $O/configs.txt
    done
  done
done
