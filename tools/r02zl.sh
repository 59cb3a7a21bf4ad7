#!/bin/bash
# r02zl: do C2 / C3 move with the leaf form?  bench lines of C3 and C2 with
# the default (split, 5 waves), split at 6 waves and the staged form, same box,
# interleaved twice
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r02zl
mkdir -p $O
for rep in 1 2; do
  for lib in main w6 staged; do
    if [ $lib = main ]; then L=""; else L=prysm_amd/lib/variants/libprysm_merkle_$lib.so; fi
    for c in c3 c2 c5; do
      PRYSM_MERKLE_LIB=$L timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/$c.json 2> $O/$c.err || { tail -5 $O/$c.err; exit 1; }
      python3 -c "import json,sys; b=json.loads(open('$O/$c.json').readline()); print('$rep $lib $c', round(b['ms_per_step'],4))" | tee -a $O/ab.txt
    done
  done
done
