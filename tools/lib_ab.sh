#!/bin/bash
# Whole-bench A/B of library variants (prysm_amd/lib/variants/libprysm_merkle_<name>.so,
# `make variant`) through PRYSM_MERKLE_LIB, alternating processes:
#   bash tools/lib_ab.sh TAG CONFIG "main nw128 nw64" [ROUNDS] [EXTRA bench args]
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$1; CFG=$2; VARS=$3; R=${4:-3}; EXTRA=${5:-}
mkdir -p $O
for r in $(seq 1 $R); do
  for v in $VARS; do
    if [ "$v" = main ]; then L=prysm_amd/lib/libprysm_merkle.so; else L=prysm_amd/lib/variants/libprysm_merkle_$v.so; fi
    PRYSM_MERKLE_LIB=$L timeout -k 10 300 python bench.py --config $CFG --no-cpu-baseline $EXTRA > $O/${CFG}_${v}_$r.json 2> $O/${CFG}_${v}_$r.err || { tail -5 $O/${CFG}_${v}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], 'round', sys.argv[4], round(d['ms_per_step'], 4))" $O/${CFG}_${v}_$r.json $CFG $v $r | tee -a $O/summary.txt
  done
done
