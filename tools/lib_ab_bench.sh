#!/bin/bash
# bench.py --config CFG against library variants, alternating, in separate
# processes (each variant = prysm_amd/lib/variants/libprysm_merkle_<name>.so,
# "main" = the default build).  The first failing run ends the script.
#
#   bash tools/lib_ab_bench.sh TAG CFG ROUNDS VARIANT [VARIANT ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1 CFG=$2 ROUNDS=$3
shift 3
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=""; else lib=prysm_amd/lib/variants/libprysm_merkle_$v.so; fi
    PRYSM_MERKLE_LIB=$lib timeout -k 10 200 python bench.py --config $CFG --no-cpu-baseline \
      > $O/${CFG}_${v}_$r.json 2> $O/${CFG}_${v}_$r.err || { tail -5 $O/${CFG}_${v}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); \
print(sys.argv[2], sys.argv[3], round(d['ms_per_step'], 4), d['config'].get('single_trie_ms'))" \
      $O/${CFG}_${v}_$r.json $v $r | tee -a $O/summary.txt
  done
done
