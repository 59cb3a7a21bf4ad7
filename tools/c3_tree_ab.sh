#!/bin/bash
# tools/c3_tree_probe.py per library variant (separate processes, alternating)
#   bash tools/c3_tree_ab.sh TAG ROUNDS VARIANT [VARIANT ...]   ("main" = default build)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1 ROUNDS=$2
shift 2
O=gpurun_out/$TAG
mkdir -p $O
for r in $(seq 1 $ROUNDS); do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=""; else lib=prysm_amd/lib/variants/libprysm_merkle_$v.so; fi
    PRYSM_MERKLE_LIB=$lib timeout -k 10 200 python tools/c3_tree_probe.py > $O/c3tree_${v}_$r.jsonl 2> $O/c3tree_${v}_$r.err \
      || { tail -5 $O/c3tree_${v}_$r.err; exit 1; }
    python -c "import json,sys; print(sys.argv[2], sys.argv[3], ' '.join(f\"{d['case']}={d['median_ms']}\" for d in map(json.loads, open(sys.argv[1]))))" \
      $O/c3tree_${v}_$r.jsonl $v $r | tee -a $O/summary.txt
  done
done
