#!/bin/bash
# r02k: per-rank step probe, 2 vs 3 buffer sets (side work of the step two
# vs three back must be done before a leaf pass starts)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02k
mkdir -p $O
for rep in 1 2; do
  for cfg in "25 8" "26 4" "27 2" "28 1"; do
    set -- $cfg
    for slots in 2 3; do
      timeout -k 10 150 python tools/rank_step_probe.py --log2n $1 --world $2 --slots $slots >> $O/rank_step_slots.jsonl 2>> $O/rank_step.err || { tail -5 $O/rank_step.err; exit 1; }
    done
  done
done
cat $O/rank_step_slots.jsonl
