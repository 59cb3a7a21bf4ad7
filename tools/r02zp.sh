#!/bin/bash
# r02zp: the 8-GPU decomposition on the final leaf form: 8 gloo ranks sharing
# one GPU (root must equal the golden 2^28 root) and one rank's pipelined
# 2^25 step emulated without the collective (2 and 3 buffer sets)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02zp
mkdir -p $O
bash tools/rehearse8.sh > $O/rehearse8.log 2>&1 || { tail -20 $O/rehearse8.log; exit 1; }
cp gpurun_out/rehearse8_summary.json $O/
for w in 8 4 2; do
  for sl in 2 3; do
    timeout -k 10 200 python tools/rank_step_probe.py --log2n 25 --world $w --slots $sl > $O/rank_step_w${w}_s$sl.txt 2>&1 || { tail -5 $O/rank_step_w${w}_s$sl.txt; exit 1; }
    tail -1 $O/rank_step_w${w}_s$sl.txt
  done
done
