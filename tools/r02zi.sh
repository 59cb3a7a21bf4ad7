#!/bin/bash
# r02zi: waves per SIMD for the split leaf form: 6 (default, 80 VGPRs, 15
# dwords spilled) vs 5 (94 VGPRs, no spill) vs 7 (72 VGPRs, 54 spilled)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02zi
mkdir -p $O
for n in 25 28 25 28; do
  timeout -k 10 300 python tools/ab_leaf.py --log2n $n --rounds 9 main split5 split7 > $O/ab.tmp 2>&1 || { cat $O/ab.tmp; exit 1; }
  grep variant $O/ab.tmp | cut -c1-150 | tee -a $O/ab.txt
done
