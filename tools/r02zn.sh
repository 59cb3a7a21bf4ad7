#!/bin/bash
# r02zn: Keccak round unroll (MK_ROUND_UNROLL) with the spill-free split leaf
# form: 2 (default, 94 VGPRs) vs 1 (94 VGPRs) vs 4 (96 VGPRs, 16 B scratch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02zn
mkdir -p $O
for n in 25 28 25 28; do
  timeout -k 10 300 python tools/ab_leaf.py --log2n $n --rounds 9 main u1 u4 > $O/ab.tmp 2>&1 || { cat $O/ab.tmp; exit 1; }
  grep variant $O/ab.tmp | cut -c1-150 | tee -a $O/ab.txt
done
