#!/bin/bash
# r02g: leaf-pass NI threshold A/B at the per-GPU tree sizes of 1/2/4/8 GPUs,
# then the first RCCL execution: 2 ranks sharing cuda:0 over backend nccl
# (RCCL may refuse two ranks on one device; the log says which).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
for n in ${AB_SIZES:-25 26 27 28}; do
  timeout -k 10 300 python tools/ab_leaf.py --log2n $n --rounds ${AB_ROUNDS:-7} ${AB_VARIANTS:-main ni23 ni24} > $O/ab_$n.json 2>&1 || { cat $O/ab_$n.json; exit 1; }
  tail -3 $O/ab_$n.json
done
if [ -n "${NCCL_PROBE:-1}" ]; then
  timeout -k 10 240 python bench.py --gpus 2 --share-device --backend nccl --log2n 24 --steps 3 --warmup 1 \
    --no-cpu-baseline > $O/nccl_share2.json 2> $O/nccl_share2.err; rc=$?
  tail -20 $O/nccl_share2.err; cat $O/nccl_share2.json; echo "nccl share-device rc=$rc"
fi
exit 0
