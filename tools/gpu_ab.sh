#!/bin/bash
# GPU parity tests, then an in-process A/B of library variants at several sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for n in ${AB_SIZES:-25 28}; do
  timeout -k 10 300 python tools/ab_leaf.py --log2n $n --rounds ${AB_ROUNDS:-7} ${AB_VARIANTS:-main} > gpurun_out/ab_$n.json 2>&1 || { cat gpurun_out/ab_$n.json; exit 1; }
  cat gpurun_out/ab_$n.json
done
for n in ${AB_TRIE_SIZES:-}; do
  timeout -k 10 300 python tools/ab_leaf.py --trie --log2n $n --rounds ${AB_ROUNDS:-7} ${AB_VARIANTS:-main} > gpurun_out/ab_trie_$n.json 2>&1 || { cat gpurun_out/ab_trie_$n.json; exit 1; }
  cat gpurun_out/ab_trie_$n.json
done
