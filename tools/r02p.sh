#!/bin/bash
# r02p: fused trie front (k_trie_front3) -- parity tests of the deposit trie,
# then one-process A/B against the three one-level launches and the C5 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_deposit_trie.py tests/test_gpu_full_size.py tests/test_gpu_fuzz.py -x -q --timeout 200 --timeout-method thread -k "trie or deposit or c5" > $O/pytest_trie.log 2>&1; rc=$?
tail -3 $O/pytest_trie.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab_leaf.py --trie --log2n 20 --rounds 9 main nofront3 > $O/ab_trie.json 2>&1 || { cat $O/ab_trie.json; exit 1; }
cat $O/ab_trie.json
for rep in 1 2; do
  for lib in main nofront3; do
    if [ $lib = main ]; then L=""; else L=prysm_amd/lib/variants/libprysm_merkle_$lib.so; fi
    PRYSM_MERKLE_LIB=$L timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > $O/c5_$lib.json 2> $O/c5_$lib.err || { tail -5 $O/c5_$lib.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c5_$lib.json')); print('$lib', d['ms_per_step'], d['config'].get('single_trie_ms'), d['config']['root'][:16])" | tee -a $O/c5_ab.txt
  done
done
