#!/bin/bash
# r02m: k_keccak_rec at 5 waves/SIMD (96 VGPRs, 4 dwords spilled) vs 4 (100 VGPRs)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02m
mkdir -p $O
V=prysm_amd/lib/variants
timeout -k 10 300 python tools/ab_leaf.py --trie --log2n 20 --rounds 9 main ${VAR:-rec5} > $O/ab_trie.json 2>&1 || { cat $O/ab_trie.json; exit 1; }
cat $O/ab_trie.json
for rep in 1 2; do
  for lib in main ${VAR:-rec5}; do
    if [ $lib = main ]; then L=""; else L=$V/libprysm_merkle_$lib.so; fi
    PRYSM_MERKLE_LIB=$L timeout -k 10 200 python bench.py --config c5 --no-cpu-baseline > $O/c5_$lib.json 2> $O/c5_$lib.err || { tail -5 $O/c5_$lib.err; exit 1; }
    python -c "import json; d=json.load(open('$O/c5_$lib.json')); print('$lib', d['ms_per_step'], d['config'].get('single_trie_ms'), d['config']['root'][:16])" | tee -a $O/c5_ab.txt
  done
done
