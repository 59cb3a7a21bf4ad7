#!/bin/bash
# r02j: does side-stream work hide under the next leaf pass?  Per-rank step
# probe (tools/rank_step_probe.py) at the per-GPU shard sizes of 2/4/8 GPUs,
# main library vs the capped-workgroup variant, alternating; then the N=1
# bench line with each library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02j
mkdir -p $O
V=prysm_amd/lib/variants
for rep in 1 2; do
  for cfg in "25 8" "26 4" "27 2"; do
    set -- $cfg
    for lib in main ${VARIANTS:-cap256}; do
      if [ $lib = main ]; then L=""; else L=$V/libprysm_merkle_$lib.so; fi
      PRYSM_MERKLE_LIB=$L timeout -k 10 120 python tools/rank_step_probe.py --log2n $1 --world $2 >> $O/rank_step.jsonl 2>> $O/rank_step.err || { tail -5 $O/rank_step.err; exit 1; }
    done
  done
done
cat $O/rank_step.jsonl
for lib in main ${VARIANTS:-cap256}; do
  if [ $lib = main ]; then L=""; else L=$V/libprysm_merkle_$lib.so; fi
  PRYSM_MERKLE_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_$lib.json 2> $O/bench_$lib.err || { tail -5 $O/bench_$lib.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/bench_$lib.json')); print('$lib', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['root_matches_golden'])"
done
