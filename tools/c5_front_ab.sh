#!/bin/bash
# C5 A/B: TriePipeline front "pipe" (the previous trie's levels 3-7 in the
# locked front's slots) vs "split" (free-running front), alternating processes
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$1
mkdir -p $O
for r in 1 2 3; do
  for f in auto split; do
    PRYSM_C5_FRONT=$f timeout -k 10 200 python bench.py --config c5 --steps ${STEPS:-100} --warmup 20 --no-cpu-baseline > $O/c5_${f}_$r.json 2> $O/c5_${f}_$r.err || { tail -5 $O/c5_${f}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('front', d['config']['front'], 'round', sys.argv[2], round(d['ms_per_step'], 4), 'single', round(d['config']['single_trie_ms'], 4))" $O/c5_${f}_$r.json $r | tee -a $O/summary.txt
  done
done
