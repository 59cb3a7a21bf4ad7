#!/bin/bash
# C3 A/B over registry.DeviceStateHasher schedules (level1 = default, list, two = round 3), alternating processes
set -u
cd "${GRAFT_REPO_ROOT:-.}"
O=gpurun_out/$1
mkdir -p $O
for r in 1 2 3; do
  for f in ${SCHEDS:-level1 list two}; do
    PRYSM_C3_SCHED=$f timeout -k 10 200 python bench.py --config c3 --steps ${STEPS:-100} --warmup 20 --no-cpu-baseline > $O/c3_f${f}_$r.json 2> $O/c3_f${f}_$r.err || { tail -5 $O/c3_f${f}_$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('schedule', sys.argv[2], 'round', sys.argv[3], round(d['ms_per_step'], 4))" $O/c3_f${f}_$r.json $f $r | tee -a $O/summary.txt
  done
done
