#!/bin/bash
# One GPU-box session: parity tests, smoke, bench.  Each GPU step has its own
# time limit; a crash/timeout/fault (exit >= 124 or signal) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
STEPS="${STEPS:-tests smoke bench}"
fatal() { local rc=$1; [ "$rc" -ge 124 ] || [ "$rc" -eq 134 ] || [ "$rc" -eq 139 ]; }
(rocminfo 2>/dev/null | grep -E "Marketing Name|gfx9|Compute Unit|Max Clock" | head -12; lscpu | grep -E "Model name|^CPU\(s\)") > $OUT/machine.txt 2>&1
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 ${TEST_TIMEOUT:-600} python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; rc=$?
      tail -30 $OUT/pytest_gpu.log; echo "pytest rc=$rc"; fatal $rc && exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
      tail -5 $OUT/smoke.log; echo "smoke rc=$rc"; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      timeout -k 10 ${BENCH_TIMEOUT:-600} python bench.py ${BENCH_ARGS:-} > $OUT/bench.json 2> $OUT/bench.err; rc=$?
      cat $OUT/bench.json; tail -5 $OUT/bench.err; echo "bench rc=$rc"; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc ;;
    multirank)
      # the N-rank path (sharding, all-gather, rank-0 finish on a side stream)
      # rehearsed with 2 and 4 ranks sharing cuda:0 over gloo; the root must
      # equal the single-rank root of the same tree
      for w in 2 4; do
        timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $w --master-addr 127.0.0.1 \
          --master-port $((29500 + w)) bench.py --gpus $w --backend gloo --share-device --log2n ${MR_LOG2N:-24} \
          --steps 3 --warmup 1 --no-cpu-baseline > $OUT/multirank_$w.json 2> $OUT/multirank_$w.err; rc=$?
        tail -3 $OUT/multirank_$w.err; cat $OUT/multirank_$w.json; echo "multirank $w rc=$rc"; fatal $rc && exit $rc; [ $rc -ne 0 ] && exit $rc
      done
      timeout -k 10 300 python bench.py --log2n ${MR_LOG2N:-24} --steps 3 --warmup 1 --no-cpu-baseline > $OUT/multirank_1.json 2>/dev/null || exit 1
      python - $OUT <<'PY' || exit 1
import json, sys
def root(w):  # the JSON line (gloo also prints connection notes to stdout)
    line = [l for l in open(f"{sys.argv[1]}/multirank_{w}.json") if l.startswith("{")][-1]
    return json.loads(line)["config"]["root"]
roots = {w: root(w) for w in (1, 2, 4)}
print("multirank roots", roots)
assert len(set(roots.values())) == 1, roots
PY
      ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py ${PROF_ARGS:---steps 5 --warmup 2 --no-cpu-baseline} > $OUT/prof.log 2>&1; rc=$?
      tail -5 $OUT/prof.log; echo "prof rc=$rc"; fatal $rc && exit $rc ;;
  esac
done
exit 0
