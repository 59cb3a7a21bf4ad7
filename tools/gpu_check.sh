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
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py ${PROF_ARGS:---steps 5 --warmup 2 --no-cpu-baseline} > $OUT/prof.log 2>&1; rc=$?
      tail -5 $OUT/prof.log; echo "prof rc=$rc"; fatal $rc && exit $rc ;;
  esac
done
exit 0
