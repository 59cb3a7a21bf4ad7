#!/bin/bash
# End-of-round evidence on one GPU: parity tests, smoke, every BASELINE config's
# bench line, and the rocprofv3 profile of the headline (tools/profile.sh).
# Each GPU step has its own time limit; any failure ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01c}
O=gpurun_out/final_$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -20 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
for c in c4 c1 c2 c3 c5; do
  timeout -k 10 400 python bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || { tail -5 $O/bench_$c.err; exit 1; }
  cat $O/bench_$c.json
done
TAG=$TAG bash tools/profile.sh > $O/profile.log 2>&1 || { tail -5 $O/profile.log; exit 1; }
cp gpurun_out/prof_$TAG/summary.json $O/pmc_summary.json
echo done
