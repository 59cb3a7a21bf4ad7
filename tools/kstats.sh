#!/bin/bash
# rocprofv3 kernel-trace stats of one tools/ab_leaf.py invocation per variant:
#   bash tools/kstats.sh TAG "AB_ARGS" VARIANT [VARIANT ...]
# -> gpurun_out/TAG/<variant>_kernel_stats.csv (one process per variant)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; ARGS=$2; shift 2
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof_$v -o run --output-format csv -- \
    python3 tools/ab_leaf.py $ARGS --rounds 5 $v > gpurun_out/$TAG/ks_$v.log 2>&1 || { tail -5 gpurun_out/$TAG/ks_$v.log; exit 1; }
  f=$(find gpurun_out/$TAG/prof_$v -name '*kernel_stats.csv' | head -1)
  cp "$f" gpurun_out/$TAG/${v}_kernel_stats.csv
  echo "== $v"; cut -d, -f1-4 gpurun_out/$TAG/${v}_kernel_stats.csv | head -8
done
