#!/bin/bash
# FETCH_SIZE + GRBM_GUI_ACTIVE of the C4 leaf kernel for library variants
# (one tools/ab_leaf.py process per variant under rocprofv3 --pmc):
#   bash tools/pmc_variant.sh TAG LOG2N KERNEL_SUBSTR VARIANT [VARIANT ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; L=$2; K=$3; shift 3
mkdir -p gpurun_out/$TAG
for v in "$@"; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d gpurun_out/$TAG/pmc_$v -o run --output-format csv -- \
    python3 tools/ab_leaf.py --log2n $L --rounds 2 $v > gpurun_out/$TAG/pmc_$v.log 2>&1 || { tail -5 gpurun_out/$TAG/pmc_$v.log; exit 1; }
  python3 - gpurun_out/$TAG/pmc_$v "$K" "$v" <<'PY'
import csv, glob, sys, collections
d, k, v = sys.argv[1:4]
acc = collections.defaultdict(list)
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if k in r["Kernel_Name"]:
            acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
per = collections.defaultdict(list)
for (disp, c), vals in acc.items():
    per[c].append(sum(vals))
fetch = sum(per["FETCH_SIZE"]) / len(per["FETCH_SIZE"]) * 1024 * 2
print(f'{{"variant": "{v}", "kernel": "{k}", "dispatches": {len(per["FETCH_SIZE"])}, "fetch_GB_corrected": {fetch/1e9:.3f}, "grbm_gui_active": {sum(per["GRBM_GUI_ACTIVE"])/len(per["GRBM_GUI_ACTIVE"]):.4g}}}')
PY
done
