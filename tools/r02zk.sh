#!/bin/bash
# r02zk: final-tree evidence with the spill-free 5-wave split leaf form as the default
# (tools/final_runs.sh) plus the trace-vs-hipEvent leaf timing check
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r02zk bash tools/final_runs.sh || exit 1
python tools/leaf_agreement.py gpurun_out/prof_r02zk > gpurun_out/final_r02zk/c4_leaf_timing_agreement.json
