#!/bin/bash
# r02zh: final-tree evidence with the 6-wave split leaf form as the default
# (tools/final_runs.sh) plus the trace-vs-hipEvent leaf timing check
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r02zh bash tools/final_runs.sh || exit 1
python tools/leaf_agreement.py gpurun_out/prof_r02zh > gpurun_out/final_r02zh/c4_leaf_timing_agreement.json
