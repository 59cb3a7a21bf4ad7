#!/bin/bash
# rocprofv3 evidence (kernel stats + separate PMC passes, tools/profile.sh)
# for the side configs' dominant kernels: C2 k_keccak64, C3 k_struct_reg,
# C5 k_keccak_rec.  Stops at the first failing step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "c2|k_keccak64" "c3|k_struct_reg<3, 6>" "c5|k_keccak_rec<35>"; do
  cfg=${spec%%|*}; kern=${spec#*|}
  TAG=$cfg PROF_ARGS="--config $cfg --steps 10 --warmup 20 --no-cpu-baseline" KERNEL="$kern" \
    bash tools/profile.sh > gpurun_out/profile_$cfg.txt 2>&1 || { echo "$cfg failed"; exit 1; }
  echo "$cfg ok"
done
