#!/bin/bash
# rocprofv3 evidence for the bench kernel: kernel-trace stats + separate PMC
# passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950; counters
# never combined with tracing domains).  Outputs under gpurun_out/prof_<tag>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
ARGS=${PROF_ARGS:---steps 10 --warmup 20 --no-cpu-baseline}  # the default bench line's steps and warmup
D=gpurun_out/prof_$TAG
mkdir -p $D
run() {  # name, rocprofv3 options...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 "$@" -d $D/$name -o run --output-format csv -- python3 bench.py $ARGS > $D/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run stats --kernel-trace --stats || exit $?
run fetch --pmc FETCH_SIZE || exit $?
run write --pmc WRITE_SIZE || exit $?
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
run lds --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CU_CYCLES SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES || exit $?
python3 tools/pmc_summary.py $D > $D/summary.json && cat $D/summary.json
