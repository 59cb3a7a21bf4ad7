# k_node_lock under rocprofv3: kernel-trace stats of the default bench step and
# one SQ/GRBM counter pass (separate runs).
export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=r05w_c4 PROF_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-side-configs" bash tools/profile.sh > gpurun_out/r05w_prof.log 2>&1; echo prof rc=$?
