# Round-5 end: the N = 1 bench line with the one-stream default, its bench-line
# tests, and the rocprofv3 kernel-trace + PMC passes of the same step.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_line.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05t_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05t_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_r05t.json 2> gpurun_out/bench_r05t.err; rc=$?; echo bench rc=$rc; [ $rc -ne 0 ] && exit $rc
TAG=r05t_c4 PROF_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-side-configs" bash tools/profile.sh > gpurun_out/r05t_prof.log 2>&1; echo prof rc=$?
