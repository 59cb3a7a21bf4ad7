export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r05o.json 2> gpurun_out/bench_r05o.err; rc=$?; echo bench rc=$rc; [ $rc -ne 0 ] && exit $rc
TAG=r05_c4 PROF_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-side-configs" bash tools/profile.sh > gpurun_out/r05o_prof.log 2>&1; echo prof rc=$?
