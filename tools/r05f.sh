export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_state_pipeline.py tests/test_gpu_lock.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05f_sp.log 2>&1; rc=$?; tail -3 gpurun_out/r05f_sp.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2 3; do timeout -k 10 120 python bench.py --config c3 --steps 200 --warmup 40 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['ms_per_step'], d['config']['single_state_ms'], d['config']['root_matches_golden'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05f_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r05f_c3.log 2>&1; echo prof c3 rc=$?
