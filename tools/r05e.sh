export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_lock.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05e_lock.log 2>&1; rc=$?; tail -3 gpurun_out/r05e_lock.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r05_c3.log 2>&1; echo prof c3 rc=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_c5 -o run --output-format csv -- python3 bench.py --config c5 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r05_c5.log 2>&1; echo prof c5 rc=$?
