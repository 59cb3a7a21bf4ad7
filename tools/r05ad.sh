export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_node_lock.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05ad.log 2>&1; rc=$?; tail -14 gpurun_out/r05ad.log; exit $rc
