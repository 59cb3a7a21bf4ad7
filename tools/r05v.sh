# k_node_lock: parity (new node-lock tests + the 2^28 full-size root), a
# one-process A/B against the k_reduce node pass (variant nonl), a bench line.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_node_lock.py tests/test_gpu_full_size.py -k "node or c4_full" -x -v --timeout 300 --timeout-method thread > gpurun_out/r05v_pytest.log 2>&1; rc=$?; tail -12 gpurun_out/r05v_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab_leaf.py --log2n 28 --rounds 9 main nonl > gpurun_out/r05v_ab.txt 2>&1; rc=$?; tail -8 gpurun_out/r05v_ab.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-side-configs > gpurun_out/r05v_bench.json 2> gpurun_out/r05v_bench.err; rc=$?; python3 -c "import json; d=json.load(open('gpurun_out/r05v_bench.json')); print(d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['step_frac_aggregate'], d['config']['root_matches_golden'])"; exit $rc
