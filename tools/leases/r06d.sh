# Fused list tops: parity, the state suites, the C3 one-state time and trace.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06d
timeout -k 10 400 python -u -m pytest tests/test_gpu_merkle_top_fused.py tests/test_gpu_lock.py tests/test_gpu_state.py tests/test_gpu_state_pipeline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06d/pytest.log 2>&1 || { tail -30 gpurun_out/r06d/pytest.log; exit 1; }
tail -2 gpurun_out/r06d/pytest.log
timeout -k 10 200 python tools/single_probe.py c3 --steps 200 --warmup 40 > gpurun_out/r06d/single.txt 2>&1 || { tail -5 gpurun_out/r06d/single.txt; exit 1; }
PRYSM_C3_SCHED=level1 timeout -k 10 200 python tools/single_probe.py c3 --steps 200 --warmup 40 >> gpurun_out/r06d/single.txt 2>&1 || { tail -5 gpurun_out/r06d/single.txt; exit 1; }
cat gpurun_out/r06d/single.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06d/tr -o run --output-format csv -- python3 tools/single_probe.py c3 --steps 30 --warmup 5 > gpurun_out/r06d/tr.log 2>&1 || { tail -5 gpurun_out/r06d/tr.log; exit 1; }
echo done
