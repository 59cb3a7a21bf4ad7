# Fused list tops + rotated struct staging: parity, C3 one state fused vs
# level1 (interleaved), the C3 stream, trace of the fused form.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06e
timeout -k 10 500 python -u -m pytest tests/test_gpu_merkle_top_fused.py tests/test_gpu_trie_top_fused.py tests/test_gpu_lock.py tests/test_gpu_state.py tests/test_gpu_state_pipeline.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06e/pytest.log 2>&1 || { tail -30 gpurun_out/r06e/pytest.log; exit 1; }
tail -2 gpurun_out/r06e/pytest.log
for s in fused level1 fused level1; do
PRYSM_C3_SCHED=$s timeout -k 10 200 python tools/single_probe.py c3 --steps 200 --warmup 40 2>/dev/null | sed "s/^/$s /" || exit 1
done
timeout -k 10 300 python bench.py --config c3 --steps 200 --warmup 40 > gpurun_out/r06e/bench_c3.json 2> gpurun_out/r06e/bench_c3.err || { tail -5 gpurun_out/r06e/bench_c3.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r06e/bench_c3.json')); print('c3 stream', d['ms_per_step'], d['config'].get('single_state_ms'), d['config']['root_matches_golden'])"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06e/tr -o run --output-format csv -- python3 tools/single_probe.py c3 --steps 30 --warmup 5 > gpurun_out/r06e/tr.log 2>&1 || { tail -5 gpurun_out/r06e/tr.log; exit 1; }
echo done
