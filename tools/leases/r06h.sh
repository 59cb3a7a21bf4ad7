# wg_level: the padded parent in spread form beside the lane/pair forms.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06h
timeout -k 10 400 python -u -m pytest tests/test_gpu_merkle_top_fused.py tests/test_gpu_trie_top_fused.py tests/test_gpu_lock.py::test_state_hasher_schedules_agree tests/test_gpu_state.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06h/pytest.log 2>&1 || { tail -30 gpurun_out/r06h/pytest.log; exit 1; }
tail -1 gpurun_out/r06h/pytest.log
timeout -k 5 60 tools/top_probe 5 merkle || exit 1
for c in c3 c5 c3 c5; do timeout -k 10 200 python tools/single_probe.py $c --steps 200 --warmup 40 2>/dev/null || exit 1; done
