# Fused trie top, per-level forms: parity, C5 one-trie time, top probe.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06c
timeout -k 10 300 python -u -m pytest tests/test_gpu_trie_top_fused.py tests/test_gpu_trie_lock.py tests/test_gpu_deposit_trie.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06c/pytest.log 2>&1 || { tail -30 gpurun_out/r06c/pytest.log; exit 1; }
tail -2 gpurun_out/r06c/pytest.log
timeout -k 10 200 python tools/single_probe.py c5 --steps 200 --warmup 40 > gpurun_out/r06c/single.txt 2>&1 || { tail -5 gpurun_out/r06c/single.txt; exit 1; }
cat gpurun_out/r06c/single.txt
