# Fused trie top: parity (every level), the trie suites, then the C5 one-trie
# time and its kernel trace.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06b
timeout -k 10 300 python -u -m pytest tests/test_gpu_trie_top_fused.py tests/test_gpu_trie_lock.py tests/test_gpu_deposit_trie.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06b/pytest.log 2>&1 || { tail -30 gpurun_out/r06b/pytest.log; exit 1; }
tail -2 gpurun_out/r06b/pytest.log
timeout -k 10 200 python tools/single_probe.py c5 --steps 200 --warmup 40 > gpurun_out/r06b/single.txt 2>&1 || { tail -5 gpurun_out/r06b/single.txt; exit 1; }
cat gpurun_out/r06b/single.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06b/tr -o run --output-format csv -- python3 tools/single_probe.py c5 --steps 30 --warmup 5 > gpurun_out/r06b/tr.log 2>&1 || { tail -5 gpurun_out/r06b/tr.log; exit 1; }
echo done
