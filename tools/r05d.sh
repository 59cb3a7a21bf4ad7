export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_trie_lock.py tests/test_gpu_deposit_trie.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05d_trie.log 2>&1; rc=$?; tail -4 gpurun_out/r05d_trie.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_leaf.py --trie --log2n 20 --rounds 9 r05head main > gpurun_out/r05d_ab.log 2>&1; rc=$?; cat gpurun_out/r05d_ab.log | grep variant; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -4 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05_c3 -o run --output-format csv -- python3 bench.py --config c3 --steps 100 --warmup 20 --no-cpu-baseline > gpurun_out/prof_r05_c3.log 2>&1; echo prof rc=$?
