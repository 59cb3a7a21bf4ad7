export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_deposit_trie.py tests/test_gpu_trie_lock.py tests/test_gpu_full_size.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05m_t.log 2>&1; rc=$?; tail -2 gpurun_out/r05m_t.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --config c5 --steps 200 --warmup 40 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5', d['ms_per_step'], d['config']['single_trie_ms'], d['config']['root_matches_golden'])"; done
