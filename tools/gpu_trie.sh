cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -q -x -k "trie or verify or merkle_root" > gpurun_out/pytest_trie.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_trie.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c5.json 2>gpurun_out/bench_c5.err; cat gpurun_out/bench_c5.json
