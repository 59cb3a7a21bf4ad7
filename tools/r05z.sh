# After the persistent shard grid: the shard/pipeline GPU tests, one rank's
# step at 2/4/8 ranks, the N = 1 bench line (same box), the 8-rank rehearsal.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_full_size.py tests/test_gpu_node_lock.py tests/test_gpu_bench_line.py tests/test_gpu_nccl.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05z_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/r05z_pytest.log; [ $rc -ne 0 ] && exit $rc
for s in "27 2" "26 4" "25 8"; do set -- $s
  timeout -k 10 120 python tools/rank_step_probe.py --log2n $1 --world $2 --slots 3 2>/dev/null | tail -1 || exit 1
done
timeout -k 10 400 python bench.py > gpurun_out/bench_r05z.json 2> gpurun_out/bench_r05z.err || { tail -5 gpurun_out/bench_r05z.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_r05z.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['step_frac_aggregate'], d['config']['root_matches_golden'], {k: (v['ms_per_step'], v['root_matches_golden']) for k, v in d['side_configs'].items()})"
bash tools/rehearse8.sh
