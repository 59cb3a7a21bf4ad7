export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_state_pipeline.py tests/test_gpu_deposit_trie.py tests/test_gpu_trie_lock.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r05k_t.log 2>&1; rc=$?; tail -2 gpurun_out/r05k_t.log; [ $rc -ne 0 ] && exit $rc
side() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'c4', round(d['ms_per_step'],3), ' '.join(f\"{k}={v['ms_per_step']:.4f}\" for k,v in d['side_configs'].items()))" $1 $2; }
for i in 1 2; do timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05k_$i.json 2>/dev/null && side gpurun_out/r05k_$i.json run$i; done
timeout -k 10 300 python bench.py --config c3 --steps 200 --warmup 40 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 alone', d['ms_per_step'])"
