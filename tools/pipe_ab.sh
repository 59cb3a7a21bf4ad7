set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pipeline or finish_nodes or frontier" -x -q --timeout 200 --timeout-method thread > gpurun_out/pipe/pytest.log 2>&1 || { tail -30 gpurun_out/pipe/pytest.log; exit 1; }
tail -2 gpurun_out/pipe/pytest.log
for p in 0 1 0 1; do
  timeout -k 10 200 python bench.py --pipeline $p --no-cpu-baseline > gpurun_out/pipe/b_$p.json 2> gpurun_out/pipe/b_$p.err || { tail -5 gpurun_out/pipe/b_$p.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/pipe/b_$p.json').read().strip().splitlines()[-1]);print($p, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['root'][:16], d['config']['pipelined'])" | tee -a gpurun_out/pipe/summary.txt
done
