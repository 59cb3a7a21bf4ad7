#!/bin/bash
# Pipelined-bench A/B on one GPU: pipeline tests, then bench.py --pipeline 0/1
# alternated at each size (ms per step, leaf-kernel hipEvent ms, root, pipelined).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pipe
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "pipeline or split_shard or finish_nodes or frontier" -x -q --timeout 200 --timeout-method thread > gpurun_out/pipe/pytest.log 2>&1 || { tail -30 gpurun_out/pipe/pytest.log; exit 1; }
tail -2 gpurun_out/pipe/pytest.log
for n in ${PIPE_SIZES:-28 25}; do
  for p in ${PIPE_MODES:-0 1 0 1}; do
    timeout -k 10 200 python bench.py --log2n $n --pipeline $p --no-cpu-baseline > gpurun_out/pipe/b_${n}_$p.json 2> gpurun_out/pipe/b_${n}_$p.err || { tail -5 gpurun_out/pipe/b_${n}_$p.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/pipe/b_${n}_$p.json').read().strip().splitlines()[-1]);print($n, $p, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['root'][:16], d['config']['pipelined'])" | tee -a gpurun_out/pipe/summary.txt
  done
done
