#!/bin/bash
# The exact 8-GPU C4 decomposition (2^28 items, 8 ranks of 2^25, frontier 10,
# pipelined) run as 8 gloo ranks sharing cuda:0; the root must equal the
# 1-GPU root.  Timing is meaningless (eight ranks share one GPU).
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 8 --backend gloo --share-device --log2n 28 --steps 2 --warmup 1 \
  --no-cpu-baseline > gpurun_out/rehearse8.json 2> gpurun_out/rehearse8.err || { tail -20 gpurun_out/rehearse8.err; exit 1; }
grep '^{' gpurun_out/rehearse8.json | tail -1 | python -c "
import json, sys
d = json.loads(sys.stdin.read())
c = d['config']
r = d['roofline']
print(json.dumps({'ranks_on_one_gpu': d['n_gpus'], 'n_items': c['n_items'], 'shard_height': c['shard_height'],
                  'frontier_log2': c['frontier_log2'], 'pipelined': c.get('pipelined'), 'root': c['root'],
                  'single_gpu_ms': c.get('single_gpu_ms'), 'parallel_efficiency': c.get('parallel_efficiency'),
                  'per_rank_leaf_frac': c.get('per_rank_leaf_frac'), 'step_frac_aggregate': r.get('step_frac_aggregate'),
                  'traffic': r.get('traffic'), 'traffic_source': r.get('traffic_source')}))
assert c['root'] == '54a62269279a90e4bda5a9da4b5bb0d5f3126bb3aacb1456cc0b0e47b9f50ba9', c['root']
assert c.get('pipelined') is True
assert c['single_gpu_ms'] and c['parallel_efficiency'] and len(c['per_rank_leaf_frac']) == 8
" | tee gpurun_out/rehearse8_summary.json
