export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2; do for p in 1 0; do timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side-configs --pipeline $p 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('pipeline', $p, d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['single_tree_ms'])"; done; done
bash tools/rehearse8.sh
