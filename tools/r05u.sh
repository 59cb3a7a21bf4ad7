# N = 1 step form A/B on a second box: pipelined (--pipeline 1) vs one stream
# (--pipeline 0, the default), three interleaved pairs of 30 timed steps.
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do for p in 1 0; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-side-configs --pipeline $p > gpurun_out/r05u_$p.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/r05u_$p.json')); print('pipeline', $p, round(d['ms_per_step'], 4), round(d['roofline']['avg_launch_ms'], 4), round(d['config']['single_tree_ms'], 4), d['config']['root_matches_golden'])"
done; done
