# Round-5 final validation: every GPU test + smoke, the N = 1 step forms
# (one stream vs pipelined, two interleaved pairs), the default bench line,
# its rocprofv3 stats/PMC passes.
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_run.sh r05aa tests || exit 1
for i in 1 2; do for p in 1 0; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-side-configs --pipeline $p > gpurun_out/r05aa_$p.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/r05aa_$p.json')); print('pipeline', $p, round(d['ms_per_step'], 4), round(d['roofline']['avg_launch_ms'], 4), d['config']['root_matches_golden'])"
done; done
timeout -k 10 400 python bench.py > gpurun_out/bench_r05aa.json 2> gpurun_out/bench_r05aa.err || exit 1
python3 -c "import json; d=json.load(open('gpurun_out/bench_r05aa.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline']['step_frac_aggregate'], d['config']['root_matches_golden'], {k: (round(v['ms_per_step'], 4), v['root_matches_golden']) for k, v in d['side_configs'].items()})"
TAG=r05aa_c4 PROF_ARGS="--steps 20 --warmup 5 --no-cpu-baseline --no-side-configs" bash tools/profile.sh > gpurun_out/r05aa_prof.log 2>&1; echo prof rc=$?
