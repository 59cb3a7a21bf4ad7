# Round-6 validation on the current tree: the whole GPU suite under a kernel
# trace (kernel coverage) + smoke, the default bench line (every side config),
# the 8-rank one-GPU rehearsal.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06j
bash tools/gpu_run.sh r06j ktests || exit 1
timeout -k 10 500 python bench.py > gpurun_out/r06j/bench.json 2> gpurun_out/r06j/bench.err || { tail -5 gpurun_out/r06j/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r06j/bench.json')); print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], d['roofline'].get('step_frac_aggregate'), d['config']['root_matches_golden']); print({k: (round(v['ms_per_step'], 4), v.get('single_state_ms', v.get('single_trie_ms', v.get('device_resident_ms'))), v['root_matches_golden']) for k, v in d['side_configs'].items()})"
bash tools/gpu_run.sh r06j rehearse8 || exit 1
echo done
