export TMPDIR=/tmp; mkdir -p gpurun_out
side() { python3 -c "
import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], 'c4', round(d['ms_per_step'],3), ' '.join(f\"{k}={v['ms_per_step']:.4f}\" for k,v in d['side_configs'].items()))" $1 $2; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r05j_a.json 2>/dev/null && side gpurun_out/r05j_a.json nocpu
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --side-warmup 1000 > gpurun_out/r05j_b.json 2>/dev/null && side gpurun_out/r05j_b.json warm1000
timeout -k 10 300 python bench.py --config c3 --steps 200 --warmup 40 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3 alone', d['ms_per_step'])"
timeout -k 10 300 python bench.py --config c5 --steps 200 --warmup 40 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 alone', d['ms_per_step'])"
timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 40 --no-cpu-baseline 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c2 alone', d['ms_per_step'])"
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/prof_r05j -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof_r05j.log 2>&1; echo prof rc=$?
