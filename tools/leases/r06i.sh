# Whole GPU suite + smoke on the current tree, the single forms and the top
# probe (both kernels), traces of the single forms.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06i
bash tools/gpu_run.sh r06i tests || exit 1
timeout -k 5 60 tools/top_probe 5 merkle || exit 1
timeout -k 5 60 tools/top_probe 5 > gpurun_out/r06i/top_probe_trie.json || exit 1
for c in c3 c5 c1; do timeout -k 10 200 python tools/single_probe.py $c --steps 200 --warmup 40 2>/dev/null || exit 1; done
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06i/tr -o run --output-format csv -- python3 tools/single_probe.py c3 c5 --steps 30 --warmup 5 > gpurun_out/r06i/tr.log 2>&1 || { tail -5 gpurun_out/r06i/tr.log; exit 1; }
echo done
