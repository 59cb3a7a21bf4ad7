# Round 6 first lease: the GPU suite on the struct-kernel slot fix, then the
# single-call latency forms (C5 one trie, C3 one state, C1) timed and traced,
# and the lone-wave permutation latency probe.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06a
bash tools/gpu_run.sh r06a tests || exit 1
timeout -k 10 200 python tools/single_probe.py c5 c3 c1 --steps 200 --warmup 40 > gpurun_out/r06a/single.txt 2>&1 || { tail -5 gpurun_out/r06a/single.txt; exit 1; }
cat gpurun_out/r06a/single.txt
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06a/tr -o run --output-format csv -- python3 tools/single_probe.py c5 c3 c1 --steps 30 --warmup 5 > gpurun_out/r06a/tr.log 2>&1 || { tail -5 gpurun_out/r06a/tr.log; exit 1; }
(cd /tmp && hipcc --offload-arch=gfx950 -O3 -std=c++17 -I$GRAFT_REPO_ROOT/prysm_amd/csrc $GRAFT_REPO_ROOT/tools/lat_probe.hip -o lat_probe) && timeout -k 10 60 /tmp/lat_probe 200 > gpurun_out/r06a/lat_probe.json; cat gpurun_out/r06a/lat_probe.json
