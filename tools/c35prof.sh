set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c35
for c in c3 c5; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c35/$c -o run --output-format csv -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c35/$c.log 2>&1 || exit 1
done
echo ok
