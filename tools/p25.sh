set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python bench.py --log2n 25 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/b25.json 2>gpurun_out/b25.err || exit $?
cat gpurun_out/b25.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/p25 -o run --output-format csv -- python3 bench.py --log2n 25 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/p25.log 2>&1 || exit $?
find gpurun_out/p25 -name "*stats*" | xargs cat
