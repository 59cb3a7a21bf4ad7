# Extra random-shape parity on the final tree: the GPU fuzz with 6 more seed
# streams at 2x scale (each a fresh set of shapes), one process per seed.
export TMPDIR=/tmp; mkdir -p gpurun_out
for sd in 11 12 13 14 15 16; do
  PRYSM_FUZZ_SEED=$sd PRYSM_FUZZ_SCALE=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_fuzz.py -x -q --timeout 280 --timeout-method thread > gpurun_out/r05ac_fuzz_$sd.log 2>&1 || { tail -20 gpurun_out/r05ac_fuzz_$sd.log; exit 1; }
  echo "seed $sd: $(tail -1 gpurun_out/r05ac_fuzz_$sd.log)"
done
