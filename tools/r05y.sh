# Shard leaf pass: one group per workgroup (main) vs the persistent grid
# (variant persist), one rank's pipelined step at 2^25 / 8 ranks and 2^26 / 4,
# interleaved separate processes.
export TMPDIR=/tmp; mkdir -p gpurun_out
for i in 1 2 3; do for v in main persist; do for s in "25 8" "26 4"; do set -- $s
  if [ $v = main ]; then L=prysm_amd/lib/libprysm_merkle.so; else L=prysm_amd/lib/variants/libprysm_merkle_$v.so; fi
  PRYSM_MERKLE_LIB=$L timeout -k 10 120 python tools/rank_step_probe.py --log2n $1 --world $2 --slots 3 2>/dev/null | tail -1 | sed "s/^/$v /" || exit 1
done; done; done
