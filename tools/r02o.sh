#!/bin/bash
# r02o: C3 as a stream of states (tools/c3_stream_probe.py), 2/3/4 buffer
# sets, main library and occupancy/workgroup-size variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02o
mkdir -p $O
V=prysm_amd/lib/variants
for lib in main ${VARIANTS:-cap256 s5 s5cap}; do
  if [ $lib = main ]; then L=""; else L=$V/libprysm_merkle_$lib.so; fi
  PRYSM_MERKLE_LIB=$L timeout -k 10 200 python tools/c3_stream_probe.py >> $O/c3_stream.jsonl 2>> $O/c3_stream.err || { tail -5 $O/c3_stream.err; exit 1; }
done
cat $O/c3_stream.jsonl
