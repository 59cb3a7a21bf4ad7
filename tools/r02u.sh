#!/bin/bash
# r02u: host-buffer merkleHash through the overlapped one-device sharded path
# -- GPU tests, then 8 GiB end to end with and without it (alternating)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for lib in main noovl; do
    if [ $lib = main ]; then L=""; else L=prysm_amd/lib/variants/libprysm_merkle_$lib.so; fi
    PRYSM_MERKLE_LIB=$L timeout -k 10 300 python tools/e2e_host.py 28 > $O/e2e_${lib}_${rep}.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('$O/e2e_${lib}_${rep}.json')); print('$lib', round(d['pageable_ms'],1), round(d['pinned_ms'],1), round(d['device_resident_ms'],2), d['pageable_root'][:16], d['pinned_root']==d['device_root'])" | tee -a $O/e2e_ab.txt
  done
done
