#!/bin/bash
# r02x: work-queue leaf pass (lq) and the reduce_tile refactor (main) against
# the pre-refactor library (old): parity first, then one-process A/Bs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r02x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
PRYSM_MERKLE_LIB=prysm_amd/lib/variants/libprysm_merkle_lq.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_size.py -x -q --timeout 200 --timeout-method thread > $O/pytest_lq.log 2>&1; rc=$?
tail -2 $O/pytest_lq.log; [ $rc -ne 0 ] && exit $rc
for n in 25 26 28; do
  timeout -k 10 300 python tools/ab_leaf.py --log2n $n --rounds 9 old main lq > $O/ab_$n.json 2>&1 || { cat $O/ab_$n.json; exit 1; }
  grep variant $O/ab_$n.json
done
