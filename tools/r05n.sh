export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_leaf.py --log2n 28 --rounds 9 main l16 l4_10_16 l6_12_18 l2_8_14 > gpurun_out/r05n_ab28.log 2>&1; rc=$?; grep -E "variant|median" gpurun_out/r05n_ab28.log | head; [ $rc -ne 0 ] && tail -5 gpurun_out/r05n_ab28.log && exit $rc
timeout -k 10 300 python -u tools/ab_leaf.py --log2n 25 --rounds 9 main l16 l4_10_16 l6_12_18 l2_8_14 > gpurun_out/r05n_ab25.log 2>&1; rc=$?; grep -E "variant|median" gpurun_out/r05n_ab25.log | head; exit $rc
