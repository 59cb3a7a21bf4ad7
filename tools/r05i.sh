export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_leaf.py --trie --log2n 20 --rounds 7 main prio1 prio3 dma6 dma18 bars1 unroll1 unroll4 > gpurun_out/r05i_ab.log 2>&1; rc=$?; grep variant gpurun_out/r05i_ab.log; [ $rc -ne 0 ] && tail -5 gpurun_out/r05i_ab.log && exit $rc
bash tools/r05h.sh
