export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/ab_leaf.py --trie --log2n 20 --rounds 9 main nl_l2 > gpurun_out/r05l_ab.log 2>&1; rc=$?; grep variant gpurun_out/r05l_ab.log; [ $rc -ne 0 ] && tail -5 gpurun_out/r05l_ab.log; exit $rc
