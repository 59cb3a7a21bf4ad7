# C1 host path: H2D chunk floor 65536 (main) vs 4096 / 2048 records, one-process A/B.
export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 200 python tools/ab_leaf.py --host-struct 16384 --rounds 300 main h2d4096 h2d2048 2>/dev/null || exit 1
timeout -k 10 200 python tools/ab_leaf.py --host-struct 131072 --rounds 100 main h2d4096 h2d2048 2>/dev/null || exit 1
