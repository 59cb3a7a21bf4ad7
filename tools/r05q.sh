export TMPDIR=/tmp; mkdir -p gpurun_out
TAG=r05q_c5 KERNEL="k_trie_rec_lock<1024u, 4, true>" PROF_ARGS="--config c5 --steps 100 --warmup 20 --no-cpu-baseline" bash tools/profile.sh > gpurun_out/r05q_c5.log 2>&1; echo c5 rc=$?
TAG=r05q_c3 KERNEL="k_struct_lock<true>" PROF_ARGS="--config c3 --steps 100 --warmup 20 --no-cpu-baseline" bash tools/profile.sh > gpurun_out/r05q_c3.log 2>&1; echo c3 rc=$?
bash tools/gpu_run.sh r05q ktests
