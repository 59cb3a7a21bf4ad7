#!/bin/bash
# The one parameterised GPU-box runner (it replaces round 2's one-off
# tools/r02*.sh scripts, which git history keeps).  Every step has its own
# time limit; the first failing step ends the run (no GPU work after a fault,
# an abort or a timeout).  Outputs under gpurun_out/<TAG>/.
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]
#
#   tests                   pytest -m gpu (every GPU test) + __graft_entry__.smoke()
#   ktests                  the same under rocprofv3 --kernel-trace --stats, then
#                           tools/kernel_coverage.py: kernels compiled but never launched
#   pytest:PATH             one test file / node id
#   bench:CFG               bench.py --config CFG (c1 c2 c3 c4 c4tree c5), JSON line kept
#                           (c1/c2/c3/c5: --steps 100 --warmup 20)
#   profile:CFG:KERNEL      rocprofv3 kernel-trace stats + separate PMC passes of CFG's
#                           bench line (tools/profile.sh); KERNEL = substring of the
#                           dominant kernel's name for the summary (empty: C4's leaf kernel)
#   ab:ARGS:VARIANTS        tools/ab_leaf.py one-process A/B; ARGS and VARIANTS use '+'
#                           for spaces (e.g. ab:--trie+--log2n+20:main+rec2)
#   rankstep:LOG2N:WORLD    tools/rank_step_probe.py (one rank's pipelined step, 3 sets)
#   rehearse8               tools/rehearse8.sh (8 gloo ranks sharing the GPU, golden root)
#   e2e:LOG2N:MODE          tools/e2e_host.py (host-buffer call incl. PCIe; MODE "tree" or empty)
#   single:CFGS             tools/single_probe.py (C5 one trie, C3 one state, C1 device-resident;
#                           CFGS '+'-joined, e.g. c3+c5), 200 steps, then a kernel trace of 30
#   topprobe                tools/top_probe (built here with -DMK_TOP_STAMPS=1): per-level cycles
#                           of the fused trie top and of C3's fused list top
#   singleab:CFGS:VARIANTS  tools/single_probe.py CFGS ('+'-joined) against library variants
#                           (VARIANTS '+'-joined; main = the default build, else
#                           prysm_amd/lib/variants/libprysm_merkle_<v>.so), 3 interleaved rounds
#   pmcsingle:CFG:KERNEL    PMC passes (LDS/waits/VALU, FETCH_SIZE, TCC hit/miss) of the
#                           single_probe loop of CFG, summarised for the kernel name substring KERNEL
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p $O
for step in "$@"; do
  IFS=: read -r kind a b <<< "$step"
  name=$(echo "$step" | sed 's/--//g' | tr ':/+ <>,.' '_______')
  case $kind in
    tests)
      timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
      tail -1 $O/pytest_gpu.log
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    ktests)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/ktests -o run --output-format csv -- \
        python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
      tail -1 $O/pytest_gpu.log
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log
      python3 tools/kernel_coverage.py $O/ktests > $O/kernel_coverage.json; tail -12 $O/kernel_coverage.json ;;
    pytest)
      timeout -k 10 600 python -u -m pytest "$a" -x -v --timeout 200 --timeout-method thread \
        > $O/$name.log 2>&1 || { tail -30 $O/$name.log; exit 1; }
      tail -1 $O/$name.log ;;
    bench)
      # sub-millisecond side configs: 100 timed steps, so the window (not the
      # clock ramp after the idle sync, nor a pipeline's drain) sets the figure
      case $a in c4|c4tree) K="";; *) K="--steps 100 --warmup 20";; esac
      timeout -k 10 400 python bench.py --config $a $K > $O/bench_$a.json 2> $O/bench_$a.err || { tail -5 $O/bench_$a.err; exit 1; }
      cat $O/bench_$a.json ;;
    profile)
      export KERNEL="${b:-k_leaf_lock_sc}"  # empty: the C4 leaf kernel
      TAG=${TAG}_$a PROF_ARGS="--config $a --steps 10 --warmup 20 --no-cpu-baseline" \
        bash tools/profile.sh > $O/profile_$a.log 2>&1 || { tail -8 $O/profile_$a.log; exit 1; }
      cp gpurun_out/prof_${TAG}_$a/summary.json $O/pmc_$a.json && echo "profile $a ok" ;;
    ab)
      timeout -k 10 400 python tools/ab_leaf.py ${a//+/ } --rounds 9 ${b//+/ } > $O/$name.log 2>&1 || { tail -8 $O/$name.log; exit 1; }
      grep variant $O/$name.log | cut -c1-160 ;;
    rankstep)
      timeout -k 10 240 python tools/rank_step_probe.py --log2n $a --world $b --slots 3 > $O/rankstep_${a}_$b.txt 2>&1 \
        || { tail -5 $O/rankstep_${a}_$b.txt; exit 1; }
      tail -1 $O/rankstep_${a}_$b.txt ;;
    rehearse8)
      bash tools/rehearse8.sh > $O/rehearse8.log 2>&1 || { tail -20 $O/rehearse8.log; exit 1; }
      cp gpurun_out/rehearse8_summary.json $O/ && echo "rehearse8 ok" ;;
    e2e)
      timeout -k 10 300 python tools/e2e_host.py $a $b > $O/e2e_${a}_$b.json 2> $O/e2e_${a}_$b.err \
        || { tail -5 $O/e2e_${a}_$b.err; exit 1; }
      cat $O/e2e_${a}_$b.json ;;
    single)
      timeout -k 10 300 python tools/single_probe.py ${a//+/ } --steps 200 --warmup 40 > $O/single_$name.txt 2>&1 \
        || { tail -5 $O/single_$name.txt; exit 1; }
      grep config $O/single_$name.txt
      timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr_$name -o run --output-format csv -- \
        python3 tools/single_probe.py ${a//+/ } --steps 30 --warmup 5 > $O/tr_$name.log 2>&1 || { tail -5 $O/tr_$name.log; exit 1; } ;;
    topprobe)
      (cd tools && hipcc --offload-arch=gfx950 -O3 -std=c++17 -DMK_TOP_STAMPS=1 -I../prysm_amd/csrc -I../include \
        top_probe.hip -o /tmp/top_probe) > $O/topprobe_build.log 2>&1 || { tail -5 $O/topprobe_build.log; exit 1; }
      timeout -k 5 60 /tmp/top_probe 5 > $O/top_probe_trie.json && timeout -k 5 60 /tmp/top_probe 5 merkle > $O/top_probe_merkle.json \
        || exit 1
      cat $O/top_probe_merkle.json ;;
    singleab)
      for r in 1 2 3; do
        for v in ${b//+/ }; do
          if [ "$v" = main ]; then L=prysm_amd/lib/libprysm_merkle.so; else L=prysm_amd/lib/variants/libprysm_merkle_$v.so; fi
          PRYSM_MERKLE_LIB=$L timeout -k 10 200 python tools/single_probe.py ${a//+/ } --steps 200 --warmup 40 \
            > $O/ab_${v}_$r.txt 2>&1 || { tail -5 $O/ab_${v}_$r.txt; exit 1; }
          sed "s/^/$v /" $O/ab_${v}_$r.txt | tee -a $O/singleab.txt
        done
      done ;;
    pmcsingle)
      D=$O/pmc_$a
      for pass in "lds:SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE" \
                  "fetch:FETCH_SIZE" "sq:TCC_HIT_sum TCC_MISS_sum"; do
        timeout -s KILL 120 rocprofv3 --pmc ${pass#*:} -d $D/${pass%%:*} -o run --output-format csv -- \
          python3 tools/single_probe.py $a --steps 20 --warmup 5 >> $D.log 2>&1 || { tail -5 $D.log; exit 1; }
      done
      KERNEL=$b python3 tools/pmc_summary.py $D > $O/pmc_$a.json && echo "pmc $a ok" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "done $TAG"
