# struct staging xor rotation: LDS probe, struct tests, C3 one state, the
# struct kernel's LDS PMC; the C5 front's L2 hit rate (one trie loop).
export TMPDIR=/tmp; mkdir -p gpurun_out/r06g
(cd /tmp && timeout -s KILL 60 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d $GRAFT_REPO_ROOT/gpurun_out/r06g/ldsprobe -o run --output-format csv -- $GRAFT_REPO_ROOT/tools/lds_bank_probe) > gpurun_out/r06g/ldsprobe.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_lock.py tests/test_gpu_state.py tests/test_gpu_state_pipeline.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06g/pytest.log 2>&1 || { tail -30 gpurun_out/r06g/pytest.log; exit 1; }
tail -1 gpurun_out/r06g/pytest.log
timeout -k 10 200 python tools/single_probe.py c3 --steps 200 --warmup 40 2>/dev/null || exit 1
D=gpurun_out/r06g/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $D/lds -o run --output-format csv -- python3 tools/single_probe.py c3 --steps 20 --warmup 5 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
KERNEL=k_struct_lock python3 tools/pmc_summary.py $D > gpurun_out/r06g/pmc_summary.json && python3 -c "
import json; d=json.load(open('gpurun_out/r06g/pmc_summary.json')); print(json.dumps(d['leaf_counters_per_dispatch']))"
D=gpurun_out/r06g/pmc5
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d $D/sq -o run --output-format csv -- python3 tools/single_probe.py c5 --steps 20 --warmup 5 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- python3 tools/single_probe.py c5 --steps 20 --warmup 5 >> $D.log 2>&1 || { tail -5 $D.log; exit 1; }
KERNEL=k_trie_rec_lock python3 tools/pmc_summary.py $D > gpurun_out/r06g/pmc5_summary.json && python3 -c "
import json; d=json.load(open('gpurun_out/r06g/pmc5_summary.json')); print(json.dumps(d['leaf_counters_per_dispatch']))"
echo done
