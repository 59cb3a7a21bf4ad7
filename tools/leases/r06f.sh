# 512-thread fused list top: parity, C3 one state; PMC of the struct kernel
# (bank conflicts after the rotated staging) from the single-state loop.
export TMPDIR=/tmp; mkdir -p gpurun_out/r06f
timeout -k 10 400 python -u -m pytest tests/test_gpu_merkle_top_fused.py tests/test_gpu_lock.py::test_state_hasher_schedules_agree tests/test_gpu_state.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06f/pytest.log 2>&1 || { tail -30 gpurun_out/r06f/pytest.log; exit 1; }
tail -2 gpurun_out/r06f/pytest.log
for s in fused level1 fused; do
PRYSM_C3_SCHED=$s timeout -k 10 200 python tools/single_probe.py c3 --steps 200 --warmup 40 2>/dev/null | sed "s/^/$s /" || exit 1
done
D=gpurun_out/r06f/pmc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE -d $D/lds -o run --output-format csv -- python3 tools/single_probe.py c3 --steps 20 --warmup 5 > $D.log 2>&1 || { tail -5 $D.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $D/fetch -o run --output-format csv -- python3 tools/single_probe.py c3 --steps 20 --warmup 5 >> $D.log 2>&1 || { tail -5 $D.log; exit 1; }
KERNEL=k_struct_lock ALL=1 python3 tools/pmc_summary.py $D > gpurun_out/r06f/pmc_summary.json && python3 -c "
import json; d=json.load(open('gpurun_out/r06f/pmc_summary.json')); print(json.dumps(d['leaf_counters_per_dispatch']))"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/r06f/tr -o run --output-format csv -- python3 tools/single_probe.py c3 --steps 30 --warmup 5 > gpurun_out/r06f/tr.log 2>&1 || { tail -5 gpurun_out/r06f/tr.log; exit 1; }
echo done
