# device-side ragged batching (CNMF_DEV_SLOTS) tests + A/B; K=20 solve PMC
export TMPDIR=/tmp
out=gpurun_out/r4b
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_solve_pipe_gpu.py tests/test_kernels_gpu.py tests/test_pipeline_gpu.py tests/test_xgmi_gpu.py -k "pipe or fused or slots or live or gram_of or early or dense or rank_beyond or dp or predict or wide_k or exact or ridge" -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 $out/pytest.log; exit 1; }
timeout -k 10 200 python bench.py --mode dp --emulate-world 8 --steps 3 --warmup 1 > $out/emu8.log 2>&1 || { echo EMU_FAILED; tail -20 $out/emu8.log; }
for i in 1 2; do
CNMF_DEV_SLOTS=1 timeout -k 10 120 python bench.py > $out/bench_on_$i.log 2>&1 &&
CNMF_DEV_SLOTS=0 timeout -k 10 120 python bench.py > $out/bench_off_$i.log 2>&1 || exit 1
done
CNMF_DEV_SLOTS=1 timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_on.log 2>&1 &&
CNMF_DEV_SLOTS=0 timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_off.log 2>&1 &&
CNMF_DEV_SLOTS=1 timeout -k 10 200 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_on.log 2>&1 &&
CNMF_DEV_SLOTS=0 timeout -k 10 200 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_off.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace -d $out/dbprof -o run -- python3 bench.py --steps 4 --warmup 4 > $out/dbprof.log 2>&1 &&
(python tools/trace_passes.py $(ls $out/dbprof/*results.db $out/dbprof/*/*results.db 2>/dev/null | head -n 1) > $out/passes.log 2>&1; true) &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d $out/pmc1 -o run --output-format csv -- python3 bench.py --k 20 --steps 1 --warmup 0 > $out/pmc1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/pmc2 -o run --output-format csv -- python3 bench.py --k 20 --steps 1 --warmup 0 > $out/pmc2.log 2>&1
echo rc=$?
