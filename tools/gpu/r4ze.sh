# hardware counters of the headline and K=20 steps at HEAD
export TMPDIR=/tmp
out=gpurun_out/r4ze
mkdir -p $out
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d $out/k10_1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 > $out/k10_1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/k10_2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 > $out/k10_2.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/k20_2 -o run --output-format csv -- python3 bench.py --k 20 --steps 1 --warmup 0 > $out/k20_2.log 2>&1
echo rc=$?
