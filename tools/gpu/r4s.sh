# KL PMC at HEAD: CSR path at 8 % density and the dense path (headline density)
export TMPDIR=/tmp
out=gpurun_out/r4s
mkdir -p $out
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d $out/kl08_1 -o run --output-format csv -- python3 bench.py --beta-loss kullback-leibler --density 0.08 --steps 1 --warmup 0 --n-iter 20 > $out/kl08_1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/kl08_2 -o run --output-format csv -- python3 bench.py --beta-loss kullback-leibler --density 0.08 --steps 1 --warmup 0 --n-iter 20 > $out/kl08_2.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES -d $out/kldense_1 -o run --output-format csv -- python3 bench.py --beta-loss kullback-leibler --steps 1 --warmup 0 --n-iter 20 > $out/kldense_1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -d $out/kldense_2 -o run --output-format csv -- python3 bench.py --beta-loss kullback-leibler --steps 1 --warmup 0 --n-iter 20 > $out/kldense_2.log 2>&1
echo rc=$?
