# float-input (non-count X) A/B on one box: default, no layout replay, unfused step, raw-slab cap 16, exact B planes; headline for calibration; kernel trace of the float run
set -e
export TMPDIR=/tmp
out=gpurun_out/r3ao
mkdir -p $out
timeout -k 10 120 python bench.py > $out/bench_head.log 2>&1
timeout -k 10 120 python bench.py --float-input > $out/float_def_1.log 2>&1
CNMF_LAYOUT_REPLAY=0 timeout -k 10 120 python bench.py --float-input > $out/float_noreplay.log 2>&1
CNMF_FUSED_STEP=0 timeout -k 10 120 python bench.py --float-input > $out/float_unfused.log 2>&1
CNMF_FUSED_MAX_SLABS=16 timeout -k 10 120 python bench.py --float-input > $out/float_slabs16.log 2>&1
CNMF_GEMM_BPLANES=3 timeout -k 10 120 python bench.py --float-input > $out/float_b3.log 2>&1
timeout -k 10 120 python bench.py --float-input > $out/float_def_2.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --float-input --steps 10 --warmup 3 > $out/prof.log 2>&1
echo done
