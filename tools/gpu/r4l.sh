# K=5..13 grid A/B: XCD map and slice width
export TMPDIR=/tmp
out=gpurun_out/r4l
mkdir -p $out
timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_def.log 2>&1 &&
CNMF_PIPE_MAP=0 timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_map0.log 2>&1 &&
CNMF_PIPE_SLICE_COLS=256 timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_c256.log 2>&1 &&
CNMF_PIPE_MAP=0 CNMF_PIPE_SLICE_COLS=256 timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_map0_c256.log 2>&1 &&
timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_def2.log 2>&1 &&
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
CNMF_PIPE_MAP=0 CNMF_PIPE_SLICE_COLS=256 timeout -k 10 120 python bench.py > $out/bench_map0_c256.log 2>&1
echo rc=$?
