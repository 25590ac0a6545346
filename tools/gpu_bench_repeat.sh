# GEMM + NMF kernel tests, then the headline bench 3x and the K-grid bench (same box), and
# a kernel-trace profile.  usage: bash tools/gpu_bench_repeat.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or nmf or planes" > $out/pytest.log 2>&1
timeout -k 10 120 python bench.py > $out/bench1.log 2>&1
timeout -k 10 120 python bench.py > $out/bench2.log 2>&1
timeout -k 10 120 python bench.py > $out/bench3.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1
