# Split-GEMM k-step depth A/B (BK 64 vs 32): GEMM tests, sweep, bench and K-grid bench.
# usage: bash tools/gpu_gemm_bk.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or nmf or planes" > $out/pytest.log 2>&1
CNMF_GEMM_BK=32 timeout -k 10 200 python tools/gemm_planes_bench.py > $out/sweep_bk32.log 2>&1
CNMF_GEMM_BK=64 timeout -k 10 200 python tools/gemm_planes_bench.py > $out/sweep_bk64.log 2>&1
CNMF_GEMM_BK=32 timeout -k 10 120 python bench.py > $out/bench_bk32.log 2>&1
timeout -k 10 120 python bench.py > $out/bench_bk64.log 2>&1
CNMF_GEMM_BK=32 timeout -k 10 120 python bench.py > $out/bench_bk32b.log 2>&1
timeout -k 10 120 python bench.py > $out/bench_bk64b.log 2>&1
CNMF_GEMM_BK=32 timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_bk32.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid_bk64.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1
