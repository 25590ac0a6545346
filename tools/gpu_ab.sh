# Bench A/B on one box: default, CNMF_GRAPHS=1, 2-stage GEMMs everywhere; repeated default.
# usage: bash tools/gpu_ab.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or graph" > $out/pytest.log 2>&1
timeout -k 10 120 python bench.py > $out/bench_a.log 2>&1
CNMF_GRAPHS=1 timeout -k 10 120 python bench.py > $out/bench_graphs.log 2>&1
CNMF_GEMM_STAGES=2 timeout -k 10 120 python bench.py > $out/bench_s2.log 2>&1
timeout -k 10 120 python bench.py > $out/bench_b.log 2>&1
timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/bench_grid.log 2>&1
CNMF_GEMM_STAGES=2 timeout -k 10 120 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/bench_grid_s2.log 2>&1
