# 4-wave 64x128 GEMM tile A/B: GEMM tests, sweep, bench with CNMF_GEMM_SMALL=3 vs 4.
# usage: bash tools/gpu_gemm_small.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" > $out/pytest.log 2>&1
timeout -k 10 200 python tools/gemm_planes_bench.py > $out/sweep.log 2>&1
CNMF_GEMM_SMALL=3 timeout -k 10 120 python bench.py > $out/bench_s3.log 2>&1
CNMF_GEMM_SMALL=4 timeout -k 10 120 python bench.py > $out/bench_s4.log 2>&1
CNMF_GEMM_SMALL=3 timeout -k 10 120 python bench.py > $out/bench_s3b.log 2>&1
CNMF_GEMM_SMALL=4 timeout -k 10 120 python bench.py > $out/bench_s4b.log 2>&1
CNMF_GEMM_SMALL=4 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1
