# Split-GEMM LDS pipeline depth A/B: GEMM tests, GEMM sweep and bench.py at 2 vs 3 stages.
# usage: bash tools/gpu_gemm_stages.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or nmf" > $out/pytest.log 2>&1
CNMF_GEMM_STAGES=2 timeout -k 10 200 python tools/gemm_planes_bench.py > $out/sweep_s2.log 2>&1
CNMF_GEMM_STAGES=3 timeout -k 10 200 python tools/gemm_planes_bench.py > $out/sweep_s3.log 2>&1
CNMF_GEMM_STAGES=2 timeout -k 10 120 python bench.py > $out/bench_s2.log 2>&1
CNMF_GEMM_STAGES=3 timeout -k 10 120 python bench.py > $out/bench_s3.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof.log 2>&1
