# 8-wave 128x128 GEMM tile (variant 5): GEMM tests + sweep.
# usage: bash tools/gpu_gemm_v5.sh <outdir under gpurun_out>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" > $out/pytest.log 2>&1
timeout -k 10 200 python tools/gemm_planes_bench.py > $out/sweep.log 2>&1
