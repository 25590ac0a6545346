#!/bin/bash
# GPU check of the preprocessing kernels (kmeans.hip, sparse.hip) + the Harmony e2e bench
# under cProfile.  usage (via gpurun): bash tools/hm_check.sh <tag>
set -o pipefail
TAG=${1:-hm}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_sparse_ops.py tests/test_preprocess.py -x -q -m gpu -k "kmeans or harmony or sparse or device or spmm" --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 && \
timeout -k 10 500 python -m cProfile -o gpurun_out/$TAG.prof tools/bench_harmony.py > gpurun_out/$TAG.log 2>&1 && \
python -c "import pstats; pstats.Stats('gpurun_out/$TAG.prof').sort_stats('tottime').print_stats(45)" > gpurun_out/${TAG}_top.txt && \
python -c "import pstats; pstats.Stats('gpurun_out/$TAG.prof').sort_stats('cumtime').print_stats(60)" > gpurun_out/${TAG}_cum.txt
