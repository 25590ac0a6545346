#!/bin/bash
# One GPU round: kernel tests, smoke, bench, and a kernel-trace profile of the bench.
# usage (via gpurun): bash tools/gpu_check.sh <tag>
set -o pipefail
TAG=${1:-run}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/bench_$TAG.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --steps 1 --warmup 0 > gpurun_out/prof_$TAG.log 2>&1
