set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/dev.log 2>&1
timeout -k 10 500 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/pytest_gpu1.log 2>&1 && \
timeout -k 10 200 python __graft_entry__.py smoke > gpurun_out/smoke1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run -- python bench.py --steps 1 --warmup 0 > gpurun_out/prof1.log 2>&1
