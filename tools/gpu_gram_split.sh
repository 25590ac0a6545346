# Gram column-split threshold A/B: kernel-trace totals of the bench at R>=64 (default) vs
# always split below 512 replicates.  usage: bash tools/gpu_gram_split.sh <outdir>
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gram" > $out/pytest.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof64 -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof64.log 2>&1
CNMF_GRAM_SPLIT_MIN_R=512 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $out/prof512 -o run -- python3 bench.py --steps 10 --warmup 3 > $out/prof512.log 2>&1
timeout -k 10 120 python bench.py > $out/bench64.log 2>&1
CNMF_GRAM_SPLIT_MIN_R=512 timeout -k 10 120 python bench.py > $out/bench512.log 2>&1
