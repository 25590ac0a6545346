# KL bench after the compaction-rule split, plus the beta GPU tests.
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "beta or online" > $out/pytest.log 2>&1
timeout -k 10 200 python bench.py --beta-loss kullback-leibler --steps 3 --warmup 1 > $out/bench_kl.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
