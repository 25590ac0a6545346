# solve probe + bench (+ solve/nmf tests)
set -e
export TMPDIR=/tmp
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "solve or nmf or coop" > $out/pytest.log 2>&1
timeout -k 10 200 python -u tools/solve_probe.py > $out/solve.log 2>&1
timeout -k 10 120 python bench.py > $out/bench.log 2>&1
timeout -k 10 120 python bench.py > $out/bench2.log 2>&1
