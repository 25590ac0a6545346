# LDS-staged partial Grams in the pipelined solve
export TMPDIR=/tmp
out=gpurun_out/r4m
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_solve_pipe_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
timeout -k 10 120 python bench.py > $out/bench.log 2>&1 &&
timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20.log 2>&1 &&
timeout -k 10 120 python bench.py --k 30 --steps 5 --warmup 2 > $out/k30.log 2>&1 &&
timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid.log 2>&1 &&
timeout -k 10 120 python bench.py > $out/bench2.log 2>&1
echo rc=$?
