# active flags written by conv_update into pinned host memory: tests + A/B
export TMPDIR=/tmp
out=gpurun_out/r4v
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_solve_pipe_gpu.py tests/test_pipeline_gpu.py -x -q --timeout 170 --timeout-method thread > $out/pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 $out/pytest.log; exit 1; }
for r in 1 2; do
  for h in 1 0; do
    CNMF_HOST_FLAGS=$h timeout -k 10 120 python bench.py > $out/bench_h${h}_$r.log 2>&1 || exit 1
  done
done &&
CNMF_HOST_FLAGS=1 timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_h1.log 2>&1 &&
CNMF_HOST_FLAGS=0 timeout -k 10 120 python bench.py --k 20 --steps 5 --warmup 2 > $out/k20_h0.log 2>&1 &&
timeout -k 10 200 python bench.py --kmin 5 --kmax 13 --steps 5 --warmup 2 > $out/grid.log 2>&1
echo rc=$?
